// oap_kmeans_lloyd_t1 — the lean Lloyd-iteration kernel for MI355X (gfx950, CDNA4).
//
// One pass over the local rows per Lloyd iteration (the reference's hot loop
// is oneDAL's step1Local, mllib-dal/src/main/native/KMeansDALImpl.cpp:70-77): distances on the
// bf16 matrix cores, top-2 argmin in registers, exact fp32 per-row cost, fixed-point per-cluster
// sums in LDS.  Unlike the general fused kernel (kmeans_assign.hip) it evaluates ONE product per
// k-step only (tier 1) and never escalates a whole 32-row tile: a row whose top-2 gap is inside
// tier 1's rigorous error bound is appended to its workgroup's segment of a deferral list and
// left untouched; the general kernel then re-decides exactly those rows (row-list mode: the
// bf16x3 split, then exact fp32 where still unsure) and accumulates them.  So the answer is the
// general kernel's — assignments identical to an exact fp32 evaluation — while the hot pass keeps
// a fixed, branch-free instruction stream whatever the data's share of near ties.
//
// Design points (CDNA4):
// * A wave owns a 32-row tile: lane (r = l & 31, h = l >> 5) holds features 16s + 8h + j of row
//   r.  The centroid plane (bf16 hi part of -2c, plus bias features) is the MFMA A operand,
//   staged once per workgroup in LDS with an odd 16-byte-slot stride (conflict-free
//   ds_read_b128); rows are the B operand straight from registers.
// * Bias features carry both norms through the MFMA as hi/lo pairs: x' = [x, 1, 1, hi|x|^2,
//   lo|x|^2], c' = [-2c, hi|c|^2, lo|c|^2, 1, 1], so the 32x32 accumulator ends at |x - c|^2
//   with no seeding VALU and only the cross term carrying bf16 error.
// * Only the hi plane lives in LDS (the general kernel also keeps the lo plane): the fixed-point
//   fp64 accumulator fits beside it and the workgroup has 12-16 waves (3-4 per SIMD), so one
//   wave's VALU epilogue, another's MFMAs and a third's HBM loads overlap.
// * Tiles are dealt block-strided (block b: positions b, b + grid, ...), so a workgroup never
//   processes more rows than kmeans_rows_per_block_bound assumes (fixed-point exactness).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "kernels/kmeans_frag.h"
#include "kernels/kmeans_internal.h"

namespace oap {
namespace kern {

namespace {

using namespace kmdev;

// The kernel's own compact argument block (fewer SGPRs than KMeansAssignArgs).
struct LeanArgs {
  const void* x;
  const float* centers;
  const float* cnorm;
  const float* cstat;
  const float* scale;
  u64* sums;
  u64* counts;
  double* cost_slab;
  int32_t* labels;
  float* mindist;
  float2* bounds;
  float* xnorm;
  const int32_t* tile_list;
  const unsigned* tile_count;
  int32_t* defer_rows;
  unsigned* defer_row_count;
  u64* deferred_rows;
  int64_t n, seg_cap;
  int ld, d, k, kpad;
  int accumulate, sums_too, delta;
};

struct LeanSmem {
  size_t plane, sc, acc, cnt, wcost, dcnt, total;
};

__host__ __device__ inline LeanSmem lean_plan(int dp, int kpad, int k, int d, bool acc, bool sums,
                                              int waves) {
  LeanSmem m;
  size_t off = 0;
  m.plane = 0;
  off = round16(size_t(kpad) * stride_bf16(dp) * 2);
  m.sc = off;
  off = round16(off + size_t(dp) * 4);
  m.acc = off;
  if (acc && sums) off += size_t(k) * (d | 1) * 8;  // odd row stride: conflict-free ds_add_f64
  off = round16(off);
  m.cnt = off;
  if (acc) off += size_t(k) * 4;
  off = round16(off);
  m.wcost = off;
  off += size_t(waves) * 8;
  m.dcnt = off;
  off += 16;
  m.total = round16(off);
  return m;
}

template <int KS, bool XB, int WAVES, bool PF>
__global__ __launch_bounds__(WAVES * 64, 1) void oap_kmeans_lloyd_t1(LeanArgs a) {
  constexpr int DP = 16 * KS;
  constexpr int NT = WAVES * 64;
  using F = Frag<KS, XB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int kpad = a.kpad, k = a.k, d = a.d;
  const bool accumulate = a.accumulate != 0;
  const LeanSmem L = lean_plan(DP, kpad, k, d, accumulate, a.sums_too != 0, WAVES);
  const int sb = stride_bf16(DP);
  __bf16* ph = reinterpret_cast<__bf16*>(smem + L.plane);
  float* sc_l = reinterpret_cast<float*>(smem + L.sc);
  double* acc_l = reinterpret_cast<double*>(smem + L.acc);
  unsigned* cnt_l = reinterpret_cast<unsigned*>(smem + L.cnt);
  double* wcost = reinterpret_cast<double*>(smem + L.wcost);
  const int tid = threadIdx.x;

  // ---- stage the centroid plane c' = [-2c, hi|c|^2, lo|c|^2, 1, 1] (bf16) once per workgroup
  for (int idx = tid; idx < kpad * DP; idx += NT) {
    const int c = idx / DP, f = idx - c * DP;
    __bf16 v;
    if (f < d) {
      v = static_cast<__bf16>(-2.f * a.centers[idx]);  // exact scaling: hi(-2c) == -2 hi(c)
    } else if (f == d || f == d + 1) {
      __bf16 hi, lo;
      bf16_split((c < k) ? a.cnorm[c] : 1e30f, hi, lo);  // padded centers: huge, finite
      v = (f == d) ? hi : lo;
    } else {
      v = static_cast<__bf16>((f == d + 2 || f == d + 3) ? 1.f : 0.f);
    }
    ph[c * sb + f] = v;
  }
  for (int f = tid; f < DP; f += NT) sc_l[f] = (a.scale && a.sums_too && f < d) ? a.scale[f] : 0.f;
  if (accumulate) {
    if (a.sums_too)
      for (int i = tid; i < k * (d | 1); i += NT) acc_l[i] = 0.0;
    for (int i = tid; i < k; i += NT) cnt_l[i] = 0u;
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const float cmax = a.cstat[0];
  // tier-1 bound on two candidates' distance error: the cross term 2 x 2(2^-8 + 2^-18)|c||x|
  // (times |x| below), the bias pairs 2^-17 (|c|^2 + |x|^2) each, fp32 accumulation
  // 4e-5 (cmax^2 + |x|^2)
  const float thr_c = 0.0157f * cmax;
  const float thr_k = 6e-5f * cmax * cmax + 1e-30f;
  const float mrel = 4e-7f * float(d + 8);                // fp32 evaluation margin (bounds)
  const float ueps = 1.f + 1e-6f + 6e-8f * float(d + 4);  // direct-form |x - c|^2 rounding
  const int64_t ntiles_all = (a.n + 31) / 32;
  const bool listed = a.tile_list != nullptr;
  const int64_t npos = listed ? int64_t(*a.tile_count) : ntiles_all;
  const int64_t stride = int64_t(gridDim.x) * WAVES;
  int64_t t = int64_t(blockIdx.x) + int64_t(gridDim.x) * wave;
  // deferral: each wave owns a sub-segment of its workgroup's segment, filled in tile order, so
  // the list (and everything the re-decision pass sums over it) is deterministic
  const int64_t sub_cap = a.seg_cap / WAVES;
  int32_t* dseg = a.defer_rows + blockIdx.x * a.seg_cap + wave * sub_cap;
  unsigned n_def = 0;  // wave-uniform
  double my_cost = 0.0;
  const int jb = d - 16 * (KS - 1) - 8 * h;  // lane-local slot of bias feature d (may be < 0)

  auto tile_of = [&](int64_t q) -> int64_t {
    if (!listed) return q < ntiles_all ? q : ntiles_all - 1;
    if (npos == 0) return 0;  // (prefetch of an empty list: any real tile)
    const int64_t tl = int64_t(a.tile_list[q < npos ? q : npos - 1]);
    return tl < 0 ? 0 : (tl < ntiles_all ? tl : ntiles_all - 1);
  };
  auto load_tile = [&](int64_t tile, F& dst) {
    int64_t row = tile * 32 + r;
    row = row < a.n ? row : a.n - 1;
    if constexpr (XB) {
      const __bf16* p = static_cast<const __bf16*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f = 16 * s + 8 * h;
        dst.v[s] = (s < KS - 1 || f < a.ld) ? *reinterpret_cast<const bf16x8*>(p + 16 * s)
                                            : bf16x8{};
      }
    } else {
      const float* p = static_cast<const float*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int f = 16 * s + 8 * h + 4 * q;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (s < KS - 1 || f < a.ld) v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
          dst.v[s][4 * q + 0] = v.x;
          dst.v[s][4 * q + 1] = v.y;
          dst.v[s][4 * q + 2] = v.z;
          dst.v[s][4 * q + 3] = v.w;
        }
    }
  };

  // fixed-point accumulation of one row into cluster b (neg: subtract it)
  auto add_row = [&](const F& xv, int b, bool neg) {
    if (h == 0) atomicAdd(&cnt_l[b], neg ? 0xffffffffu : 1u);
    if (!a.sums_too) return;
    const float sgn = neg ? -1.f : 1.f;
    double* ap = acc_l + b * (d | 1) + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int f0 = 16 * s + 8 * h;
      const float4 s0 = *reinterpret_cast<const float4*>(sc_l + f0);
      const float4 s1 = *reinterpret_cast<const float4*>(sc_l + f0 + 4);
      const float scv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      if (s < KS - 1) {  // k-steps below KS-1 hold real features only (KS = ceil((d+4)/16))
#pragma unroll
        for (int j = 0; j < 8; ++j)
          atomicAdd(ap + 16 * s + j, sgn * static_cast<double>(rintf(xv.at(s, j) * scv[j])));
      } else {
        const int nv = d - f0;  // real features of this lane's half of the last k-step
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < nv)
            atomicAdd(ap + 16 * s + j, sgn * static_cast<double>(rintf(xv.at(s, j) * scv[j])));
      }
    }
  };

  auto process = [&](const int64_t pos, const F& x, F& xn, const int64_t pf) {
    const int64_t tile = tile_of(pos);
    const int64_t row = tile * 32 + r;
    const bool valid = pos < npos && row < a.n;
    if constexpr (PF) load_tile(tile_of(pf), xn);  // next tile: in flight under this one's work
    int old = -1;
    if (a.delta && valid) old = a.labels[row];
    float nx2 = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) nx2 = fmaf(x.at(s, j), x.at(s, j), nx2);
    nx2 += __shfl_xor(nx2, 32, 64);
    if (a.xnorm && pos < npos) {  // per-tile max |x|^2 (the delta scan's pruning margin)
      float tmax = nx2;
#pragma unroll
      for (int m = 16; m >= 1; m >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, m, 64));
      if (lane == 0) a.xnorm[tile] = tmax;
    }
    // MFMA B operand: the row's bf16 values with the bias slots [1, 1, hi|x|^2, lo|x|^2]
    bf16x8 xh[KS];
    {
      __bf16 nh, nl;
      bf16_split(nx2, nh, nl);
      const __bf16 one = static_cast<__bf16>(1.f);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 v;
        if constexpr (XB) {
          v = x.v[s];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = static_cast<__bf16>(x.v[s][j]);
        }
        if (s == KS - 1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            v[j] = (j == jb || j == jb + 1) ? one : v[j];
            v[j] = (j == jb + 2) ? nh : v[j];
            v[j] = (j == jb + 3) ? nl : v[j];
          }
        }
        xh[s] = v;
      }
    }
    // ---- tier 1: one bf16 product per k-step; top-2 on integer keys (the distance's bits with
    // the low 10 mantissa bits replaced by the in-chunk offset; value order, lowest index first)
    int k1 = 0x7fffffff, k2 = 0x7fffffff;
    auto mfma_chunk = [&](int c0, f32x16& acc) {
      const __bf16* ap = ph + size_t(c0 + r) * sb + 8 * h;
      bf16x8 av[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) av[s] = *reinterpret_cast<const bf16x8*>(ap + 16 * s);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], xh[0], f32x16{}, 0, 0, 0);
#pragma unroll
      for (int s = 1; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[s], xh[s], acc, 0, 0, 0);
    };
    auto epilogue = [&](int c0, const f32x16& acc) {
      int t1[4], t2[4];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int off = 8 * (e >> 2) + (e & 3);
        const int key = (__float_as_int(acc[e]) & ~0x3ff) | off;
        const int q = e & 3;
        if (e < 4) {
          t1[q] = key;
          t2[q] = 0x7fffffff;
        } else {
          t2[q] = med3_i32(t1[q], t2[q], key);  // 2nd smallest of {t1, t2, key}, t1 <= t2
          t1[q] = min(t1[q], key);
        }
      }
      auto merge2 = [](int& x1, int& x2, int y1, int y2) {
        x2 = min(max(x1, y1), min(x2, y2));
        x1 = min(x1, y1);
      };
      merge2(t1[0], t2[0], t1[1], t2[1]);
      merge2(t1[2], t2[2], t1[3], t2[3]);
      merge2(t1[0], t2[0], t1[2], t2[2]);
      const int base = c0 + 4 * h;  // disjoint from every in-chunk offset's bits
      const int i1 = t1[0] | base, i2 = t2[0] | base;
      k2 = min(max(k1, i1), min(k2, i2));
      k1 = min(k1, i1);
    };
    for (int c0 = 0; c0 < kpad; c0 += 32) {  // other waves' MFMAs overlap this epilogue
      f32x16 acc;
      mfma_chunk(c0, acc);
      epilogue(c0, acc);
    }
    {
      const int o1 = __shfl_xor(k1, 32, 64), o2 = __shfl_xor(k2, 32, 64);
      k2 = min(max(k1, o1), min(k2, o2));
      k1 = min(k1, o1);
    }
    const float b1 = __int_as_float(k1 & ~0x3ff), b2 = __int_as_float(k2 & ~0x3ff);
    const float tt = fmaf(thr_c, sqrtf(nx2), thr_k) + 2.5e-4f * fabsf(b2);  // + key truncation
    const bool unsure = valid && !(b2 - b1 > tt);
    // ---- defer unsure rows to the exact re-decision (one LDS atomic per wave with any)
    const unsigned long long um = __ballot(unsure && h == 0);
    if (um) {
      if (unsure && h == 0)
        dseg[n_def + __popcll(um & ((1ull << lane) - 1ull))] = static_cast<int32_t>(row);
      n_def += static_cast<unsigned>(__popcll(um));
    }
    const bool done = valid && !unsure;
    int b = k1 & 0x3ff;
    b = (b < k) ? b : 0;  // only for degenerate (NaN / all-inf) inputs
    float cb[KS][8];
    load_row8<KS>(a.centers + size_t(b) * DP + 8 * h, cb);  // L2-resident; lands under the adds
    if (done && accumulate) {
      if (!a.delta) {
        add_row(x, b, false);
      } else if (old >= 0 && old != b) {  // delta: only moved rows change the statistics
        add_row(x, b, false);
        add_row(x, min(old, k - 1), true);
      }
    }
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = x.at(s, j) - cb[s][j];
        part = fmaf(e, e, part);
      }
    const float rowcost = part + __shfl_xor(part, 32, 64);
    if (done && h == 0) {
      if (a.labels) a.labels[row] = b;
      if (a.mindist) a.mindist[row] = rowcost;
      if (a.bounds) {
        const float lo = b2 - (tt + mrel * (nx2 + cmax * cmax));
        a.bounds[row] = make_float2(sqrtf(rowcost) * ueps + 1e-30f, sqrtf(fmaxf(lo, 0.f)) * (1.f - 1e-6f));
      }
      my_cost += double(rowcost);
    }
  };

  if constexpr (PF) {
    F xa, xb;
    load_tile(tile_of(t), xa);
    for (; t < npos; t += 2 * stride) {  // t is wave-uniform: every branch stays uniform
      process(t, xa, xb, t + stride);
      if (t + stride >= npos) break;
      process(t + stride, xb, xa, t + 2 * stride);
    }
  } else {
    F xa;
    for (; t < npos; t += stride) {
      load_tile(tile_of(t), xa);
      process(t, xa, xa, 0);
    }
  }

  // ---- deterministic per-block cost (fixed shuffle tree, waves in index order), flushes
  const double wsum = wave_sum_f64(my_cost);
  if (lane == 0) {
    wcost[wave] = wsum;
    a.defer_row_count[blockIdx.x * kDeferSubs + wave] = n_def;
    if (a.deferred_rows && n_def) atomicAdd(a.deferred_rows, u64(n_def));
  }
  __syncthreads();
  if (tid == 0 && a.cost_slab) {
    double tot = 0.0;
    for (int w = 0; w < WAVES; ++w) tot += wcost[w];
    a.cost_slab[blockIdx.x] = tot;
  }
  if (accumulate) {
    for (int i = tid; a.sums_too && i < k * d; i += NT) {
      const int c = i / d, f = i - c * d;
      const double v = acc_l[c * (d | 1) + f];  // an exact integer, |v| < 2^53
      if (v != 0.0) atomicAdd(&a.sums[i], static_cast<u64>(static_cast<long long>(v)));
    }
    for (int i = tid; i < k; i += NT) {
      const int c = static_cast<int>(cnt_l[i]);  // signed: delta mode subtracts
      if (c) atomicAdd(&a.counts[i], static_cast<u64>(static_cast<long long>(c)));
    }
  }
}

template <int KS, bool XB, int WAVES, bool PF>
void launch_lean(const LeanArgs& a, int grid, hipStream_t s) {
  const LeanSmem L = lean_plan(16 * KS, a.kpad, a.k, a.d, a.accumulate, a.sums_too, WAVES);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&oap_kmeans_lloyd_t1<KS, XB, WAVES, PF>),
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_lloyd_t1<KS, XB, WAVES, PF>), dim3(grid), dim3(WAVES * 64),
                     L.total, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

template <int KS, bool XB>
void launch_lean_v(const LeanArgs& a, int grid, int variant, hipStream_t s) {
  switch (variant) {  // workgroup shape (one workgroup per CU: the LDS plan)
    case 1: launch_lean<KS, XB, 8, true>(a, grid, s); break;    // 2 waves/SIMD + prefetch
    case 2: launch_lean<KS, XB, 12, true>(a, grid, s); break;   // 3 waves/SIMD + prefetch
    case 3: launch_lean<KS, XB, 12, false>(a, grid, s); break;  // 3 waves/SIMD
    default: launch_lean<KS, XB, 16, false>(a, grid, s); break; // 4 waves/SIMD
  }
}

template <bool XB>
void launch_lean_xb(const LeanArgs& a, int grid, int variant, hipStream_t s) {
  switch ((a.d + 4 + 15) / 16) {
    case 1: launch_lean_v<1, XB>(a, grid, variant, s); break;
    case 2: launch_lean_v<2, XB>(a, grid, variant, s); break;
    case 3: launch_lean_v<3, XB>(a, grid, variant, s); break;
    case 4: launch_lean_v<4, XB>(a, grid, variant, s); break;
    case 5: launch_lean_v<5, XB>(a, grid, variant, s); break;
    case 6: launch_lean_v<6, XB>(a, grid, variant, s); break;
    case 7: launch_lean_v<7, XB>(a, grid, variant, s); break;
    case 8: launch_lean_v<8, XB>(a, grid, variant, s); break;
    default: OAP_THROW(ConfigError, "kmeans_lloyd: unsupported d=" << a.d);
  }
}

}  // namespace

bool kmeans_lloyd_supported(int d, int k, bool accumulate, bool sums_too) {
  if (d + 4 > 128) return false;
  const int dp = (d + 4 + 15) / 16 * 16;
  if (dp != kmeans_dp(d)) return false;  // the centroid buffer's row stride must match
  const int kpad = (k + 31) / 32 * 32;
  if (kpad > 1024) return false;  // keys carry a 10-bit index
  return lean_plan(dp, kpad, k, d, accumulate, sums_too, 16).total <= kLdsLimit;
}

int kmeans_lloyd_grid(int64_t n, int num_cus) {
  const int64_t tiles = (n + 31) / 32;
  const int64_t cap = num_cus > 256 ? num_cus : 256;
  return static_cast<int>(tiles < cap ? (tiles < 1 ? 1 : tiles) : cap);
}

int kmeans_lloyd_waves(int variant) {
  switch (variant) {
    case 1: return 8;
    case 2: case 3: return 12;
    default: return 16;
  }
}

int64_t kmeans_lloyd_seg_cap(int64_t n, int grid, int waves) {
  const int64_t tiles = (n + 31) / 32;
  const int64_t per_block = (tiles + grid - 1) / grid;  // positions of one workgroup
  return int64_t(waves) * ((per_block + waves - 1) / waves) * 32;
}

int kmeans_lloyd(const KMeansAssignArgs& a, int grid, int variant, hipStream_t s) {
  OAP_CHECK(kmeans_lloyd_supported(a.d, a.k, a.accumulate, a.sums_too) && !a.precise &&
                !a.merge && a.cstat && a.defer_rows && a.defer_row_count &&
                a.row_seg_cap == kmeans_lloyd_seg_cap(a.n, grid, kmeans_lloyd_waves(variant)) &&
                a.ld == kmeans_ld(a.d, a.xbf16),
            "kmeans_lloyd: unsupported arguments");
  OAP_CHECK(!a.delta || (a.labels && a.tile_list && a.tile_count),
            "kmeans_lloyd: delta mode needs labels and the scan's tile list");
  if (a.n == 0) return 0;
  LeanArgs l;
  l.x = a.x;
  l.centers = a.centers;
  l.cnorm = a.cnorm;
  l.cstat = a.cstat;
  l.scale = a.scale;
  l.sums = a.sums;
  l.counts = a.counts;
  l.cost_slab = a.cost_slab;
  l.labels = a.labels;
  l.mindist = a.mindist;
  l.bounds = reinterpret_cast<float2*>(a.bounds);
  l.xnorm = a.xnorm;
  l.tile_list = a.delta ? a.tile_list : nullptr;
  l.tile_count = a.delta ? a.tile_count : nullptr;
  l.defer_rows = a.defer_rows;
  l.defer_row_count = a.defer_row_count;
  l.deferred_rows = a.deferred_rows;
  l.n = a.n;
  l.seg_cap = a.row_seg_cap;
  l.ld = a.ld;
  l.d = a.d;
  l.k = a.k;
  l.kpad = a.kpad;
  l.accumulate = a.accumulate;
  l.sums_too = a.sums_too;
  l.delta = a.delta;
  if (a.xbf16)
    launch_lean_xb<true>(l, grid, variant, s);
  else
    launch_lean_xb<false>(l, grid, variant, s);
  return grid;
}

}  // namespace kern
}  // namespace oap
