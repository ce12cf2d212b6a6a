// oap_kmeans_lean_img — the steady-state Lloyd pass of the headline K-Means fit (gfx950, CDNA4).
//
// Every Lloyd iteration after the first of a delta-accumulating fit over f32 rows (SURVEY.md
// §2.6 K1; the reference's hot loop is oneDAL's step1Local, KMeansDALImpl.cpp:70-77) reads the
// resident fp16 operand image that the first pass wrote (kmeans_lloyd.hip, img_mode 1) instead of
// the rows: tier-1 distances on v_mfma_f32_32x32x16_f16, the top-2 per row in registers, rows
// inside the tier's rigorous error bound deferred to oap_kmeans_exact_rows, and only the rows
// whose label changed read their f32 values (fixed-point +x / -x).  It is the same arithmetic as
// oap_kmeans_lloyd_t1's image branch (labels, bounds, deferral lists and statistics are bitwise
// those of that kernel), but as its own kernel:
// * compile-time everything: no chunk keys, no cost, no timing switches, no f32-row operand
//   path — the branch-free instruction stream the general kernel could not give its image branch
//   (runtime switches, ~70 spilled SGPRs, and a join that waited vmcnt(0) on every tile: the
//   moved-row flush's row loads, younger than the next tile's image prefetch, merged into every
//   tile's wait state);
// * the moved-row flush runs at the top of a tile, before that tile's loads are issued, and
//   drains its own loads — so no tile ever waits for the prefetch it has just issued;
// * the chunk loop is software-pipelined (CFG bit 0): chunk c + 1's MFMA chain is issued before
//   chunk c's epilogue, into a second accumulator, so the matrix pipe works under the wave's
//   own VALU as well as under the other waves';
// * the last chunk folds only its real centroid groups (k = 200: 4 of 16 keys per lane);
// * labels are stored only for rows that moved (the others already hold theirs).
// When the plane at the image's scale is not representable (beta max|c| > 2^9) the kernel does
// nothing and oap_kmeans_lloyd_t1 (img_mode 3) runs the f32-row pass instead: both test the same
// device values, so exactly one of them runs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "kernels/kmeans_frag.h"
#include "kernels/kmeans_internal.h"

namespace oap {
namespace kern {

namespace {

using namespace kmdev;

#define OAP_AI __attribute__((always_inline))

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr float kBias = 16.f;  // the bias features' unit (kmeans_lloyd.hip kBiasUnit)
constexpr int kMv = 64;        // per-wave LDS slots of staged moved rows

struct ImgArgs {
  const f16x8* img;  // [tiles][KS][64] fragments
  const float* img_beta;
  const float* x;  // f32 rows [n][ld] (moved rows only)
  const float* centers;
  const float* cnorm;
  const float* cstat;
  const float* scale;
  u64* sums;
  u64* counts;
  int32_t* labels;
  float2* bounds;
  const int32_t* tile_list;
  const unsigned* tile_count;
  int32_t* defer_rows;
  unsigned* defer_row_count;
  u64* stat;  // optional [deferred rows, moved rows, image passes]
  int64_t n, seg_cap, tiles_per_block;
  int ld, d, k, kpad;
};

struct ImgSmem {
  size_t plane, sc, acc, cnt, mv, total;
};

// fp16 plane; fixed-point accumulator rows of DP + 1 doubles (odd: conflict-free ds_add_f64; the
// padded features add zeros into their own columns, so the moved-row adds need no predicate)
__host__ __device__ inline ImgSmem img_plan(int dp, int kpad, int k, int waves) {
  ImgSmem m;
  size_t off = 0;
  m.plane = 0;
  off = round16(size_t(kpad) * stride_bf16(dp) * 2);
  m.sc = off;
  off = round16(off + size_t(dp) * 4);
  m.acc = off;
  off = round16(off + size_t(k) * (dp + 1) * 8);
  m.cnt = off;
  off = round16(off + size_t(k) * 4);
  m.mv = off;
  off += size_t(waves) * kMv * 8;
  m.total = round16(off);
  return m;
}

__device__ inline void split_h(float v, _Float16& hi, _Float16& lo) {
  hi = static_cast<_Float16>(v);
  lo = static_cast<_Float16>(v - static_cast<float>(hi));
}

// CFG: bit 0 software-pipelined chunk loop; bit 1 operands two tiles ahead (else one); bits 2+
// timing ablations (probe builds only): 4 no epilogue, 8 no MFMA, 16 no plane reads, 32 no image
// loads, 64 no moved-row accumulation, 128 no per-row stores
template <int KS, int WAVES, int CFG>
__global__ __launch_bounds__(WAVES * 64, 1) void oap_kmeans_lean_img(ImgArgs a) {
  constexpr bool PIPE = (CFG & 1) != 0;
  constexpr int PD = (CFG & 2) ? 2 : 1;
  constexpr bool NO_EPI = (CFG & 4) != 0, NO_MFMA = (CFG & 8) != 0, NO_LDS = (CFG & 16) != 0;
  constexpr bool NO_LOAD = (CFG & 32) != 0, NO_ACC = (CFG & 64) != 0, NO_ST = (CFG & 128) != 0;
  constexpr int DP = 16 * KS, NT = WAVES * 64, RS = DP + 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const float cmax = a.cstat[0];
  const float alpha = a.img_beta[0];
  if (!(alpha * cmax <= 512.f)) return;  // (kmeans_lloyd img_mode 3 takes this pass)
  const int k = a.k, kpad = a.kpad, d = a.d;
  const ImgSmem L = img_plan(DP, kpad, k, WAVES);
  const int sb = stride_bf16(DP);
  _Float16* ph = reinterpret_cast<_Float16*>(smem + L.plane);
  float* sc_l = reinterpret_cast<float*>(smem + L.sc);
  double* acc_l = reinterpret_cast<double*>(smem + L.acc);
  int* cnt_l = reinterpret_cast<int*>(smem + L.cnt);
  const int tid = threadIdx.x;
  const float a2 = alpha * alpha;
  const float inv_a2 = 1.f / a2;  // (a power of two)
  // ---- the plane c' = [-2 alpha c, 0 .., hi, lo (alpha^2 |c|^2 / 16), 16, 16] (kmeans_lloyd.hip)
  for (int idx = tid; idx < kpad * DP; idx += NT) {
    const int c = idx / DP, f = idx - c * DP;
    _Float16 v;
    if (f < d) {
      v = static_cast<_Float16>(-2.f * alpha * a.centers[idx]);
    } else if (f == DP - 4 || f == DP - 3) {
      _Float16 hi, lo;
      split_h((c < k) ? a2 * a.cnorm[c] * (1.f / kBias) : 60000.f, hi, lo);
      v = (f == DP - 4) ? hi : lo;
    } else {
      v = static_cast<_Float16>(f >= DP - 2 ? kBias : 0.f);
    }
    ph[c * sb + f] = v;
  }
  for (int f = tid; f < DP; f += NT) sc_l[f] = f < d ? a.scale[f] : 0.f;
  for (int i = tid; i < k * RS; i += NT) acc_l[i] = 0.0;
  for (int i = tid; i < k; i += NT) cnt_l[i] = 0;
  __syncthreads();

  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  int2* mv_l = reinterpret_cast<int2*>(smem + L.mv) + wave * kMv;
  // tier-1 bound (kmeans_lloyd.hip, f32 rows): cross term, subnormals, bias pairs, accumulation
  const float cm_s = alpha * cmax;
  const float thr_c = 0.0040f * cm_s;
  const float thr_k = 6e-5f * cm_s * cm_s + float(d) * 6.2e-5f + 1e-30f;
  const float mrel = 4e-7f * float(d + 8);
  const int64_t ntiles_all = (a.n + 31) / 32;
  const bool listed = a.tile_list != nullptr;
  const int64_t T = a.tiles_per_block;
  const int64_t t0 = int64_t(blockIdx.x) * T;
  const int64_t npos = listed ? int64_t(a.tile_count[blockIdx.x])
                              : (t0 < ntiles_all ? (ntiles_all - t0 < T ? ntiles_all - t0 : T) : 0);
  const int32_t* seg = listed ? a.tile_list + blockIdx.x * T : nullptr;
  constexpr int64_t stride = WAVES;
  const int64_t sub_cap = a.seg_cap / WAVES;
  int32_t* dseg = a.defer_rows + blockIdx.x * a.seg_cap + wave * sub_cap;
  unsigned n_def = 0;  // wave-uniform
  const int64_t row0 = t0 * 32;
  const int64_t wrows = row0 < a.n ? (a.n - row0 < T * 32 ? a.n - row0 : T * 32) : 0;
  const __amdgpu_buffer_rsrc_t rs_lab = buf_rsrc(a.labels + row0, uint32_t(wrows * 4));
  const __amdgpu_buffer_rsrc_t rs_bnd =
      buf_rsrc(a.bounds ? a.bounds + row0 : nullptr, a.bounds ? uint32_t(wrows * 8) : 0u);
  const __amdgpu_buffer_rsrc_t rs_def = buf_rsrc(dseg, uint32_t(sub_cap * 4));
  const bool want_bounds = a.bounds != nullptr;
  // last chunk: its real 8-centroid groups (the earlier chunks are all real: kpad = 32 ceil(k/32))
  const int c_last = kpad - 32;
  const int ng_last = (k - c_last + 7) >> 3;  // 1..4

  auto tile_of = [&](int64_t q) OAP_AI -> int64_t {
    if (npos == 0) return 0;
    q = q < npos ? q : npos - 1;
    if (!listed) return t0 + q;
    typedef const int32_t __attribute__((address_space(4)))* seg_cptr;  // (scalar load)
    const int64_t tl = int64_t(((seg_cptr)(seg))[q]);
    return tl < 0 ? 0 : (tl < ntiles_all ? tl : ntiles_all - 1);
  };
  auto load_img = [&](int64_t tile, f16x8(&dst)[KS]) OAP_AI {
    if constexpr (!NO_LOAD) {
      const f16x8* p = a.img + tile * (KS * 64) + lane;
#pragma unroll
      for (int s = 0; s < KS; ++s) dst[s] = p[s * 64];
    }
  };

  // ---- moved rows: staged (row, new | old << 16) in the wave's LDS slots, accumulated 32 at a
  // time with every lane busy (fixed-point +x into new, -x into old)
  unsigned n_mv = 0;  // wave-uniform
  u64 moved_total = 0;
  auto flush = [&](unsigned cnt) OAP_AI {  // entries [0, min(cnt, 32))
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool on = unsigned(r) < cnt;
    const int2 e = mv_l[on ? r : 0];
    float xv[KS][8];
    {
      const float* p = a.x + int64_t(e.x) * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int f = 16 * s + 8 * h + 4 * q;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (s < KS - 1 || f < a.ld) v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
          xv[s][4 * q + 0] = v.x;
          xv[s][4 * q + 1] = v.y;
          xv[s][4 * q + 2] = v.z;
          xv[s][4 * q + 3] = v.w;
        }
    }
    if (on) {
      const int b = e.y & 0xffff, bo = e.y >> 16;
      if (h == 0) {
        atomicAdd(&cnt_l[b], 1);
        atomicAdd(&cnt_l[bo], -1);
      }
      double* ap = acc_l + b * RS + 8 * h;
      double* aq = acc_l + bo * RS + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float4 s0 = *reinterpret_cast<const float4*>(sc_l + 16 * s + 8 * h);
        const float4 s1 = *reinterpret_cast<const float4*>(sc_l + 16 * s + 8 * h + 4);
        const float scv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // (features >= d: scale 0, a zero into a pad column)
          const double v = static_cast<double>(rintf(xv[s][j] * scv[j]));
          atomicAdd(ap + 16 * s + j, v);
          atomicAdd(aq + 16 * s + j, -v);
        }
      }
    }
    if (cnt > 32) {  // slide the rest down (read all before any write: in-order LDS)
      const int2 rest = mv_l[32 + r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (h == 0 && unsigned(r) < cnt - 32) mv_l[r] = rest;
    }
    moved_total += cnt < 32 ? cnt : 32;
    // drain the row loads here: a younger load left pending would make every later tile's
    // wait for its operand prefetch wait for it too (vmcnt counts in issue order)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  };

  // ---- one tile: X holds its operands (landed or in flight), pf receives tile pos + PD stride
  auto body = [&](const int64_t pos, f16x8(&X)[KS], f16x8(&pf)[KS]) OAP_AI {
    if constexpr (!NO_ACC) {
      if (n_mv >= 32) {  // (before this tile's loads are issued)
        flush(n_mv);
        n_mv -= 32;
      }
    }
    const int64_t tile = tile_of(pos);
    const int64_t row = tile * 32 + r;
    const bool valid = pos < npos && row < a.n;
    const uint32_t roff = uint32_t(row - row0);
    int old = buf_load_b32(rs_lab, roff * 4, valid);
    load_img(tile_of(pos + PD * stride), pf);
    // alpha^2 |x|^2 from the bias pair (h = 1 lanes' slots 6, 7 of the last k-step)
    const float mine =
        kBias * (static_cast<float>(X[KS - 1][6]) + static_cast<float>(X[KS - 1][7]));
    const float other = xor32_f(mine);
    const float nx2_s = h ? mine : other;
    int k1 = 0x7fffffff, k2 = 0x7fffffff;
    auto frags = [&](int c0, f16x8(&av)[KS]) OAP_AI {
      if constexpr (NO_LDS) {
#pragma unroll
        for (int s = 0; s < KS; ++s) av[s] = X[(s + 1) % KS];
      } else {
        const _Float16* ap = ph + size_t(c0 + r) * sb + 8 * h;
#pragma unroll
        for (int s = 0; s < KS; ++s) av[s] = *reinterpret_cast<const f16x8*>(ap + 16 * s);
      }
    };
    auto chain = [&](const f16x8(&av)[KS], f32x16& acc) OAP_AI {
      if constexpr (NO_MFMA) {
#pragma unroll
        for (int q = 0; q < 4 && q < KS; ++q) {
          const f32x4 w = __builtin_bit_cast(f32x4, av[q]);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[4 * q + e] = w[e];
        }
      } else {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[0], X[0], f32x16{}, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < KS; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s], X[s], acc, 0, 0, 0);
      }
    };
    // keys: the distance's bits with the low 10 mantissa bits replaced by the centroid's offset
    // (value order, lowest index first); padded centroids carry the largest finite bias and
    // never win.  NG groups of 8 centroids (4 per lane); the pair fold is 3 VALU per 2 keys.
    auto epi = [&](auto ng_t, int c0, const f32x16& acc) OAP_AI {
      constexpr int NG = decltype(ng_t)::value;
      if constexpr (NO_EPI) {
        k1 = min(k1, (__float_as_int(acc[0]) & ~0x3ff) | (c0 + 4 * h));
        return;
      }
      int key[4 * NG];
#pragma unroll
      for (int e = 0; e < 4 * NG; ++e)
        key[e] = (__float_as_int(acc[e]) & ~0x3ff) | (8 * (e >> 2) + (e & 3));
      int t1 = min(key[0], key[1]), t2 = max(key[0], key[1]);
#pragma unroll
      for (int e = 2; e < 4 * NG; e += 2) {
        t2 = min(t2, med3_i32_pure(t1, key[e], key[e + 1]));
        t1 = min(min(t1, key[e]), key[e + 1]);
      }
      const int base = c0 + 4 * h;
      const int i1 = t1 | base, i2 = t2 | base;
      k2 = min(max(k1, i1), min(k2, i2));
      k1 = min(k1, i1);
    };
    auto epi_last = [&](const f32x16& acc) OAP_AI {
      switch (ng_last) {  // (wave-uniform)
        case 1: epi(std::integral_constant<int, 1>{}, c_last, acc); break;
        case 2: epi(std::integral_constant<int, 2>{}, c_last, acc); break;
        case 3: epi(std::integral_constant<int, 3>{}, c_last, acc); break;
        default: epi(std::integral_constant<int, 4>{}, c_last, acc); break;
      }
    };
    const std::integral_constant<int, 4> full{};
    f16x8 av[KS];
    if constexpr (!PIPE) {
      for (int c0 = 0; c0 < c_last; c0 += 32) {
        f32x16 acc;
        frags(c0, av);
        chain(av, acc);
        epi(full, c0, acc);
      }
      f32x16 acc;
      frags(c_last, av);
      chain(av, acc);
      epi_last(acc);
    } else {
      // chunk c's epilogue runs while chunk c + 1's MFMA chain is in the matrix pipe (its
      // fragment reads land under the tail of chunk c's chain; the fragment registers are dead
      // during the epilogue: two accumulators fit the 128-register budget without spills)
      f32x16 accA, accB;
      frags(0, av);
      chain(av, accA);
      int c0 = 0;
      bool last_in_b = false;
      while (c0 < c_last) {  // invariant: accA holds chunk c0 (issued)
        frags(c0 + 32, av);
        chain(av, accB);
        epi(full, c0, accA);
        c0 += 32;
        if (c0 == c_last) {
          last_in_b = true;
          break;
        }
        frags(c0 + 32, av);
        chain(av, accA);
        epi(full, c0, accB);
        c0 += 32;
      }
      if (last_in_b)
        epi_last(accB);
      else
        epi_last(accA);
    }
    // ---- the two halves of the row: top-2 of the union
    const int o1 = xor32_i(k1), o2 = xor32_i(k2);
    k2 = min(max(k1, o1), min(k2, o2));
    k1 = min(k1, o1);
    const float b1 = __int_as_float(k1 & ~0x3ff);
    const float b2 = __int_as_float(k2 & ~0x3ff);
    const float tt = fmaf(thr_c, __builtin_amdgcn_sqrtf(nx2_s), thr_k) + 5e-5f * nx2_s +
                     2.5e-4f * fabsf(b2);
    // rows beyond fp16's comfortable range (alpha |x| >= 2^10) are always re-decided
    const bool unsure = valid && (!(b2 - b1 > tt) || !(nx2_s < 1048576.f));
    // ---- defer unsure rows (wave-private sub-segment, in tile order)
    const unsigned long long um = __ballot(unsure && h == 0);
    buf_store_b32(rs_def, (n_def + __popcll(um & ((1ull << lane) - 1ull))) * 4u,
                  static_cast<int32_t>(row), !NO_ST && unsure && h == 0);
    n_def += static_cast<unsigned>(__popcll(um));
    const bool done = valid && !unsure;
    int b = k1 & 0x3ff;
    b = (b < k) ? b : 0;  // only for degenerate (NaN / all-inf) inputs
    const bool moved = done && old >= 0 && old != b;
    if constexpr (!NO_ACC) {
      const unsigned long long mm = __ballot(moved && h == 0);
      if (mm) {
        if (moved && h == 0)
          mv_l[n_mv + __popcll(mm & ((1ull << lane) - 1ull))] =
              make_int2(static_cast<int>(row), b | (min(old, k - 1) << 16));
        n_mv += static_cast<unsigned>(__popcll(mm));
      }
    }
    // labels: only the rows that moved (the others already hold theirs)
    buf_store_b32(rs_lab, roff * 4, b, !NO_ST && moved && h == 0);
    // bounds (when a following iteration may scan): the pick's alpha^2 distance is <= b1 + tt,
    // every other one >= b2 - tt
    float2 bnd = make_float2(0.f, 0.f);
    if (want_bounds) {
      const float mg = mrel * (nx2_s + cm_s * cm_s);
      const float up = (b1 + tt + mg) * inv_a2, lo = (b2 - (tt + mg)) * inv_a2;
      bnd = make_float2(__builtin_amdgcn_sqrtf(fmaxf(up, 0.f)) * (1.f + 1e-6f) + 1e-30f,
                        __builtin_amdgcn_sqrtf(fmaxf(lo, 0.f)) * (1.f - 1e-6f));
    }
    buf_store_f2(rs_bnd, roff * 8, bnd, !NO_ST && done && h == 0);
  };

  int64_t t = wave;
  if constexpr (PD == 1) {
    f16x8 xa[KS], xb[KS];
    load_img(tile_of(t), xa);
    if constexpr (NO_LOAD) {
#pragma unroll
      for (int s = 0; s < KS; ++s) xa[s] = xb[s] = f16x8{};
    }
    for (; t < npos; t += 2 * stride) {  // t is wave-uniform: every branch stays uniform
      body(t, xa, xb);
      if (t + stride >= npos) break;
      body(t + stride, xb, xa);
    }
  } else {
    f16x8 xa[KS], xb[KS], xc[KS];
    load_img(tile_of(t), xa);
    load_img(tile_of(t + stride), xb);
    if constexpr (NO_LOAD) {
#pragma unroll
      for (int s = 0; s < KS; ++s) xa[s] = xb[s] = xc[s] = f16x8{};
    }
    for (; t < npos; t += 3 * stride) {
      body(t, xa, xc);
      if (t + stride >= npos) break;
      body(t + stride, xb, xa);
      if (t + 2 * stride >= npos) break;
      body(t + 2 * stride, xc, xb);
    }
  }
  if constexpr (!NO_ACC) {
    while (n_mv) {  // (at most 63 staged)
      flush(n_mv);
      n_mv = n_mv > 32 ? n_mv - 32 : 0;
    }
  }
  if (lane == 0) {
    if (a.stat && blockIdx.x == 0 && wave == 0) atomicAdd(a.stat + 2, 1ull);  // (image passes)
    a.defer_row_count[blockIdx.x * kDeferSubs + wave] = n_def;
    if (a.stat && n_def) atomicAdd(a.stat, u64(n_def));
    if (a.stat && moved_total) atomicAdd(a.stat + 1, moved_total);
  }
  __syncthreads();
  for (int i = tid; i < k * d; i += NT) {
    const int c = i / d, f = i - c * d;
    const double v = acc_l[c * RS + f];  // an exact integer, |v| < 2^53
    if (v != 0.0) atomicAdd(&a.sums[i], static_cast<u64>(static_cast<long long>(v)));
  }
  for (int i = tid; i < k; i += NT) {
    const int c = cnt_l[i];
    if (c) atomicAdd(&a.counts[i], static_cast<u64>(static_cast<long long>(c)));
  }
}

template <int KS, int WAVES, int CFG>
void launch_img(const ImgArgs& a, int grid, hipStream_t s) {
  const ImgSmem L = img_plan(16 * KS, a.kpad, a.k, WAVES);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&oap_kmeans_lean_img<KS, WAVES, CFG>),
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_lean_img<KS, WAVES, CFG>), dim3(grid), dim3(WAVES * 64), L.total,
                     s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

constexpr int kImgDefaultCfg = 1;  // pipelined chunk loop, operands one tile ahead

template <int KS, int WAVES>
void launch_img_cfg(const ImgArgs& a, int grid, int cfg, hipStream_t s) {
  if constexpr (KS == 4 && WAVES == 16) {  // the headline shape: every probe configuration
    switch (cfg) {
      case 0: launch_img<4, 16, 0>(a, grid, s); return;
      case 1: launch_img<4, 16, 1>(a, grid, s); return;
      case 2: launch_img<4, 16, 2>(a, grid, s); return;
      case 3: launch_img<4, 16, 3>(a, grid, s); return;
      case 1 | 4: launch_img<4, 16, 1 | 4>(a, grid, s); return;
      case 1 | 8: launch_img<4, 16, 1 | 8>(a, grid, s); return;
      case 1 | 16: launch_img<4, 16, 1 | 16>(a, grid, s); return;
      case 1 | 32: launch_img<4, 16, 1 | 32>(a, grid, s); return;
      case 1 | 64: launch_img<4, 16, 1 | 64>(a, grid, s); return;
      case 1 | 128: launch_img<4, 16, 1 | 128>(a, grid, s); return;
      case 1 | 4 | 8 | 16: launch_img<4, 16, 1 | 4 | 8 | 16>(a, grid, s); return;
      case 1 | 4 | 64 | 128: launch_img<4, 16, 1 | 4 | 64 | 128>(a, grid, s); return;
      case 1 | 8 | 64 | 128: launch_img<4, 16, 1 | 8 | 64 | 128>(a, grid, s); return;
      case 1 | 4 | 16 | 64 | 128: launch_img<4, 16, 1 | 4 | 16 | 64 | 128>(a, grid, s); return;
      case 1 | 4 | 32 | 64 | 128: launch_img<4, 16, 1 | 4 | 32 | 64 | 128>(a, grid, s); return;
      case 4 | 64 | 128: launch_img<4, 16, 4 | 64 | 128>(a, grid, s); return;
      case 1 | 4 | 8 | 16 | 64 | 128:
        launch_img<4, 16, 1 | 4 | 8 | 16 | 64 | 128>(a, grid, s);
        return;
      default: break;
    }
  }
  launch_img<KS, WAVES, kImgDefaultCfg>(a, grid, s);
}

template <int WAVES>
void launch_img_w(const ImgArgs& a, int grid, int cfg, hipStream_t s) {
  switch ((a.d + 4 + 15) / 16) {
    case 1: launch_img_cfg<1, WAVES>(a, grid, cfg, s); break;
    case 2: launch_img_cfg<2, WAVES>(a, grid, cfg, s); break;
    case 3: launch_img_cfg<3, WAVES>(a, grid, cfg, s); break;
    case 4: launch_img_cfg<4, WAVES>(a, grid, cfg, s); break;
    case 5: launch_img_cfg<5, WAVES>(a, grid, cfg, s); break;
    case 6: launch_img_cfg<6, WAVES>(a, grid, cfg, s); break;
    case 7: launch_img_cfg<7, WAVES>(a, grid, cfg, s); break;
    case 8: launch_img_cfg<8, WAVES>(a, grid, cfg, s); break;
    default: OAP_THROW(ConfigError, "kmeans_lean_img: unsupported d=" << a.d);
  }
}

}  // namespace

bool kmeans_lean_img_supported(int d, int k, int waves) {
  if (d + 4 > 128 || k < 1 || (waves != 12 && waves != 16)) return false;
  const int dp = (d + 4 + 15) / 16 * 16;
  if (dp != kmeans_dp(d)) return false;
  const int kpad = (k + 31) / 32 * 32;
  if (kpad > 1024) return false;
  return img_plan(dp, kpad, k, waves).total <= kLdsLimit;
}

void kmeans_lean_img(const KMeansAssignArgs& a, int grid, int waves, int cfg, hipStream_t s) {
  OAP_CHECK(kmeans_lean_img_supported(a.d, a.k, waves) && !a.xbf16 && a.ximg && a.img_beta &&
                a.delta && a.labels && a.scale && a.sums && a.counts && a.accumulate &&
                a.sums_too && a.defer_rows && a.defer_row_count && a.cstat && !a.xnorm &&
                !a.cost_slab && !a.mindist && !a.centers_all && a.chunk_mode == 0 &&
                a.row_seg_cap == kmeans_lloyd_seg_cap(a.n, grid, waves) &&
                a.ld == kmeans_ld(a.d, false) && (!a.tile_list || a.tile_count),
            "kmeans_lean_img: unsupported arguments");
  if (a.n == 0) return;
  ImgArgs l;
  l.img = static_cast<const f16x8*>(a.ximg);
  l.img_beta = a.img_beta;
  l.x = static_cast<const float*>(a.x);
  l.centers = a.centers;
  l.cnorm = a.cnorm;
  l.cstat = a.cstat;
  l.scale = a.scale;
  l.sums = a.sums;
  l.counts = a.counts;
  l.labels = a.labels;
  l.bounds = reinterpret_cast<float2*>(a.bounds);
  l.tile_list = a.tile_list;
  l.tile_count = a.tile_count;
  l.defer_rows = a.defer_rows;
  l.defer_row_count = a.defer_row_count;
  l.stat = a.deferred_rows;
  l.n = a.n;
  l.seg_cap = a.row_seg_cap;
  l.tiles_per_block = kmeans_lloyd_tiles_per_block(a.n, grid);
  l.ld = a.ld;
  l.d = a.d;
  l.k = a.k;
  l.kpad = a.kpad;
  if (waves == 12)
    launch_img_w<12>(l, grid, cfg < 0 ? kImgDefaultCfg : cfg, s);
  else
    launch_img_w<16>(l, grid, cfg < 0 ? kImgDefaultCfg : cfg, s);
}

}  // namespace kern
}  // namespace oap
