// K-Means kernels for MI355X (gfx950, CDNA4).
//
// Replaces the oneDAL step1Local / step2Master pair the reference calls every Lloyd iteration
// (mllib-dal/src/main/native/KMeansDALImpl.cpp:70-77 and :101-130).
//
// oap_kmeans_assign_mfma<KS, PRECISE> — the fused hot kernel (K1), one launch per iteration:
//   * Layout: a wave owns a 32-row tile; lane (r = l&31, h = l>>5) holds features
//     f = 16s + 8h + j (s < KS, j < 8) of row r in registers.  Centroids are the MFMA A operand
//     (32 per block of rows), staged ONCE per workgroup in LDS with an odd-16B-slot row stride
//     (conflict-free ds_read_b128); data rows are the B operand straight from registers.  The
//     32x32 accumulator gives each lane one data row x 16 centroids, so argmin is a per-lane scan
//     plus one cross-half exchange — no LDS round trip.
//   * Fast path (default): the cross term x.c runs on the bf16 matrix cores as a 3-product split
//     (x_hi c_hi + x_hi c_lo + x_lo c_hi, each operand = hi + lo bf16 parts, fp32 accumulate):
//     3 x v_mfma_f32_32x32x16_bf16 replace 8 x v_mfma_f32_32x32x2_f32 per 16 features, i.e.
//     ~5x the fp32 matrix rate.  Its error is bounded by 4.6e-5 |x| |c| per distance; every row
//     whose best/second-best gap is below that bound (plus the fp32 path's own bound) is
//     re-decided by the exact-fp32 MFMA pass below for its whole tile.  Result: assignments are
//     IDENTICAL to the exact-fp32 kernel (tested bitwise), at bf16-split speed.
//   * Exact path (PRECISE, and the refinement): v_mfma_f32_32x32x2_f32 (exact fp32 products,
//     one rounding each) with the same feature order, so both paths agree bit for bit.
//   * Exact per-row cost |x - c_best|^2 re-computed in fp32 from the chosen center (no expansion
//     cancellation in the reported trainingCost).
//   * Centroid sums accumulated as 64-bit FIXED POINT (x * 2^e_f, e_f per feature from the global
//     column max so no sum can overflow) with ds_add_u64 into an LDS accumulator, flushed once per
//     workgroup with 64-bit integer atomics.  Integer addition is associative: sums are bitwise
//     identical for any block schedule, rank count and RCCL reduction order — a reproducibility
//     property the reference's root-merged fp64 archives cannot offer (KMeansDALImpl.cpp:97-130).
//   * Persistent grid: one 512-thread workgroup per CU (8 waves = 2 per SIMD, one wave's VALU
//     epilogue overlapping the other's MFMAs), register prefetch of the next tile.
// oap_kmeans_finalize — K2+K3 fused: new centroids (Spark rule: empty clusters keep their center,
//   spark-3.1.1/mllib/clustering/KMeans.scala:306-330) and the tolerance test Σ(Δc)² <= tol²
//   evaluated redundantly on every rank (no root, no broadcast — SURVEY.md §2.7 C2/C3/C5).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "kernels/device_utils.h"
#include "kernels/kernels.h"

namespace oap {
namespace kern {

namespace {

constexpr int kThreads = 512;  // 8 waves
constexpr int kWaves = kThreads / 64;
constexpr size_t kLdsLimit = 160 * 1024;

__host__ __device__ inline size_t round16(size_t v) { return (v + 15) / 16 * 16; }
__host__ __device__ inline int stride_bf16(int dp) { return dp + 8; }  // (dp+8)/8 odd slots
__host__ __device__ inline int stride_f32(int dp) { return dp + 4; }   // (dp+4)/4 odd slots

struct Smem {
  size_t planes, cn, acc, cnt, wcost, total;
};
__host__ __device__ inline Smem smem_plan(int dp, int kpad, int k, int d, bool precise,
                                          bool lds_acc) {
  Smem m;
  size_t off = 0;
  m.planes = 0;
  off += precise ? size_t(kpad) * stride_f32(dp) * 4 : size_t(2) * kpad * stride_bf16(dp) * 2;
  off = round16(off);
  m.cn = off;
  off = round16(off + size_t(kpad) * 4);
  m.acc = off;
  if (lds_acc) off += size_t(k) * (d | 1) * 8;  // odd row stride: conflict-free ds_add_u64
  m.cnt = off;
  if (lds_acc) off += size_t(k) * 8;
  off = round16(off);
  m.wcost = off;
  off += kWaves * 8;
  m.total = round16(off);
  return m;
}

// Exact fp32 argmin over all kpad centroids for the lane's row (both halves see the result).
// cbase row stride `stride`; reads A fragments as float4 (16-B aligned by construction).
template <int KS>
__device__ inline void exact_argmin(const float* __restrict__ cbase, int stride,
                                    const float (&x)[KS][8], const float* __restrict__ cn,
                                    int kpad, int d, int r, int h, float& best, int& bidx) {
  best = INFINITY;
  bidx = 0x7fffffff;
  for (int c0 = 0; c0 < kpad; c0 += 32) {
    f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float* cp = cbase + size_t(c0 + r) * stride + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (16 * s + 4 * q < d) {  // wave-uniform: skip groups that are all padding
          float4 a4 = *reinterpret_cast<const float4*>(cp + 16 * s + 4 * q);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, x[s][4 * q + 0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, x[s][4 * q + 1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, x[s][4 * q + 2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, x[s][4 * q + 3], acc, 0, 0, 0);
        }
      }
    }
    // accumulator element 4g+q <-> centroid c0 + 8g + 4h + q, data row r
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float4 c4 = *reinterpret_cast<const float4*>(cn + c0 + 8 * g + 4 * h);
      float cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float dist = fmaf(-2.f, acc[4 * g + q], cv[q]);
        if (dist < best) {
          best = dist;
          bidx = c0 + 8 * g + 4 * h + q;
        }
      }
    }
  }
  float ob = __shfl_xor(best, 32, 64);
  int oi = __shfl_xor(bidx, 32, 64);
  if (ob < best || (ob == best && oi < bidx)) {
    best = ob;
    bidx = oi;
  }
}

template <int KS, bool PRECISE>
__global__ __launch_bounds__(kThreads, 2) void oap_kmeans_assign_mfma(KMeansAssignArgs a,
                                                                       int lds_acc) {
  constexpr int DP = 16 * KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int kpad = a.kpad, k = a.k, d = a.d;
  const Smem L = smem_plan(DP, kpad, k, d, PRECISE, lds_acc != 0);
  const int sb = stride_bf16(DP), s32 = stride_f32(DP);
  __bf16* ph = reinterpret_cast<__bf16*>(smem + L.planes);
  __bf16* pl = ph + size_t(kpad) * sb;
  float* p32 = reinterpret_cast<float*>(smem + L.planes);
  float* cn = reinterpret_cast<float*>(smem + L.cn);
  u64* acc_l = reinterpret_cast<u64*>(smem + L.acc);
  u64* cnt_l = reinterpret_cast<u64*>(smem + L.cnt);
  double* wcost = reinterpret_cast<double*>(smem + L.wcost);
  const int tid = threadIdx.x;
  const bool accumulate = a.accumulate && !a.merge;

  // ---- stage the centroids once per workgroup
  for (int idx = tid; idx < kpad * DP; idx += kThreads) {
    int c = idx / DP, f = idx - c * DP;
    float v = a.centers[idx];
    if constexpr (PRECISE) {
      p32[c * s32 + f] = v;
    } else {
      __bf16 hi, lo;
      bf16_split(v, hi, lo);
      ph[c * sb + f] = hi;
      pl[c * sb + f] = lo;
    }
  }
  for (int c = tid; c < kpad; c += kThreads) cn[c] = (c < k) ? a.cnorm[c] : INFINITY;
  if (lds_acc && accumulate) {
    for (int i = tid; i < k * (d | 1); i += kThreads) acc_l[i] = 0ull;
    for (int i = tid; i < k; i += kThreads) cnt_l[i] = 0ull;
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  float thr1 = 0.f, thr0 = 0.f;
  if constexpr (!PRECISE) {
    const float cmax = a.cstat ? a.cstat[0] : 0.f;
    thr1 = 1.25e-4f * cmax;  // 2 candidates x (bf16-split + accumulation) + fp32-path bound
    thr0 = 2e-6f * cmax * cmax + 1e-30f;
  }

  double my_cost = 0.0;
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t stride = int64_t(gridDim.x) * kWaves;
  int64_t t = int64_t(blockIdx.x) * kWaves + wave;

  float xn[KS][8];
  auto load_tile = [&](int64_t tt, float (&dst)[KS][8]) {
    const int64_t row = tt * 32 + r;
    const bool ok = tt < ntiles && row < a.n;
    const float* p = a.x + (ok ? row : 0) * a.ld + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int f = 16 * s + 8 * h + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok && f < a.ld) v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
        dst[s][4 * q + 0] = v.x;
        dst[s][4 * q + 1] = v.y;
        dst[s][4 * q + 2] = v.z;
        dst[s][4 * q + 3] = v.w;
      }
    }
  };
  load_tile(t, xn);

  for (; t < ntiles; t += stride) {
    float x[KS][8];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[s][j] = xn[s][j];
    const int64_t row = t * 32 + r;
    const bool valid = row < a.n;
    load_tile(t + stride, xn);  // prefetch, hidden behind the MFMA work of this tile

    int bidx;
    if constexpr (PRECISE) {
      float best;
      exact_argmin<KS>(p32, s32, x, cn, kpad, d, r, h, best, bidx);
    } else {
      bf16x8 xh[KS], xl[KS];
      float nx2 = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 hi, lo;
          bf16_split(x[s][j], hi, lo);
          xh[s][j] = hi;
          xl[s][j] = lo;
          nx2 = fmaf(x[s][j], x[s][j], nx2);
        }
      nx2 += __shfl_xor(nx2, 32, 64);
      float b1 = INFINITY, b2 = INFINITY;
      int bi = 0x7fffffff;
      for (int c0 = 0; c0 < kpad; c0 += 32) {
        f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                      0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const __bf16* ah_p = ph + size_t(c0 + r) * sb + 8 * h;
        const __bf16* al_p = pl + size_t(c0 + r) * sb + 8 * h;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          if (16 * s < d) {
            bf16x8 ah = *reinterpret_cast<const bf16x8*>(ah_p + 16 * s);
            bf16x8 al = *reinterpret_cast<const bf16x8*>(al_p + 16 * s);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xl[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, xh[s], acc, 0, 0, 0);
          }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float4 c4 = *reinterpret_cast<const float4*>(cn + c0 + 8 * g + 4 * h);
          float cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float dist = fmaf(-2.f, acc[4 * g + q], cv[q]);
            if (dist < b1) {
              b2 = b1;
              b1 = dist;
              bi = c0 + 8 * g + 4 * h + q;
            } else {
              b2 = fminf(b2, dist);
            }
          }
        }
      }
      {  // merge the two halves' top-2
        float o1 = __shfl_xor(b1, 32, 64), o2 = __shfl_xor(b2, 32, 64);
        int oi = __shfl_xor(bi, 32, 64);
        if (o1 < b1 || (o1 == b1 && oi < bi)) {
          b2 = fminf(b1, o2);
          b1 = o1;
          bi = oi;
        } else {
          b2 = fminf(o1, b2);
        }
      }
      const bool unsure = valid && !(b2 - b1 > fmaf(thr1, sqrtf(nx2), thr0));
      if (__any(unsure)) {
        // rare: re-decide the whole tile exactly (identical to the PRECISE kernel)
        exact_argmin<KS>(a.centers, DP, x, cn, kpad, d, r, h, b1, bi);
        if (lane == 0 && a.refine_tiles) atomicAdd(a.refine_tiles, 1ull);
      }
      bidx = bi;
    }
    if (bidx >= k) bidx = 0;  // only reachable for degenerate (NaN / all-inf) inputs

    // exact squared distance to the chosen center
    const float* cb = PRECISE ? (p32 + size_t(bidx) * s32 + 8 * h)
                              : (a.centers + size_t(bidx) * DP + 8 * h);
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (16 * s < d) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float4 c4 = *reinterpret_cast<const float4*>(cb + 16 * s + 4 * q);
          float e0 = x[s][4 * q] - c4.x, e1 = x[s][4 * q + 1] - c4.y;
          float e2 = x[s][4 * q + 2] - c4.z, e3 = x[s][4 * q + 3] - c4.w;
          part = fmaf(e0, e0, part);
          part = fmaf(e1, e1, part);
          part = fmaf(e2, e2, part);
          part = fmaf(e3, e3, part);
        }
      }
    }
    const float rowcost = part + __shfl_xor(part, 32, 64);
    if (!valid) continue;
    if (h == 0) {
      if (a.merge) {
        if (rowcost < a.mindist[row]) {
          a.mindist[row] = rowcost;
          a.labels[row] = a.base + bidx;
        }
      } else {
        if (a.labels) a.labels[row] = a.base + bidx;
        if (a.mindist) a.mindist[row] = rowcost;
      }
      my_cost += double(rowcost);
    }
    if (accumulate) {
      if (h == 0) atomicAdd(lds_acc ? &cnt_l[bidx] : &a.counts[bidx], 1ull);
      if (a.sums_too) {
        u64* ap = lds_acc ? acc_l + size_t(bidx) * (d | 1) : a.sums + size_t(bidx) * d;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int f0 = 16 * s + 8 * h + 4 * q;
            if (f0 < d) {
              float4 sc = *reinterpret_cast<const float4*>(a.scale + f0);
              float scv[4] = {sc.x, sc.y, sc.z, sc.w};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                if (f0 + j < d) {
                  long long qv = static_cast<long long>(rintf(x[s][4 * q + j] * scv[j]));
                  atomicAdd(ap + f0 + j, static_cast<u64>(qv));
                }
              }
            }
          }
        }
      }
    }
  }

  // ---- deterministic per-block cost: fixed shuffle tree, then waves in index order
  const double wsum = wave_sum_f64(my_cost);
  if (lane == 0) wcost[wave] = wsum;
  __syncthreads();
  if (tid == 0 && a.cost_slab) {
    double tot = 0.0;
    for (int w = 0; w < kWaves; ++w) tot += wcost[w];
    a.cost_slab[blockIdx.x] = tot;
  }
  if (lds_acc && accumulate) {
    if (a.sums_too)
      for (int i = tid; i < k * d; i += kThreads) {
        const int b = i / d, f = i - b * d;
        u64 v = acc_l[b * (d | 1) + f];
        if (v) atomicAdd(&a.sums[i], v);
      }
    for (int i = tid; i < k; i += kThreads) {
      u64 v = cnt_l[i];
      if (v) atomicAdd(&a.counts[i], v);
    }
  }
}

// Generic fallback (d > 128 or too many centroids for LDS): one thread per row, VALU distances.
__global__ __launch_bounds__(256) void oap_kmeans_assign_generic(KMeansAssignArgs a, int dp) {
  __shared__ double wsum[4];
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  double my_cost = 0.0;
  for (int64_t row = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; row < a.n; row += stride) {
    const float* xr = a.x + row * a.ld;
    float best = INFINITY;
    int bidx = 0;
    for (int c = 0; c < a.k; ++c) {
      const float* cr = a.centers + size_t(c) * dp;
      float acc = 0.f;
      for (int f = 0; f < a.d; ++f) {
        float df = xr[f] - cr[f];
        acc = fmaf(df, df, acc);
      }
      if (acc < best) {
        best = acc;
        bidx = c;
      }
    }
    if (a.merge) {
      if (best < a.mindist[row]) {
        a.mindist[row] = best;
        a.labels[row] = a.base + bidx;
      }
    } else {
      if (a.labels) a.labels[row] = a.base + bidx;
      if (a.mindist) a.mindist[row] = best;
    }
    my_cost += double(best);
    if (a.accumulate && !a.merge) {
      atomicAdd(&a.counts[bidx], 1ull);
      for (int f = 0; a.sums_too && f < a.d; ++f) {
        long long q = static_cast<long long>(rintf(xr[f] * a.scale[f]));
        atomicAdd(&a.sums[size_t(bidx) * a.d + f], static_cast<u64>(q));
      }
    }
  }
  double v = wave_sum_f64(my_cost);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0 && a.cost_slab) {
    double t = 0.0;
    for (int w = 0; w < int(blockDim.x / 64); ++w) t += wsum[w];
    a.cost_slab[blockIdx.x] = t;
  }
}

__global__ void oap_kmeans_accumulate(const float* x, int64_t n, int ld, int d,
                                      const int32_t* labels, int k, const float* scale, u64* sums,
                                      u64* counts) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n * d; i += stride) {
    int64_t row = i / d;
    int f = static_cast<int>(i - row * d);
    int b = labels[row];
    if (b < 0 || b >= k) continue;
    if (f == 0) atomicAdd(&counts[b], 1ull);
    if (!sums) continue;
    long long q = static_cast<long long>(rintf(x[row * ld + f] * scale[f]));
    atomicAdd(&sums[size_t(b) * d + f], static_cast<u64>(q));
  }
}

__global__ __launch_bounds__(256) void oap_kmeans_finalize(KMeansFinalizeArgs a) {
  __shared__ int s_conv, s_nonempty;
  __shared__ double s_shift[256];
  __shared__ float s_norm[256];
  if (threadIdx.x == 0) {
    s_conv = 1;
    s_nonempty = 0;
  }
  __syncthreads();
  double my_max = 0.0;
  float my_nmax = 0.f;
  for (int c = threadIdx.x; c < a.k; c += blockDim.x) {
    const long long cntv = static_cast<long long>(a.counts[c]);
    double* c64 = a.centers64 + size_t(c) * a.d;
    double shift2 = 0.0, nrm = 0.0;
    if (cntv > 0) {
      atomicAdd(&s_nonempty, 1);
      for (int f = 0; f < a.d; ++f) {
        long long sv = static_cast<long long>(a.sums[size_t(c) * a.d + f]);
        double nv = double(sv) * a.inv_scale[f] / double(cntv);  // same formula as the CPU engine
        double df = nv - c64[f];
        shift2 += df * df;
        c64[f] = nv;
      }
      if (shift2 > a.tol * a.tol) atomicAnd(&s_conv, 0);
      if (shift2 > my_max) my_max = shift2;
    }
    for (int f = 0; f < a.d; ++f) {
      float v = static_cast<float>(c64[f]);
      a.centers32[size_t(c) * a.dp + f] = v;
      nrm += double(v) * double(v);
    }
    a.cnorm[c] = static_cast<float>(nrm);
    my_nmax = fmaxf(my_nmax, sqrtf(static_cast<float>(nrm)));
  }
  s_shift[threadIdx.x] = my_max;
  s_norm[threadIdx.x] = my_nmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    double mx = 0.0;
    float nm = 0.f;
    for (int i = 0; i < int(blockDim.x); ++i) {
      mx = fmax(mx, s_shift[i]);
      nm = fmaxf(nm, s_norm[i]);
    }
    KMeansFlags* fl = static_cast<KMeansFlags*>(a.flags);
    fl->converged = s_conv;
    fl->nonempty = s_nonempty;
    fl->cost = a.cost_in ? a.cost_in[0] : 0.0;
    fl->max_shift2 = mx;
    if (a.cstat) a.cstat[0] = nm * 1.0000001f;
  }
}

__global__ void oap_kmeans_prepare_centers(const double* c64, int k, int d, int dp, float* c32,
                                           float* cnorm, float* cstat, int kpad) {
  __shared__ float s_norm[256];
  float nmax = 0.f;
  for (int c = threadIdx.x; c < kpad; c += blockDim.x) {
    if (c >= k) {
      cnorm[c] = INFINITY;
      for (int f = 0; f < dp; ++f) c32[size_t(c) * dp + f] = 0.f;
      continue;
    }
    double nrm = 0.0;
    for (int f = 0; f < dp; ++f) {
      float v = f < d ? static_cast<float>(c64[size_t(c) * d + f]) : 0.f;
      c32[size_t(c) * dp + f] = v;
      nrm += double(v) * double(v);
    }
    cnorm[c] = static_cast<float>(nrm);
    nmax = fmaxf(nmax, sqrtf(static_cast<float>(nrm)));
  }
  s_norm[threadIdx.x] = nmax;
  __syncthreads();
  if (threadIdx.x == 0 && cstat) {
    float m = 0.f;
    for (int i = 0; i < int(blockDim.x); ++i) m = fmaxf(m, s_norm[i]);
    cstat[0] = m * 1.0000001f;
  }
}

template <int KS, bool P>
void launch_mfma(const KMeansAssignArgs& a, int grid, hipStream_t s, bool lds_acc) {
  const Smem L = smem_plan(16 * KS, a.kpad, a.k, a.d, P, lds_acc);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&oap_kmeans_assign_mfma<KS, P>),
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_assign_mfma<KS, P>), dim3(grid), dim3(kThreads), L.total, s, a,
                     lds_acc ? 1 : 0);
  OAP_HIP_CHECK(hipGetLastError());
}

template <bool P>
void dispatch_ks(int ks, const KMeansAssignArgs& a, int grid, hipStream_t s, bool lds_acc) {
  switch (ks) {
    case 1: launch_mfma<1, P>(a, grid, s, lds_acc); break;
    case 2: launch_mfma<2, P>(a, grid, s, lds_acc); break;
    case 3: launch_mfma<3, P>(a, grid, s, lds_acc); break;
    case 4: launch_mfma<4, P>(a, grid, s, lds_acc); break;
    case 5: launch_mfma<5, P>(a, grid, s, lds_acc); break;
    case 6: launch_mfma<6, P>(a, grid, s, lds_acc); break;
    case 7: launch_mfma<7, P>(a, grid, s, lds_acc); break;
    case 8: launch_mfma<8, P>(a, grid, s, lds_acc); break;
    default: OAP_THROW(ConfigError, "kmeans_assign: unsupported KS=" << ks);
  }
}

}  // namespace

// --------------------------------------------------------------------------- host wrappers
int kmeans_ld(int d) { return (d + 3) / 4 * 4; }
int kmeans_dp(int d) { return d <= 128 ? (d + 15) / 16 * 16 : d; }
int kmeans_cost_slab_size(int num_cus) { return num_cus > 8192 ? num_cus : 8192; }

int kmeans_lds_kmax(int d, bool precise) {
  if (d > 128) return 0;
  const int dp = kmeans_dp(d);
  int kp = 32;
  if (smem_plan(dp, kp, 0, d, precise, false).total > kLdsLimit) return 0;
  while (smem_plan(dp, kp + 32, 0, d, precise, false).total <= kLdsLimit) kp += 32;
  return kp;
}

int kmeans_assign(const KMeansAssignArgs& a, int num_cus, hipStream_t s) {
  OAP_CHECK(a.kpad % 32 == 0 && a.kpad >= a.k, "kpad must be a multiple of 32 >= k");
  OAP_CHECK(a.ld == kmeans_ld(a.d), "row stride " << a.ld << " != kmeans_ld(" << a.d << ")");
  OAP_CHECK(!a.merge || (a.labels && a.mindist), "merge mode needs labels and mindist");
  if (a.n == 0) return 0;
  const int dp = kmeans_dp(a.d);
  const bool generic = a.d > 128 || a.kpad > kmeans_lds_kmax(a.d, a.precise);
  if (generic) {
    int grid = grid_for(a.n, 256, 4096);
    hipLaunchKernelGGL(oap_kmeans_assign_generic, dim3(grid), dim3(256), 0, s, a, dp);
    OAP_HIP_CHECK(hipGetLastError());
    return grid;
  }
  const bool acc = a.accumulate && !a.merge;
  const bool lds_acc =
      acc && a.sums_too && smem_plan(dp, a.kpad, a.k, a.d, a.precise, true).total <= kLdsLimit;
  const int64_t tiles = (a.n + 31) / 32;
  const int64_t g = (tiles + kWaves - 1) / kWaves;
  int grid = static_cast<int>(g < num_cus ? g : num_cus);
  if (grid < 1) grid = 1;
  if (a.precise)
    dispatch_ks<true>(dp / 16, a, grid, s, lds_acc);
  else
    dispatch_ks<false>(dp / 16, a, grid, s, lds_acc);
  return grid;
}

void kmeans_accumulate(const float* x, int64_t n, int ld, int d, const int32_t* labels, int k,
                       const float* scale, unsigned long long* sums, unsigned long long* counts,
                       hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(oap_kmeans_accumulate, dim3(grid_for(n * d, 256)), dim3(256), 0, s, x, n, ld,
                     d, labels, k, scale, sums, counts);
  OAP_HIP_CHECK(hipGetLastError());
}

void kmeans_finalize(const KMeansFinalizeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(oap_kmeans_finalize, dim3(1), dim3(256), 0, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

void kmeans_prepare_centers(const double* centers64, int k, int d, int dp, float* centers32,
                            float* cnorm, float* cstat, int kpad, hipStream_t s) {
  hipLaunchKernelGGL(oap_kmeans_prepare_centers, dim3(1), dim3(256), 0, s, centers64, k, d, dp,
                     centers32, cnorm, cstat, kpad);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
