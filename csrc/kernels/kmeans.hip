// K-Means kernels for MI355X (gfx950, CDNA4).
//
// Replaces the oneDAL step1Local/step2Master pair the reference calls per Lloyd iteration
// (mllib-dal/src/main/native/KMeansDALImpl.cpp:70-77 and :101-130).
//
// oap_kmeans_assign_f32<S> — the fused hot kernel (K1):
//   * distance cross-term X·Cᵀ on the matrix cores with v_mfma_f32_32x32x2_f32 (exact fp32,
//     one rounding per product — no TF32-style truncation exists or is used on gfx950);
//     centroids are the A operand (32 centroids per MFMA row block, staged once per block in
//     LDS as two k-half planes with an odd-16B-slot row stride => conflict-free ds_read_b128),
//     data rows are the B operand held in registers (32 rows per wave, S features per lane);
//   * argmin kept in registers: the 32x32 accumulator puts one data row per lane column and 16
//     centroids per lane, so the argmin is a per-lane scan plus one cross-half exchange;
//   * exact per-row cost |x - c_best|^2 re-computed from LDS (no expansion cancellation);
//   * centroid sums accumulated as 64-bit FIXED POINT (x * 2^e_f, e_f per feature chosen from
//     the global column max so the global sum cannot overflow) with ds_add_u64 into an LDS
//     accumulator, flushed once per block with 64-bit integer atomics.  Integer addition is
//     associative, so the sums are bitwise identical for any block schedule, any number of
//     ranks and any RCCL reduction order — the reproducibility property the reference cannot
//     offer (it exchanges fp64 oneDAL archives through a root, KMeansDALImpl.cpp:97-130).
//   * persistent grid (one 512-thread block per CU, 8 waves = 2 per SIMD) walking 32-row tiles
//     with a register prefetch of the next tile.
// oap_kmeans_finalize — K2+K3 fused: new centroids (Spark rule: empty clusters keep their
//   center, mllib/clustering/KMeans.scala:306-330 in the reference's shadow copy) + the
//   tolerance test Σ(Δc)² <= tol² evaluated redundantly on every rank (no broadcast, C5).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "kernels/kernels.h"

namespace oap {
namespace kern {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned long long u64;

constexpr int kThreads = 512;  // 8 waves
constexpr int kWaves = kThreads / 64;

__host__ __device__ inline int plane_ld(int S) {
  int l = (S + 3) / 4 * 4;
  if (((l / 4) & 1) == 0) l += 4;  // odd number of 16-B slots per row -> conflict-free b128
  return l;
}

__device__ inline float shfl_xor_f(float v, int m) { return __shfl_xor(v, m, 64); }
__device__ inline int shfl_xor_i(int v, int m) { return __shfl_xor(v, m, 64); }

__device__ inline double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// LDS carve for the fused assign kernel.
struct AssignSmem {
  size_t planes, cn, acc, cnt, wcost, total;
};
__host__ __device__ inline AssignSmem assign_smem(int S, int kpad, int k, int d, bool lds_acc) {
  AssignSmem m;
  size_t off = 0;
  m.planes = off;
  off += size_t(2) * kpad * plane_ld(S) * sizeof(float);
  m.cn = off;
  off += size_t(kpad) * sizeof(float);
  off = (off + 15) / 16 * 16;
  m.acc = off;
  if (lds_acc) off += size_t(k) * d * sizeof(u64);
  m.cnt = off;
  if (lds_acc) off += size_t(k) * sizeof(u64);
  off = (off + 15) / 16 * 16;
  m.wcost = off;
  off += kWaves * sizeof(double);
  m.total = (off + 15) / 16 * 16;
  return m;
}

constexpr size_t kLdsLimit = 160 * 1024;

template <int S>
__global__ __launch_bounds__(kThreads, 2) void oap_kmeans_assign_f32(KMeansAssignArgs a,
                                                                      int lds_acc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int kpad = a.kpad, k = a.k, d = a.d;
  const int ldc = plane_ld(S);
  const AssignSmem L = assign_smem(S, kpad, k, d, lds_acc != 0);
  float* planes = reinterpret_cast<float*>(smem + L.planes);
  float* cn = reinterpret_cast<float*>(smem + L.cn);
  u64* acc = reinterpret_cast<u64*>(smem + L.acc);
  u64* cnt = reinterpret_cast<u64*>(smem + L.cnt);
  double* wcost = reinterpret_cast<double*>(smem + L.wcost);

  const int tid = threadIdx.x;
  // ---- stage centroids into the two k-half planes: plane h row c holds C[c][h*S + s].
  for (int idx = tid; idx < kpad * 2 * S; idx += kThreads) {
    int c = idx / (2 * S), f = idx - c * (2 * S);
    int h = f / S, s = f - h * S;
    float v = (c < k && f < d) ? a.centers[size_t(c) * d + f] : 0.f;
    planes[(size_t(h) * kpad + c) * ldc + s] = v;
  }
  for (int c = tid; c < kpad; c += kThreads) cn[c] = (c < k) ? a.cnorm[c] : INFINITY;
  if (lds_acc && a.accumulate) {
    for (int i = tid; i < k * d; i += kThreads) acc[i] = 0ull;
    for (int i = tid; i < k; i += kThreads) cnt[i] = 0ull;
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int fbase = h * S;

  float sc[S];
#pragma unroll
  for (int s = 0; s < S; ++s)
    sc[s] = (a.accumulate && a.sums_too && fbase + s < d) ? a.scale[fbase + s] : 0.f;

  double my_cost = 0.0;
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t stride = int64_t(gridDim.x) * kWaves;
  int64_t t = int64_t(blockIdx.x) * kWaves + wave;

  float xn[S];
  auto load_tile = [&](int64_t tt, float* dst) {
    int64_t row = tt * 32 + j;
    if (tt < ntiles && row < a.n) {
      const float2* p = reinterpret_cast<const float2*>(a.x + row * a.ld + fbase);
#pragma unroll
      for (int s = 0; s < S / 2; ++s) {
        float2 v = p[s];
        dst[2 * s] = v.x;
        dst[2 * s + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int s = 0; s < S; ++s) dst[s] = 0.f;
    }
  };
  load_tile(t, xn);

  for (; t < ntiles; t += stride) {
    float x[S];
#pragma unroll
    for (int s = 0; s < S; ++s) x[s] = xn[s];
    const int64_t row = t * 32 + j;
    const bool valid = row < a.n;
    load_tile(t + stride, xn);  // prefetch: hidden behind kpad/32 * S MFMAs

    float best = INFINITY;
    int bidx = 0x7fffffff;
    for (int c0 = 0; c0 < kpad; c0 += 32) {
      f32x16 accv = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                     0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const float* cp = planes + (size_t(h) * kpad + c0 + j) * ldc;
#pragma unroll
      for (int s = 0; s + 3 < S; s += 4) {
        float4 a4 = *reinterpret_cast<const float4*>(cp + s);
        accv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, x[s], accv, 0, 0, 0);
        accv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, x[s + 1], accv, 0, 0, 0);
        accv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, x[s + 2], accv, 0, 0, 0);
        accv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, x[s + 3], accv, 0, 0, 0);
      }
      if constexpr (S % 4 == 2) {
        float2 a2 = *reinterpret_cast<const float2*>(cp + (S - 2));
        accv = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.x, x[S - 2], accv, 0, 0, 0);
        accv = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.y, x[S - 1], accv, 0, 0, 0);
      }
      // accumulator element r: centroid c0 + (r&3) + 8*(r>>2) + 4*h, data row j.
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float4 c4 = *reinterpret_cast<const float4*>(cn + c0 + 8 * g + 4 * h);
        float cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float dist = fmaf(-2.f, accv[4 * g + q], cv[q]);
          int ci = c0 + 8 * g + 4 * h + q;
          if (dist < best) {
            best = dist;
            bidx = ci;
          }
        }
      }
    }
    // combine the two lane halves (complementary centroid subsets of the same row)
    {
      float ob = shfl_xor_f(best, 32);
      int oi = shfl_xor_i(bidx, 32);
      if (ob < best || (ob == best && oi < bidx)) {
        best = ob;
        bidx = oi;
      }
    }
    if (bidx >= k) bidx = 0;  // only reachable for degenerate (NaN) inputs
    // exact squared distance to the chosen center
    float part = 0.f;
    {
      const float* cb = planes + (size_t(h) * kpad + bidx) * ldc;
#pragma unroll
      for (int s = 0; s + 3 < S; s += 4) {
        float4 c4 = *reinterpret_cast<const float4*>(cb + s);
        float d0 = x[s] - c4.x, d1 = x[s + 1] - c4.y, d2 = x[s + 2] - c4.z, d3 = x[s + 3] - c4.w;
        part = fmaf(d0, d0, part);
        part = fmaf(d1, d1, part);
        part = fmaf(d2, d2, part);
        part = fmaf(d3, d3, part);
      }
      if constexpr (S % 4 == 2) {
        float2 c2 = *reinterpret_cast<const float2*>(cb + (S - 2));
        float d0 = x[S - 2] - c2.x, d1 = x[S - 1] - c2.y;
        part = fmaf(d0, d0, part);
        part = fmaf(d1, d1, part);
      }
    }
    float rowcost = part + shfl_xor_f(part, 32);
    const float w = (a.weights && valid) ? a.weights[row] : 1.f;
    if (valid) {
      if (h == 0) {
        if (a.labels) a.labels[row] = bidx;
        if (a.mindist) a.mindist[row] = rowcost;
        my_cost += double(rowcost) * double(w);
      }
      if (a.accumulate) {
        if (lds_acc) {
          if (h == 0) atomicAdd(&cnt[bidx], 1ull);
          u64* ap = acc + size_t(bidx) * d + fbase;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            if (a.sums_too && fbase + s < d) {
              long long q = static_cast<long long>(rintf(x[s] * sc[s]));
              atomicAdd(ap + s, static_cast<u64>(q));
            }
          }
        } else {
          if (h == 0) atomicAdd(&a.counts[bidx], 1ull);
          u64* ap = a.sums + size_t(bidx) * d + fbase;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            if (a.sums_too && fbase + s < d) {
              long long q = static_cast<long long>(rintf(x[s] * sc[s]));
              atomicAdd(ap + s, static_cast<u64>(q));
            }
          }
        }
      }
    }
  }

  // ---- deterministic per-block cost: fixed shuffle tree, then waves in index order
  double wsum = wave_sum_f64(my_cost);
  if (lane == 0) wcost[wave] = wsum;
  __syncthreads();
  if (tid == 0 && a.cost_slab) {
    double tot = 0.0;
    for (int w = 0; w < kWaves; ++w) tot += wcost[w];
    a.cost_slab[blockIdx.x] = tot;
  }
  if (lds_acc && a.accumulate) {
    if (a.sums_too)
      for (int i = tid; i < k * d; i += kThreads) {
        u64 v = acc[i];
        if (v) atomicAdd(&a.sums[i], v);
      }
    for (int i = tid; i < k; i += kThreads) {
      u64 v = cnt[i];
      if (v) atomicAdd(&a.counts[i], v);
    }
  }
}

// Generic fallback (d > 128): one thread per row, VALU distances, global atomics.
__global__ __launch_bounds__(256) void oap_kmeans_assign_generic(KMeansAssignArgs a) {
  __shared__ double wsum[4];
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  double my_cost = 0.0;
  for (int64_t row = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; row < a.n; row += stride) {
    const float* xr = a.x + row * a.ld;
    float best = INFINITY;
    int bidx = 0;
    for (int c = 0; c < a.k; ++c) {
      const float* cr = a.centers + size_t(c) * a.d;
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
    const float w = a.weights ? a.weights[row] : 1.f;
    if (a.labels) a.labels[row] = bidx;
    if (a.mindist) a.mindist[row] = best;
    my_cost += double(best) * w;
    if (a.accumulate) {
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

__global__ void oap_sum_f64(const double* in, int m, double* out) {
  // single wave, fixed order: lane-strided partials then a fixed shuffle tree
  double v = 0.0;
  for (int i = threadIdx.x; i < m; i += 64) v += in[i];
  v = wave_sum_f64(v);
  if (threadIdx.x == 0) out[0] = v;
}

__global__ __launch_bounds__(256) void oap_kmeans_finalize(KMeansFinalizeArgs a) {
  __shared__ int s_conv, s_nonempty;
  __shared__ double s_shift[256];
  if (threadIdx.x == 0) {
    s_conv = 1;
    s_nonempty = 0;
  }
  __syncthreads();
  double my_max = 0.0;
  for (int c = threadIdx.x; c < a.k; c += blockDim.x) {
    long long cntv = static_cast<long long>(a.counts[c]);
    double* c64 = a.centers64 + size_t(c) * a.d;
    double shift2 = 0.0, nrm = 0.0;
    if (cntv > 0) {
      atomicAdd(&s_nonempty, 1);
      double inv_n = 1.0 / double(cntv);
      for (int f = 0; f < a.d; ++f) {
        long long sv = static_cast<long long>(a.sums[size_t(c) * a.d + f]);
        double nv = double(sv) * a.inv_scale[f] * inv_n;
        double df = nv - c64[f];
        shift2 += df * df;
        c64[f] = nv;
      }
      if (shift2 > a.tol * a.tol) atomicAnd(&s_conv, 0);
      if (shift2 > my_max) my_max = shift2;
    }
    for (int f = 0; f < a.d; ++f) {
      float v = static_cast<float>(c64[f]);
      a.centers32[size_t(c) * a.d + f] = v;
      nrm += double(v) * double(v);
    }
    a.cnorm[c] = static_cast<float>(nrm);
  }
  s_shift[threadIdx.x] = my_max;
  __syncthreads();
  if (threadIdx.x == 0) {
    double mx = 0.0;
    for (int i = 0; i < int(blockDim.x); ++i) mx = fmax(mx, s_shift[i]);
    KMeansFlags* fl = static_cast<KMeansFlags*>(a.flags);
    fl->converged = s_conv;
    fl->nonempty = s_nonempty;
    fl->cost = a.cost_in ? a.cost_in[0] : 0.0;
    fl->max_shift2 = mx;
  }
}

__global__ void oap_kmeans_prepare_centers(const double* c64, int k, int d, float* c32,
                                           float* cnorm, int kpad) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= kpad) return;
  if (c >= k) {
    cnorm[c] = INFINITY;
    return;
  }
  double nrm = 0.0;
  for (int f = 0; f < d; ++f) {
    float v = static_cast<float>(c64[size_t(c) * d + f]);
    c32[size_t(c) * d + f] = v;
    nrm += double(v) * double(v);
  }
  cnorm[c] = static_cast<float>(nrm);
}

// ----------------------------------------------------------------------------- ingestion
template <typename Src, typename Dst>
__device__ inline Dst cvt(Src v);
template <>
__device__ inline float cvt<double, float>(double v) {
  return static_cast<float>(v);
}
template <>
__device__ inline float cvt<float, float>(float v) {
  return v;
}
template <>
__device__ inline __hip_bfloat16 cvt<double, __hip_bfloat16>(double v) {
  return __float2bfloat16(static_cast<float>(v));
}
template <>
__device__ inline __hip_bfloat16 cvt<float, __hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}

template <typename Src, typename Dst>
__global__ void oap_convert_pad(const Src* src, int64_t rows, int cols, int64_t src_ld, Dst* dst,
                                int64_t dst_ld) {
  int64_t total = rows * dst_ld;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = i / dst_ld;
    int c = static_cast<int>(i - r * dst_ld);
    Dst v = cvt<Src, Dst>(Src(0));
    if (c < cols) v = cvt<Src, Dst>(src[r * src_ld + c]);
    dst[i] = v;
  }
}

__global__ void oap_column_absmax(const float* x, int64_t rows, int cols, int64_t ld,
                                  float* out) {
  // block handles a strip of rows; each thread a column subset; atomicMax on int bits (>=0)
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    float m = 0.f;
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) m = fmaxf(m, fabsf(x[r * ld + c]));
    atomicMax(reinterpret_cast<int*>(out) + c, __float_as_int(m));
  }
}

__device__ inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ inline float u01(uint64_t h) {  // [0,1) with 24 random bits
  return static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
}

__global__ void oap_synth_blobs(float* x, int64_t rows, int cols, int64_t ld, int64_t row0,
                                int ncenters, float box, float sigma, uint64_t seed) {
  int64_t total = rows * ld;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = i / ld;
    int c = static_cast<int>(i - r * ld);
    if (c >= cols) {
      x[i] = 0.f;
      continue;
    }
    int64_t grow = row0 + r;
    uint64_t lab = splitmix64(seed ^ (uint64_t(grow) * 0x2545F4914F6CDD1Dull)) % uint64_t(ncenters);
    uint64_t hc = splitmix64(seed * 31ull + lab * 1315423911ull + uint64_t(c) * 2654435761ull);
    float center = (u01(hc) * 2.f - 1.f) * box;
    uint64_t h1 = splitmix64(seed ^ 0xABCDEFull ^ (uint64_t(grow) << 20) ^ uint64_t(c));
    uint64_t h2 = splitmix64(h1);
    float u1 = fmaxf(u01(h1), 1e-7f), u2 = u01(h2);
    float gauss = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    x[i] = center + sigma * gauss;
  }
}

__global__ void oap_elementwise_min(float* acc, const float* v, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    acc[i] = fminf(acc[i], v[i]);
}

__global__ void oap_bernoulli_select(const float* cost, int64_t n, int64_t row0, double factor,
                                     uint64_t seed, int step, int32_t* flag) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    uint64_t hsh = splitmix64(seed ^ (uint64_t(step) << 48) ^ uint64_t(row0 + i));
    double u = double(hsh >> 11) * (1.0 / 9007199254740992.0);
    flag[i] = (u < factor * double(cost[i])) ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void oap_reduce_sum_f32(const float* v, int64_t n,
                                                          double* slab) {
  __shared__ double ws[4];
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    acc += double(v[i]);
  acc = wave_sum_f64(acc);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) slab[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void oap_gather_rows(const float* x, int64_t ld, int cols, const int64_t* idx,
                                int64_t m, float* out) {
  int64_t total = m * cols;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = i / cols;
    int c = static_cast<int>(i - r * cols);
    out[i] = x[idx[r] * ld + c];
  }
}

__global__ void oap_compact_flags(const int32_t* flag, int64_t n, int64_t* out,
                                  unsigned long long* counter) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    if (flag[i]) out[atomicAdd(counter, 1ull)] = i;
}

inline int grid_for(int64_t n, int block) {
  int64_t g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

template <int S>
void launch_assign_s(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  bool lds_acc = a.accumulate && a.sums_too &&
                 assign_smem(S, a.kpad, a.k, a.d, true).total <= kLdsLimit;
  AssignSmem L = assign_smem(S, a.kpad, a.k, a.d, lds_acc);
  if (L.total > kLdsLimit) {
    // centroid planes alone do not fit: caller should have used the generic kernel
    OAP_THROW(ConfigError, "kmeans_assign: k=" << a.k << " d=" << a.d
                                                << " exceeds the LDS plane budget");
  }
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_assign_f32<S>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL(oap_kmeans_assign_f32<S>, dim3(grid), dim3(kThreads), L.total, s, a,
                     lds_acc ? 1 : 0);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace

// --------------------------------------------------------------------------- host wrappers
int kmeans_ld(int d) {
  int S = (d + 1) / 2;
  S = (S + 1) / 2 * 2;  // even, so the upper half starts 8-B aligned
  if (S <= 32) return 2 * (S < 2 ? 2 : S);
  if (S <= 64) return 2 * ((S + 7) / 8 * 8);
  return (d + 3) / 4 * 4;  // generic kernel
}

int kmeans_cost_slab_size(int num_cus) { return num_cus > 8192 ? num_cus : 8192; }

int kmeans_assign(const KMeansAssignArgs& a, int num_cus, hipStream_t s) {
  OAP_CHECK(a.kpad % 32 == 0 && a.kpad >= a.k, "kpad must be a multiple of 32 >= k");
  OAP_CHECK(a.ld == kmeans_ld(a.d), "row stride " << a.ld << " != kmeans_ld(" << a.d << ")");
  if (a.n == 0) return 0;
  const int S = a.ld / 2;
  bool generic = a.d > 128 || assign_smem(S, a.kpad, a.k, a.d, false).total > kLdsLimit;
  if (generic) {
    int grid = grid_for(a.n, 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(oap_kmeans_assign_generic, dim3(grid), dim3(256), 0, s, a);
    OAP_HIP_CHECK(hipGetLastError());
    return grid;
  }
  int64_t tiles = (a.n + 31) / 32;
  int64_t g = (tiles + kWaves - 1) / kWaves;
  int grid = static_cast<int>(g < num_cus ? g : num_cus);
  if (grid < 1) grid = 1;
  switch (S) {
#define OAP_CASE(SV) \
  case SV: launch_assign_s<SV>(a, grid, s); break;
    OAP_CASE(2) OAP_CASE(4) OAP_CASE(6) OAP_CASE(8) OAP_CASE(10) OAP_CASE(12) OAP_CASE(14)
    OAP_CASE(16) OAP_CASE(18) OAP_CASE(20) OAP_CASE(22) OAP_CASE(24) OAP_CASE(26) OAP_CASE(28)
    OAP_CASE(30) OAP_CASE(32) OAP_CASE(40) OAP_CASE(48) OAP_CASE(56) OAP_CASE(64)
#undef OAP_CASE
    default: OAP_THROW(ConfigError, "kmeans_assign: unsupported S=" << S);
  }
  return grid;
}

void kmeans_finalize(const KMeansFinalizeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(oap_kmeans_finalize, dim3(1), dim3(256), 0, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

void sum_f64(const double* in, int m, double* out, hipStream_t s) {
  hipLaunchKernelGGL(oap_sum_f64, dim3(1), dim3(64), 0, s, in, m, out);
  OAP_HIP_CHECK(hipGetLastError());
}

void kmeans_prepare_centers(const double* centers64, int k, int d, float* centers32, float* cnorm,
                            int kpad, hipStream_t s) {
  int grid = (kpad + 255) / 256;
  hipLaunchKernelGGL(oap_kmeans_prepare_centers, dim3(grid), dim3(256), 0, s, centers64, k, d,
                     centers32, cnorm, kpad);
  OAP_HIP_CHECK(hipGetLastError());
}

void convert_pad(const void* src, DType src_t, int64_t rows, int cols, int64_t src_ld, void* dst,
                 DType dst_t, int64_t dst_ld, hipStream_t s) {
  if (rows == 0) return;
  int grid = grid_for(rows * dst_ld, 256);
  if (src_t == DType::F64 && dst_t == DType::F32)
    hipLaunchKernelGGL((oap_convert_pad<double, float>), dim3(grid), dim3(256), 0, s,
                       static_cast<const double*>(src), rows, cols, src_ld,
                       static_cast<float*>(dst), dst_ld);
  else if (src_t == DType::F32 && dst_t == DType::F32)
    hipLaunchKernelGGL((oap_convert_pad<float, float>), dim3(grid), dim3(256), 0, s,
                       static_cast<const float*>(src), rows, cols, src_ld,
                       static_cast<float*>(dst), dst_ld);
  else if (src_t == DType::F64 && dst_t == DType::BF16)
    hipLaunchKernelGGL((oap_convert_pad<double, __hip_bfloat16>), dim3(grid), dim3(256), 0, s,
                       static_cast<const double*>(src), rows, cols, src_ld,
                       static_cast<__hip_bfloat16*>(dst), dst_ld);
  else if (src_t == DType::F32 && dst_t == DType::BF16)
    hipLaunchKernelGGL((oap_convert_pad<float, __hip_bfloat16>), dim3(grid), dim3(256), 0, s,
                       static_cast<const float*>(src), rows, cols, src_ld,
                       static_cast<__hip_bfloat16*>(dst), dst_ld);
  else
    OAP_THROW(ConfigError, "convert_pad: unsupported " << dtype_name(src_t) << " -> "
                                                       << dtype_name(dst_t));
  OAP_HIP_CHECK(hipGetLastError());
}

void column_absmax(const float* x, int64_t rows, int cols, int64_t ld, float* out,
                   hipStream_t s) {
  if (rows == 0) return;
  int grid = static_cast<int>(rows < 2048 ? rows : 2048);
  hipLaunchKernelGGL(oap_column_absmax, dim3(grid), dim3(256), 0, s, x, rows, cols, ld, out);
  OAP_HIP_CHECK(hipGetLastError());
}

void synth_blobs(float* x, int64_t rows, int cols, int64_t ld, int64_t row0, int ncenters,
                 float box, float sigma, uint64_t seed, hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL(oap_synth_blobs, dim3(grid_for(rows * ld, 256)), dim3(256), 0, s, x, rows,
                     cols, ld, row0, ncenters, box, sigma, seed);
  OAP_HIP_CHECK(hipGetLastError());
}

int reduce_sum_f32(const float* v, int64_t n, double* slab, hipStream_t s) {
  int grid = 256;
  hipLaunchKernelGGL(oap_reduce_sum_f32, dim3(grid), dim3(256), 0, s, v, n, slab);
  OAP_HIP_CHECK(hipGetLastError());
  return grid;
}

void gather_rows(const float* x, int64_t ld, int cols, const int64_t* idx, int64_t m, float* out,
                 hipStream_t s) {
  if (m == 0) return;
  hipLaunchKernelGGL(oap_gather_rows, dim3(grid_for(m * cols, 256)), dim3(256), 0, s, x, ld,
                     cols, idx, m, out);
  OAP_HIP_CHECK(hipGetLastError());
}

void compact_flags(const int32_t* flag, int64_t n, int64_t* out_idx, unsigned long long* counter,
                   hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(oap_compact_flags, dim3(grid_for(n, 256)), dim3(256), 0, s, flag, n,
                     out_idx, counter);
  OAP_HIP_CHECK(hipGetLastError());
}

void elementwise_min(float* acc, const float* v, int64_t n, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(oap_elementwise_min, dim3(grid_for(n, 256)), dim3(256), 0, s, acc, v, n);
  OAP_HIP_CHECK(hipGetLastError());
}

void bernoulli_select(const float* cost, int64_t n, int64_t row0, double factor, uint64_t seed,
                      int step, int32_t* flag, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(oap_bernoulli_select, dim3(grid_for(n, 256)), dim3(256), 0, s, cost, n,
                     row0, factor, seed, step, flag);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
