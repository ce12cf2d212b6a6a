// oap_kmeans_wide_t1 — K-Means tier-1 assignment for wide rows (d > 128) on MFMA, gfx950.
//
// The lean kernel (kmeans_lloyd.hip) keeps a 32-row tile's features in registers and the whole
// centroid plane in LDS; past 128 features neither fits.  Here a workgroup of 8 waves (one
// 32-row tile each) walks the features in 128-wide chunks: per chunk the fp16 centroid slice
// (prepared once per iteration by oap_kmeans_wide_prep: -2 alpha c, zero padded) is copied into
// LDS with 16-byte loads, every wave converts its rows' slice to fp16 and accumulates
// v_mfma_f32_32x32x16_f16 products for ALL centroids (k <= 256: 8 accumulator tiles, 128
// AGPR/VGPRs per lane).  A final bias k-step adds alpha^2 (|c|^2 + |x|^2) as hi/lo fp16 pairs,
// exactly as in the lean kernel, so the accumulators end at alpha^2 |x - c|^2; the epilogue's
// integer-key top-2 and the rigorous tier-1 bound decide every row whose runner-up is outside the
// bound and defer the rest to oap_kmeans_wide_exact, which recomputes them with the generic
// kernel's fp32 direct form (identical labels to kmeans.hip's d > 128 path).
// Reference hot loop: oneDAL step1Local (mllib-dal/src/main/native/KMeansDALImpl.cpp:70-77).
#include "kernels/kmeans_wide.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "kernels/device_utils.h"
#include "kernels/kmeans_frag.h"

namespace oap {
namespace kern {

namespace {

using kmdev::med3_i32;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int kWaves = 8, kThreads = 64 * kWaves;
constexpr int kFC = 128;        // features per chunk
constexpr int kSB = kFC + 8;    // LDS row stride (halves): odd 16-byte slot count
constexpr int kMaxK = 256;      // centroids per pass
constexpr float kUnit = 16.f;   // bias features' unit

struct WideArgs {
  const void* x;
  const _Float16* plane;  // [kpad][FC * kFC] fp16 of -2 alpha c (zero padded)
  const _Float16* bias;   // [kpad][16] fp16 bias slots [hi, lo (alpha^2 |c|^2 / 16), 16, 16]
  const float* cstat;     // [0] = max |c|
  int32_t* labels;
  int32_t* defer;
  unsigned* defer_count;
  int64_t n, tiles_per_block;
  int ld, d, k, fc;
};

__device__ inline float wide_alpha(float cmax) {
  const float c = fmaxf(cmax, 1e-30f);
  return exp2f(floorf(log2f(256.f / c)));
}

__device__ inline void split_f16(float v, _Float16& hi, _Float16& lo) {
  hi = static_cast<_Float16>(v);
  lo = static_cast<_Float16>(v - static_cast<float>(hi));
}

// fp16 centroid slices and bias slots for this iteration's centers (c32: [kpad][dp] fp32).
__global__ void oap_kmeans_wide_prep(const float* __restrict__ c32,
                                     const float* __restrict__ cnorm,
                                     const float* __restrict__ cstat, int k, int kpad, int d,
                                     int dp, int fc, _Float16* __restrict__ plane,
                                     _Float16* __restrict__ bias) {
  const float alpha = wide_alpha(cstat[0]);
  const float a2 = alpha * alpha;
  const int64_t w = int64_t(fc) * kFC;
  const int64_t total = int64_t(kpad) * w;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int c = int(i / w), f = int(i - int64_t(c) * w);
    plane[i] = static_cast<_Float16>((c < k && f < d) ? -2.f * alpha * c32[size_t(c) * dp + f]
                                                       : 0.f);
  }
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < int64_t(kpad) * 16;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int c = int(i / 16), f = int(i % 16);
    _Float16 hi, lo;
    // padded centers: the largest finite bias (their distance never wins)
    split_f16(c < k ? a2 * cnorm[c] * (1.f / kUnit) : 60000.f, hi, lo);
    _Float16 v = static_cast<_Float16>(0.f);
    if (f == 0) v = hi;
    if (f == 1) v = lo;
    if (f == 2 || f == 3) v = static_cast<_Float16>(kUnit);
    bias[i] = v;
  }
}

template <bool XB, int NCC>
__global__ __launch_bounds__(kThreads, 1) void oap_kmeans_wide_t1(WideArgs a) {
  constexpr int KP = NCC * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* pl = reinterpret_cast<_Float16*>(smem);  // [KP][kSB]
  _Float16* bl = pl + KP * kSB;                       // [KP][16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int d = a.d, k = a.k;
  const float cmax = a.cstat[0];
  const float alpha = wide_alpha(cmax);
  const float a2 = alpha * alpha;
  const float cm_s = alpha * cmax;
  // tier-1 bound (alpha^2 units), as the lean kernel's: fp16 cross term 4 x 2^-10 |ac||ax|,
  // subnormals and the bias pairs, fp32 accumulation over the longer chain (scaled with d)
  const float dacc = fmaxf(1.f, float(d) / 128.f);
  const float thr_c = 0.0040f * cm_s;
  const float thr_k = 6e-5f * dacc * cm_s * cm_s + float(d) * 6.2e-5f + 1e-30f;
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t T = a.tiles_per_block;
  const int64_t t0 = int64_t(blockIdx.x) * T;
  const int64_t t1 = t0 + T < ntiles ? t0 + T : ntiles;

  for (int i = tid; i < KP * 2; i += kThreads)  // bias slots: 2 x 16-byte per centroid
    reinterpret_cast<uint4*>(bl)[i] = reinterpret_cast<const uint4*>(a.bias)[i];

  for (int64_t tb = t0; tb < t1; tb += kWaves) {
    const int64_t tile = tb + wave;
    const bool live = tile < t1;  // (wave-uniform; dead waves still stage and sync)
    const int64_t row = tile * 32 + r;
    const int64_t rowc = row < a.n ? row : a.n - 1;
    f32x16 acc[NCC];
#pragma unroll
    for (int cc = 0; cc < NCC; ++cc) acc[cc] = f32x16{};
    float nx2 = 0.f;
    for (int fc = 0; fc < a.fc; ++fc) {
      __syncthreads();
      {  // centroid slice fc -> LDS (16-byte copies)
        const _Float16* src = a.plane + size_t(fc) * kFC;
        const int64_t w = int64_t(a.fc) * kFC;
        for (int i = tid; i < KP * (kFC / 8); i += kThreads) {
          const int c = i / (kFC / 8), q = i - c * (kFC / 8);
          *reinterpret_cast<uint4*>(pl + c * kSB + 8 * q) =
              *reinterpret_cast<const uint4*>(src + c * w + 8 * q);
        }
      }
      __syncthreads();
      if (!live) continue;
      f16x8 xh[8];
      const int fb = fc * kFC + 8 * h;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int f = fb + 16 * s;
        float v[8];
        if constexpr (XB) {
          bf16x8 b = bf16x8{};
          const __bf16* xp = static_cast<const __bf16*>(a.x) + rowc * a.ld + f;
          if (f < a.ld) b = *reinterpret_cast<const bf16x8*>(xp);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = static_cast<float>(b[j]);
        } else {
          const float* p = static_cast<const float*>(a.x) + rowc * a.ld + f;
          float4 u0 = make_float4(0.f, 0.f, 0.f, 0.f), u1 = u0;
          if (f < a.ld) u0 = *reinterpret_cast<const float4*>(p);
          if (f + 4 < a.ld) u1 = *reinterpret_cast<const float4*>(p + 4);
          v[0] = u0.x;
          v[1] = u0.y;
          v[2] = u0.z;
          v[3] = u0.w;
          v[4] = u1.x;
          v[5] = u1.y;
          v[6] = u1.z;
          v[7] = u1.w;
        }
        f16x8 hv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          nx2 = fmaf(v[j], v[j], nx2);
          hv[j] = static_cast<_Float16>(alpha * v[j]);
        }
        xh[s] = hv;
      }
#pragma unroll
      for (int cc = 0; cc < NCC; ++cc) {
        const _Float16* ap = pl + (cc * 32 + r) * kSB + 8 * h;
#pragma unroll
        for (int s = 0; s < 8; ++s)
          acc[cc] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
              *reinterpret_cast<const f16x8*>(ap + 16 * s), xh[s], acc[cc], 0, 0, 0);
      }
    }
    if (!live) continue;
    nx2 += __shfl_xor(nx2, 32, 64);
    const float nx2_s = a2 * nx2;
    {  // bias k-step: [16, 16, hi, lo (alpha^2 |x|^2 / 16)] against [hi, lo (|c|^2), 16, 16]
      _Float16 nh, nl;
      split_f16(nx2_s * (1.f / kUnit), nh, nl);
      const _Float16 z = static_cast<_Float16>(0.f), u = static_cast<_Float16>(kUnit);
      const f16x8 xb = h == 0 ? f16x8{u, u, nh, nl, z, z, z, z} : f16x8{z, z, z, z, z, z, z, z};
#pragma unroll
      for (int cc = 0; cc < NCC; ++cc)
        acc[cc] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
            *reinterpret_cast<const f16x8*>(bl + (cc * 32 + r) * 16 + 8 * h), xb, acc[cc], 0, 0,
            0);
    }
    // ---- top-2 on integer keys (the lean kernel's epilogue)
    int k1 = 0x7fffffff, k2 = 0x7fffffff;
#pragma unroll
    for (int cc = 0; cc < NCC; ++cc) {
      int q1[4], q2[4];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int off = 8 * (e >> 2) + (e & 3);
        const int key = (__float_as_int(acc[cc][e]) & ~0x3ff) | off;
        const int q = e & 3;
        if (e < 4) {
          q1[q] = key;
          q2[q] = 0x7fffffff;
        } else {
          q2[q] = med3_i32(q1[q], q2[q], key);
          q1[q] = min(q1[q], key);
        }
      }
      auto merge2 = [](int& x1, int& x2, int y1, int y2) {
        x2 = min(max(x1, y1), min(x2, y2));
        x1 = min(x1, y1);
      };
      merge2(q1[0], q2[0], q1[1], q2[1]);
      merge2(q1[2], q2[2], q1[3], q2[3]);
      merge2(q1[0], q2[0], q1[2], q2[2]);
      const int base = 32 * cc + 4 * h;
      const int i1 = q1[0] | base, i2 = q2[0] | base;
      k2 = min(max(k1, i1), min(k2, i2));
      k1 = min(k1, i1);
    }
    const int o1 = __shfl_xor(k1, 32, 64), o2 = __shfl_xor(k2, 32, 64);
    k2 = min(max(k1, o1), min(k2, o2));
    k1 = min(k1, o1);
    const float b1 = __int_as_float(k1 & ~0x3ff), b2 = __int_as_float(k2 & ~0x3ff);
    const float tt = fmaf(thr_c, sqrtf(nx2_s), thr_k) + 5e-5f * nx2_s + 2.5e-4f * fabsf(b2);
    const bool valid = row < a.n;
    const bool unsure = valid && (!(b2 - b1 > tt) || !(nx2_s < 1048576.f) || !(b1 == b1));
    int b = k1 & 0x3ff;
    b = b < k ? b : 0;
    if (valid && h == 0) {
      if (unsure) {
        const unsigned slot = atomicAdd(a.defer_count, 1u);
        a.defer[slot] = static_cast<int32_t>(row);
      } else {
        a.labels[row] = b;
      }
    }
  }
}

// Exact re-decision of the deferred rows: the generic kernel's fp32 direct form (fmaf chain over
// the features in order) and first-minimum ties.  A wave takes kExactRows deferred rows at once
// (their features in LDS, read as broadcasts); lanes own centroids c = lane + 64 m and stream the
// transposed centers (coalesced, L2-resident) once per batch instead of once per row.
constexpr int kExactRows = 8;

template <typename T>
__global__ __launch_bounds__(64) void oap_kmeans_wide_exact(const T* __restrict__ x, int ld, int d,
                                                            const float* __restrict__ ct, int kp,
                                                            int k, const int32_t* __restrict__ rows,
                                                            const unsigned* __restrict__ count,
                                                            int32_t* __restrict__ labels) {
  extern __shared__ float xs[];  // [kExactRows][d]
  const int lane = threadIdx.x;
  const unsigned nrows = *count;
  for (unsigned q0 = blockIdx.x * unsigned(kExactRows); q0 < nrows;
       q0 += gridDim.x * unsigned(kExactRows)) {
    const int nb = int(nrows - q0 < unsigned(kExactRows) ? nrows - q0 : kExactRows);
    __syncthreads();
    for (int rr = 0; rr < kExactRows; ++rr) {
      const int64_t row = rows[q0 + (rr < nb ? rr : 0)];
      for (int f = lane; f < d; f += 64) xs[rr * d + f] = static_cast<float>(x[row * ld + f]);
    }
    __syncthreads();
    float best[kExactRows];
    int bidx[kExactRows];
#pragma unroll
    for (int rr = 0; rr < kExactRows; ++rr) {
      best[rr] = INFINITY;
      bidx[rr] = 0x7fffffff;
    }
    // (centroids ascending per lane: strict < keeps the first minimum)
    for (int c = lane; c < k; c += 64) {
      float acc[kExactRows];
#pragma unroll
      for (int rr = 0; rr < kExactRows; ++rr) acc[rr] = 0.f;
      for (int f = 0; f < d; ++f) {
        const float cf = ct[size_t(f) * kp + c];
#pragma unroll
        for (int rr = 0; rr < kExactRows; ++rr) {
          const float df = xs[rr * d + f] - cf;
          acc[rr] = fmaf(df, df, acc[rr]);
        }
      }
#pragma unroll
      for (int rr = 0; rr < kExactRows; ++rr)
        if (acc[rr] < best[rr]) {
          best[rr] = acc[rr];
          bidx[rr] = c;
        }
    }
#pragma unroll
    for (int rr = 0; rr < kExactRows; ++rr) {
      float bv = best[rr];
      int bi = bidx[rr];
      for (int m = 32; m >= 1; m >>= 1) {  // smallest value, then smallest index
        const float ob = __shfl_xor(bv, m, 64);
        const int oi = __shfl_xor(bi, m, 64);
        if (ob < bv || (ob == bv && oi < bi)) {
          bv = ob;
          bi = oi;
        }
      }
      if (lane == 0 && rr < nb) labels[rows[q0 + rr]] = bi < k ? bi : 0;
    }
  }
}

__global__ void oap_kmeans_wide_transpose(const float* __restrict__ c32, int k, int kp, int d,
                                          int dp, float* __restrict__ ct) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < int64_t(d) * kp;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int f = int(i / kp), c = int(i - int64_t(f) * kp);
    ct[i] = c < k ? c32[size_t(c) * dp + f] : 0.f;
  }
}

// Per-row cost against the labelled center: one wave per row (features over lanes).
template <typename T>
__global__ __launch_bounds__(256) void oap_kmeans_wide_cost(const T* __restrict__ x, int64_t n,
                                                            int ld, int d,
                                                            const float* __restrict__ c32, int dp,
                                                            const int32_t* __restrict__ labels,
                                                            float* __restrict__ mindist,
                                                            double* __restrict__ slab) {
  __shared__ double wsum[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double my = 0.0;
  for (int64_t row = blockIdx.x * 4ll + wave; row < n; row += int64_t(gridDim.x) * 4) {
    const T* xr = x + row * ld;
    const float* cr = c32 + size_t(labels[row]) * dp;
    float part = 0.f;
    for (int f = lane; f < d; f += 64) {
      const float df = static_cast<float>(xr[f]) - cr[f];
      part = fmaf(df, df, part);
    }
    const float rc = wave_sum_f32(part);
    if (lane == 0) {
      my += double(rc);
      if (mindist) mindist[row] = rc;
    }
  }
  if (lane == 0) wsum[wave] = my;
  __syncthreads();
  if (threadIdx.x == 0) slab[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

template <bool XB, int NCC>
void launch_wide(const WideArgs& w, int grid, hipStream_t s) {
  const size_t lds = sizeof(_Float16) * (size_t(NCC) * 32 * kSB + size_t(NCC) * 32 * 16);
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(
        hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_wide_t1<XB, NCC>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((oap_kmeans_wide_t1<XB, NCC>), dim3(grid), dim3(kThreads), lds, s, w);
  OAP_HIP_CHECK(hipGetLastError());
}

template <bool XB>
void launch_wide_xb(const WideArgs& w, int ncc, int grid, hipStream_t s) {
  switch (ncc) {
    case 1: launch_wide<XB, 1>(w, grid, s); break;
    case 2: launch_wide<XB, 2>(w, grid, s); break;
    case 3: launch_wide<XB, 3>(w, grid, s); break;
    case 4: launch_wide<XB, 4>(w, grid, s); break;
    case 5: launch_wide<XB, 5>(w, grid, s); break;
    case 6: launch_wide<XB, 6>(w, grid, s); break;
    case 7: launch_wide<XB, 7>(w, grid, s); break;
    default: launch_wide<XB, 8>(w, grid, s); break;
  }
}

}  // namespace

bool kmeans_wide_supported(int d, int k) { return d > 128 && d <= 4096 && k >= 1 && k <= kMaxK; }

void kmeans_wide_assign(const KMeansAssignArgs& a, int num_cus, int32_t* defer,
                        unsigned* defer_count, hipStream_t s) {
  OAP_CHECK(kmeans_wide_supported(a.d, a.k) && a.labels && a.kpad >= a.k && a.kpad % 32 == 0,
            "kmeans_wide_assign: unsupported shape d=" << a.d << " k=" << a.k);
  if (a.n == 0) return;
  const int fc = (a.d + kFC - 1) / kFC;
  const int ncc = (a.k + 31) / 32;
  const int dp = kmeans_dp(a.d);
  // per-call scratch: the fp16 plane [ncc*32][fc*128] + bias [ncc*32][16]
  const size_t plane_h = size_t(ncc) * 32 * fc * kFC, bias_h = size_t(ncc) * 32 * 16;
  const size_t ct_f = size_t(a.d) * ncc * 32;  // transposed fp32 centers (exact pass)
  void* scratch = nullptr;
  OAP_HIP_CHECK(hipMallocAsync(&scratch, ct_f * 4 + (plane_h + bias_h) * sizeof(_Float16) + 64,
                               s));
  float* ct = static_cast<float*>(scratch);
  _Float16* plane = reinterpret_cast<_Float16*>(ct + ct_f);
  _Float16* bias = plane + plane_h;
  hipLaunchKernelGGL(oap_kmeans_wide_prep, dim3(grid_for(int64_t(plane_h), 256, 4096)),
                     dim3(256), 0, s, a.centers, a.cnorm, a.cstat, a.k, ncc * 32, a.d, dp, fc,
                     plane, bias);
  OAP_HIP_CHECK(hipGetLastError());
  OAP_HIP_CHECK(hipMemsetAsync(defer_count, 0, sizeof(unsigned), s));
  WideArgs w;
  w.x = a.x;
  w.plane = plane;
  w.bias = bias;
  w.cstat = a.cstat;
  w.labels = a.labels;
  w.defer = defer;
  w.defer_count = defer_count;
  w.n = a.n;
  w.ld = a.ld;
  w.d = a.d;
  w.k = a.k;
  w.fc = fc;
  const int64_t tiles = (a.n + 31) / 32;
  const int64_t grid = std::min<int64_t>((tiles + kWaves - 1) / kWaves, int64_t(num_cus));
  w.tiles_per_block = (tiles + grid - 1) / grid;
  if (a.xbf16)
    launch_wide_xb<true>(w, ncc, int(grid), s);
  else
    launch_wide_xb<false>(w, ncc, int(grid), s);
  // exact re-decision of the deferred rows (the count stays on the device)
  const int kp = ncc * 32;
  hipLaunchKernelGGL(oap_kmeans_wide_transpose, dim3(grid_for(int64_t(a.d) * kp, 256, 4096)),
                     dim3(256), 0, s, a.centers, a.k, kp, a.d, dp, ct);
  const int egrid = int(std::min<int64_t>((a.n + kExactRows - 1) / kExactRows,
                                          int64_t(num_cus) * 16));
  const size_t elds = sizeof(float) * kExactRows * size_t(a.d);
  static bool eattr = false;
  if (!eattr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_wide_exact<float>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    OAP_HIP_CHECK(
        hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_wide_exact<__bf16>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    eattr = true;
  }
  if (a.xbf16)
    hipLaunchKernelGGL(oap_kmeans_wide_exact<__bf16>, dim3(egrid), dim3(64), elds, s,
                       static_cast<const __bf16*>(a.x), a.ld, a.d, ct, kp, a.k, defer,
                       defer_count, a.labels);
  else
    hipLaunchKernelGGL(oap_kmeans_wide_exact<float>, dim3(egrid), dim3(64), elds, s,
                       static_cast<const float*>(a.x), a.ld, a.d, ct, kp, a.k, defer,
                       defer_count, a.labels);
  OAP_HIP_CHECK(hipGetLastError());
  OAP_HIP_CHECK(hipFreeAsync(scratch, s));
}

int kmeans_wide_cost(const KMeansAssignArgs& a, double* slab, int max_blocks, hipStream_t s) {
  if (a.n == 0) return 0;
  const int dp = kmeans_dp(a.d);
  const int grid = int(std::min<int64_t>((a.n + 3) / 4, int64_t(max_blocks)));
  if (a.xbf16)
    hipLaunchKernelGGL(oap_kmeans_wide_cost<__bf16>, dim3(grid), dim3(256), 0, s,
                       static_cast<const __bf16*>(a.x), a.n, a.ld, a.d, a.centers, dp, a.labels,
                       a.mindist, slab);
  else
    hipLaunchKernelGGL(oap_kmeans_wide_cost<float>, dim3(grid), dim3(256), 0, s,
                       static_cast<const float*>(a.x), a.n, a.ld, a.d, a.centers, dp, a.labels,
                       a.mindist, slab);
  OAP_HIP_CHECK(hipGetLastError());
  return grid;
}

}  // namespace kern
}  // namespace oap
