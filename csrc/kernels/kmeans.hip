// K-Means support kernels (MI355X / gfx950) and the assign dispatcher.
//
// * kmeans_assign: picks the fused MFMA kernel (kmeans_assign.hip) when d <= 128 and the
//   centroids fit one LDS plan, else the generic VALU kernel below.
// * oap_kmeans_finalize — K2+K3 fused: new centroids from the allreduced
//   fixed-point sums (Spark rule: empty clusters keep their center,
//   spark-3.1.1/mllib/clustering/KMeans.scala:306-330) and the tolerance test Σ(Δc)² <= tol²,
//   evaluated redundantly on every rank — the reference needs a root merge plus a `converged`
//   broadcast for this (KMeansDALImpl.cpp:101-130, :207-214).
// * oap_kmeans_accumulate — label-driven fixed-point accumulation for the chunked large-k path.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "kernels/device_utils.h"
#include "kernels/kmeans_internal.h"

namespace oap {
namespace kern {

namespace {

// Generic fallback (d > 128): one thread per row, VALU distances, global integer atomics.
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
        const float df = xr[f] - cr[f];
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
        const long long q = static_cast<long long>(rintf(xr[f] * a.scale[f]));
        atomicAdd(&a.sums[size_t(bidx) * a.d + f], static_cast<u64>(q));
      }
    }
  }
  const double v = wave_sum_f64(my_cost);
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
    const int64_t row = i / d;
    const int f = static_cast<int>(i - row * d);
    const int b = labels[row];
    if (b < 0 || b >= k) continue;
    if (f == 0) atomicAdd(&counts[b], 1ull);
    if (!sums) continue;
    const long long q = static_cast<long long>(rintf(x[row * ld + f] * scale[f]));
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
        const long long sv = static_cast<long long>(a.sums[size_t(c) * a.d + f]);
        const double nv = double(sv) * a.inv_scale[f] / double(cntv);  // == CPU engine formula
        const double df = nv - c64[f];
        shift2 += df * df;
        c64[f] = nv;
      }
      if (shift2 > a.tol * a.tol) atomicAnd(&s_conv, 0);
      if (shift2 > my_max) my_max = shift2;
    }
    for (int f = 0; f < a.d; ++f) {
      const float v = static_cast<float>(c64[f]);
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
      const float v = f < d ? static_cast<float>(c64[size_t(c) * d + f]) : 0.f;
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

}  // namespace

// --------------------------------------------------------------------------- host wrappers
int kmeans_ld(int d) { return (d + 3) / 4 * 4; }
int kmeans_dp(int d) { return d <= 128 ? (d + 15) / 16 * 16 : d; }
int kmeans_cost_slab_size(int num_cus) { return num_cus > 8192 ? num_cus : 8192; }
int kmeans_lds_kmax(int d, bool precise) { return kmeans_mfma_kmax(d, precise); }

int64_t kmeans_rows_per_block_bound(int64_t n) {
  const int64_t tiles = (n + 31) / 32;
  const int64_t per_wave = (tiles + 2047) / 2048;  // grid >= 256 blocks x 8 waves once busy
  return 256 * (per_wave < 1 ? 1 : per_wave);
}

int kmeans_assign(const KMeansAssignArgs& a, int num_cus, hipStream_t s) {
  OAP_CHECK(a.kpad % 32 == 0 && a.kpad >= a.k, "kpad must be a multiple of 32 >= k");
  OAP_CHECK(a.ld == kmeans_ld(a.d), "row stride " << a.ld << " != kmeans_ld(" << a.d << ")");
  OAP_CHECK(!a.merge || (a.labels && a.mindist), "merge mode needs labels and mindist");
  if (a.n == 0) return 0;
  const int dp = kmeans_dp(a.d);
  const bool generic = a.d > 128 || a.kpad > kmeans_mfma_kmax(a.d, a.precise);
  if (generic) {
    const int grid = grid_for(a.n, 256, 4096);
    hipLaunchKernelGGL(oap_kmeans_assign_generic, dim3(grid), dim3(256), 0, s, a, dp);
    OAP_HIP_CHECK(hipGetLastError());
    return grid;
  }
  const int grid = kmeans_mfma_grid(a.n, num_cus);
  launch_kmeans_assign_mfma(a, grid, s);
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
