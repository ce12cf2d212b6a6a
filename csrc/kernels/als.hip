// Implicit-feedback ALS: per-row normal equations + Cholesky solve, one wave per row.
//
// The numerical spec is Spark's computeFactors (mllib-dal/src/main/scala/org/apache/spark-3.1.1/
// ml/recommendation/ALS.scala:1718-1800): for destination row u with ratings (i, r_ui)
//   A = Y^T Y + sum_i c1 y_i y_i^T + lambda * n_u * I,   c1 = alpha |r_ui|,
//   b = sum_{r_ui > 0} (1 + c1) y_i,                     n_u = #{r_ui > 0},
// solved by Cholesky (CholeskySolver, :757-788).  It replaces the reference's oneDAL
// implicit_als step4Local (native/ALSDALImpl.cpp:301-316).
//
// MI355X mapping: a 64-thread workgroup takes rows from an atomic work queue (power-law row
// lengths balance dynamically).  The rating-weighted Gramian sum_i c1 y_i y_i^T is a small SYRK
// over the row's gathered factors and runs on v_mfma_f32_16x16x4_f32 (exact fp32 products) with
// the lower-triangle 16x16 tiles resident in accumulator registers; b and n_u ride along on the
// VALU.  The assembled matrix goes to LDS (packed lower triangle) for a wave-parallel
// right-looking Cholesky and the two triangular solves.
#include "kernels/device_utils.h"
#include "kernels/kernels.h"
#include "runtime/common.h"

namespace oap {
namespace kern {

namespace {

constexpr int kAlsThreads = 64;

struct SolveArgs {
  const int64_t* rowptr;
  const int32_t* cols;
  const float* vals;
  int64_t nrows;
  const float* src;  // [n_src][ld]
  int ld, r;
  const float* yty;  // [r][r] (implicit) or null
  float alpha, lambda;
  int implicit;
  float* dst;        // [nrows][ld]
  unsigned long long* queue;  // work counter (zeroed before launch)
  unsigned long long* fail;   // rows whose matrix was not positive definite
};

__device__ inline int tri(int i) { return i * (i + 1) / 2; }

template <int NB>
__global__ __launch_bounds__(kAlsThreads) void oap_als_solve(SolveArgs a) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int NT = NB * (NB + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int r = a.r, lane = threadIdx.x;
  float* L = lds;                   // packed lower triangle, r(r+1)/2
  float* bv = lds + tri(r - 1) + r; // r
  const int kk = lane >> 4, c = lane & 15;

  while (true) {
    unsigned long long row_u = 0;
    if (lane == 0) row_u = atomicAdd(a.queue, 1ull);
    const int64_t row = static_cast<int64_t>(__shfl(row_u, 0, 64));
    if (row >= a.nrows) break;
    const int64_t p0 = a.rowptr[row], p1 = a.rowptr[row + 1];

    f4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    float bacc[NB];
#pragma unroll
    for (int f = 0; f < NB; ++f) bacc[f] = 0.f;
    int nexp = 0;
    for (int64_t p = p0; p < p1; p += 4) {
      const int64_t idx = p + kk;
      const bool ok = idx < p1;
      const int item = ok ? a.cols[idx] : 0;
      const float rv = ok ? a.vals[idx] : 0.f;
      float wa, wb;
      if (a.implicit) {
        const float c1 = a.alpha * fabsf(rv);
        wa = c1;
        wb = rv > 0.f ? 1.f + c1 : 0.f;
        nexp += (ok && rv > 0.f && c == 0) ? 1 : 0;
      } else {  // explicit: A += y y^T, b += r y
        wa = ok ? 1.f : 0.f;
        wb = rv;
        nexp += (ok && c == 0) ? 1 : 0;
      }
      const float* yrow = a.src + static_cast<int64_t>(item) * a.ld + c;
      float yv[NB], av[NB];
#pragma unroll
      for (int f = 0; f < NB; ++f) {
        yv[f] = ok ? yrow[16 * f] : 0.f;
        av[f] = wa * yv[f];
        bacc[f] = fmaf(wb, yv[f], bacc[f]);
      }
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[bi], yv[bj], acc[t], 0, 0, 0);
    }
    // reduce b over the 4 rating groups; n_u over the wave
#pragma unroll
    for (int f = 0; f < NB; ++f) {
      bacc[f] += __shfl_xor(bacc[f], 16, 64);
      bacc[f] += __shfl_xor(bacc[f], 32, 64);
    }
    for (int m = 32; m >= 1; m >>= 1) nexp += __shfl_xor(nexp, m, 64);
    const float lam = a.lambda * static_cast<float>(nexp);

    // assemble A (lower) = Gram + YtY + lam I into LDS; tile element (i = 16bi + 4kk + e,
    // j = 16bj + c).  The lane coordinates are laundered so the per-element addresses are not
    // hoisted out of the row loop as hundreds of live registers.
    {
      int lid = lane;
      asm volatile("" : "+v"(lid));
      const int kk = lid >> 4, c = lid & 15;
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 16 * bi + 4 * kk + e, j = 16 * bj + c;
            if (i < r && j <= i) {
              float v = acc[t][e];
              if (a.yty) v += a.yty[i * r + j];
              if (i == j) v += lam;
              L[tri(i) + j] = v;
            }
          }
    }
    if (kk == 0) {
#pragma unroll
      for (int f = 0; f < NB; ++f)
        if (16 * f + c < r) bv[16 * f + c] = bacc[f];
    }
    __syncthreads();

    // right-looking Cholesky on the packed lower triangle
    bool spd = true;
    for (int j = 0; j < r; ++j) {
      const float djj = L[tri(j) + j];
      if (!(djj > 0.f)) {
        spd = false;
        break;
      }
      const float d = sqrtf(djj), inv = 1.f / d;
      __syncthreads();
      for (int i = j + 1 + lane; i < r; i += 64) L[tri(i) + j] *= inv;
      if (lane == 0) L[tri(j) + j] = d;
      __syncthreads();
      const int m = r - j - 1;
      const int cnt = tri(m - 1) + m;  // m(m+1)/2 trailing elements
      for (int t = lane; t < cnt; t += 64) {
        const int ii = static_cast<int>((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
        int i2 = ii;
        if (tri(i2) > t) --i2;
        if (tri(i2 + 1) <= t) ++i2;
        const int k2 = t - tri(i2);
        const int i = j + 1 + i2, k = j + 1 + k2;
        L[tri(i) + k] -= L[tri(i) + j] * L[tri(k) + j];
      }
      __syncthreads();
    }
    float* out = a.dst + row * a.ld;
    if (!spd) {
      if (lane == 0) atomicAdd(a.fail, 1ull);
      for (int i = lane; i < a.ld; i += 64) out[i] = 0.f;
      __syncthreads();
      continue;
    }
    // forward L z = b, backward L^T x = z (in place in bv)
    for (int j = 0; j < r; ++j) {
      const float z = bv[j] / L[tri(j) + j];
      __syncthreads();
      if (lane == 0) bv[j] = z;
      for (int i = j + 1 + lane; i < r; i += 64) bv[i] -= L[tri(i) + j] * z;
      __syncthreads();
    }
    for (int j = r - 1; j >= 0; --j) {
      const float x = bv[j] / L[tri(j) + j];
      __syncthreads();
      if (lane == 0) bv[j] = x;
      for (int i = lane; i < j; i += 64) bv[i] -= L[tri(j) + i] * x;
      __syncthreads();
    }
    for (int i = lane; i < a.ld; i += 64) out[i] = i < r ? bv[i] : 0.f;
    __syncthreads();
  }
}

template <int NB>
void launch_solve(const SolveArgs& a, int grid, hipStream_t s) {
  const size_t lds = (size_t(a.r) * (a.r + 1) / 2 + size_t(a.r)) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_als_solve<NB>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(oap_als_solve<NB>, dim3(grid), dim3(kAlsThreads), lds, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

__global__ void oap_f64_to_f32(const double* in, float* out, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    out[i] = static_cast<float>(in[i]);
}

__global__ void oap_als_init(const int32_t* ids, int64_t n, int r, int ld, uint64_t seed,
                             float* out) {
  for (int64_t row = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; row < n;
       row += int64_t(gridDim.x) * blockDim.x) {
    double nrm = 0.0;
    for (int f = 0; f < r; ++f) {
      const double g = als_init_gaussian(seed, ids[row], f);
      nrm += g * g;
    }
    nrm = sqrt(nrm);
    for (int f = 0; f < ld; ++f)
      out[row * ld + f] = f < r ? static_cast<float>(als_init_gaussian(seed, ids[row], f) / nrm)
                                : 0.f;
  }
}

}  // namespace

int als_max_rank() { return 128; }

void als_solve(const AlsSolveArgs& s, int num_cus, hipStream_t st) {
  OAP_CHECK(s.r >= 1 && s.r <= als_max_rank(), "GPU ALS supports rank <= " << als_max_rank());
  OAP_CHECK(s.ld % 16 == 0 && s.ld >= s.r, "ALS factor stride must be a multiple of 16 >= rank");
  if (s.nrows == 0) return;
  SolveArgs a;
  a.rowptr = s.rowptr;
  a.cols = s.cols;
  a.vals = s.vals;
  a.nrows = s.nrows;
  a.src = s.src;
  a.ld = s.ld;
  a.r = s.r;
  a.yty = s.yty;
  a.alpha = s.alpha;
  a.lambda = s.lambda;
  a.implicit = s.implicit ? 1 : 0;
  a.dst = s.dst;
  a.queue = s.queue;
  a.fail = s.fail;
  OAP_HIP_CHECK(hipMemsetAsync(s.queue, 0, sizeof(unsigned long long), st));
  const size_t lds = (size_t(s.r) * (s.r + 1) / 2 + size_t(s.r)) * sizeof(float);
  const int per_cu = std::max<int>(1, std::min<int>(16, int((160 * 1024) / (lds + 1024))));
  const int grid = static_cast<int>(std::min<int64_t>(s.nrows, int64_t(num_cus) * per_cu));
  switch ((s.r + 15) / 16) {
    case 1: launch_solve<1>(a, grid, st); break;
    case 2: launch_solve<2>(a, grid, st); break;
    case 3: launch_solve<3>(a, grid, st); break;
    case 4: launch_solve<4>(a, grid, st); break;
    case 5: launch_solve<5>(a, grid, st); break;
    case 6: launch_solve<6>(a, grid, st); break;
    case 7: launch_solve<7>(a, grid, st); break;
    default: launch_solve<8>(a, grid, st); break;
  }
}

void f64_to_f32(const double* in, float* out, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(oap_f64_to_f32, dim3(grid_for(n, 256, 1024)), dim3(256), 0, s, in, out, n);
  OAP_HIP_CHECK(hipGetLastError());
}

void als_init_factors(const int32_t* ids, int64_t n, int r, int ld, uint64_t seed, float* out,
                      hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(oap_als_init, dim3(grid_for(n, 64, 4096)), dim3(64), 0, s, ids, n, r, ld,
                     seed, out);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
