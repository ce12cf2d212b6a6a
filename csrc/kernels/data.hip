// Data-movement / utility kernels: ingestion conversion + padding, column statistics, on-device
// synthetic data, deterministic reductions, row gathers and stream compaction.
//
// Ingestion replaces the reference's row-by-row JNI copies into oneDAL tables
// (mllib-dal/src/main/native/OneDAL.cpp:50-60): the host streams raw chunks,
// the device converts dtype and applies the padded row layout the MFMA kernels expect.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cmath>

#include "kernels/device_utils.h"
#include "kernels/kernels.h"

namespace oap {
namespace kern {

namespace {

template <typename Src, typename Dst>
__device__ inline Dst cvt(Src v) {
  return static_cast<Dst>(static_cast<float>(v));
}
template <>
__device__ inline double cvt<double, double>(double v) {
  return v;
}

template <typename Src, typename Dst>
__global__ void oap_convert_pad(const Src* src, int64_t rows, int cols, int64_t src_ld, Dst* dst,
                                int64_t dst_ld) {
  const int64_t total = rows * dst_ld;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = i / dst_ld;
    int c = static_cast<int>(i - r * dst_ld);
    dst[i] = c < cols ? cvt<Src, Dst>(src[r * src_ld + c]) : cvt<Src, Dst>(Src(0));
  }
}

// Column max |x| when ld % 4 == 0: the matrix is read as a flat float4 stream (fully coalesced);
// the thread stride is a multiple of ld/4, so every thread always sees the same 4 columns.
__global__ __launch_bounds__(256) void oap_column_absmax4(const float4* x, int64_t rows,
                                                          int ld4, int cols, float* out) {
  __shared__ float part[256 * 4];
  const int per_block = (256 / ld4) * ld4;  // threads with a fixed column group
  const int t = threadIdx.x;
  float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < per_block) {
    const int cg = t % ld4;
    const int64_t rstride = int64_t(gridDim.x) * (per_block / ld4);
    for (int64_t r = int64_t(blockIdx.x) * (per_block / ld4) + t / ld4; r < rows; r += rstride) {
      const float4 v = x[r * ld4 + cg];
      m.x = fmaxf(m.x, fabsf(v.x));
      m.y = fmaxf(m.y, fabsf(v.y));
      m.z = fmaxf(m.z, fabsf(v.z));
      m.w = fmaxf(m.w, fabsf(v.w));
    }
  }
  part[t * 4 + 0] = m.x;
  part[t * 4 + 1] = m.y;
  part[t * 4 + 2] = m.z;
  part[t * 4 + 3] = m.w;
  __syncthreads();
  for (int c = t; c < ld4 * 4 && c < cols; c += blockDim.x) {
    float mm = 0.f;
    const int cg = c / 4, lane = c % 4;
    for (int i = cg; i < per_block; i += ld4) mm = fmaxf(mm, part[i * 4 + lane]);
    atomicMax(reinterpret_cast<int*>(out) + c, __float_as_int(mm));  // mm >= 0: int order
  }
}

// Per-block fp64 partial sums of |x|^2 over the rows (features < cols), the same flat float4
// stream: K-Means takes the exact cost of its last assignment from its own statistics,
// sum_i |x_i - c|^2 = sum_i |x_i|^2 - 2 c.S + n |c|^2 (drivers/kmeans.cpp), which needs this
// sum once per table.  Squares of fp32 values are exact in fp64; a fixed grid and per-thread row
// order make the partials (summed in order by the caller) deterministic.
__global__ __launch_bounds__(256) void oap_row_sqnorm_partials4(const float4* x, int64_t rows,
                                                               int ld4, int cols, double* part) {
  __shared__ double red[4];
  const int per_block = (256 / ld4) * ld4;
  const int t = threadIdx.x;
  double acc = 0.0;
  if (t < per_block) {
    const int cg = t % ld4, c0 = 4 * cg;
    const double m0 = c0 < cols ? 1.0 : 0.0, m1 = c0 + 1 < cols ? 1.0 : 0.0;
    const double m2 = c0 + 2 < cols ? 1.0 : 0.0, m3 = c0 + 3 < cols ? 1.0 : 0.0;
    const int64_t rstride = int64_t(gridDim.x) * (per_block / ld4);
    for (int64_t r = int64_t(blockIdx.x) * (per_block / ld4) + t / ld4; r < rows; r += rstride) {
      const float4 v = x[r * ld4 + cg];
      const double a = double(v.x), b = double(v.y), c = double(v.z), e = double(v.w);
      acc += (a * a * m0 + b * b * m1) + (c * c * m2 + e * e * m3);
    }
  }
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if ((t & 63) == 0) red[t >> 6] = acc;
  __syncthreads();
  if (t == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// bf16 rows with ld % 8 == 0: the same flat-stream scheme with 16-byte groups of 8 columns.
__global__ __launch_bounds__(256) void oap_column_absmax8_bf16(const bf16x8* x, int64_t rows,
                                                               int ld8, int cols, float* out) {
  __shared__ float part[256 * 8];
  const int per_block = (256 / ld8) * ld8;
  const int t = threadIdx.x;
  float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (t < per_block) {
    const int cg = t % ld8;
    const int64_t rstride = int64_t(gridDim.x) * (per_block / ld8);
    for (int64_t r = int64_t(blockIdx.x) * (per_block / ld8) + t / ld8; r < rows; r += rstride) {
      const bf16x8 v = x[r * ld8 + cg];
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf(static_cast<float>(v[j])));
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[t * 8 + j] = m[j];
  __syncthreads();
  for (int c = t; c < ld8 * 8 && c < cols; c += blockDim.x) {
    float mm = 0.f;
    const int cg = c / 8, lane = c % 8;
    for (int i = cg; i < per_block; i += ld8) mm = fmaxf(mm, part[i * 8 + lane]);
    atomicMax(reinterpret_cast<int*>(out) + c, __float_as_int(mm));  // mm >= 0: int order
  }
}

template <typename T>
__global__ void oap_column_absmax(const T* x, int64_t rows, int cols, int64_t ld, float* out) {
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    float m = 0.f;
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x)
      m = fmaxf(m, fabsf(static_cast<float>(x[r * ld + c])));
    atomicMax(reinterpret_cast<int*>(out) + c, __float_as_int(m));  // m >= 0: int order == float
  }
}

template <typename T>
__global__ void oap_synth_blobs(T* x, int64_t rows, int cols, int64_t ld, int64_t row0,
                                int ncenters, float box, float sigma, uint64_t seed) {
  const int64_t total = rows * ld;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = i / ld;
    int c = static_cast<int>(i - r * ld);
    if (c >= cols) {
      x[i] = static_cast<T>(0.f);
      continue;
    }
    int64_t grow = row0 + r;
    uint64_t lab = splitmix64(seed ^ (uint64_t(grow) * 0x2545F4914F6CDD1Dull)) % uint64_t(ncenters);
    uint64_t hc = splitmix64(seed * 31ull + lab * 1315423911ull + uint64_t(c) * 2654435761ull);
    float center = (u01_24(hc) * 2.f - 1.f) * box;
    uint64_t h1 = splitmix64(seed ^ 0xABCDEFull ^ (uint64_t(grow) << 20) ^ uint64_t(c));
    uint64_t h2 = splitmix64(h1);
    float u1 = fmaxf(u01_24(h1), 1e-7f), u2 = u01_24(h2);
    float gauss = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    x[i] = static_cast<T>(center + sigma * gauss);
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

__global__ void oap_sum_f64(const double* in, int m, double* out) {
  double v = 0.0;  // single wave, fixed order
  for (int i = threadIdx.x; i < m; i += 64) v += in[i];
  v = wave_sum_f64(v);
  if (threadIdx.x == 0) out[0] = v;
}

template <typename T>
__global__ void oap_gather_rows(const T* x, int64_t ld, int cols, const int64_t* idx,
                                int64_t m, float* out) {
  const int64_t total = m * cols;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = i / cols;
    int c = static_cast<int>(i - r * cols);
    out[i] = static_cast<float>(x[idx[r] * ld + c]);
  }
}

__global__ void oap_compact_flags(const int32_t* flag, int64_t n, int64_t* out,
                                  unsigned long long* counter) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    if (flag[i]) out[atomicAdd(counter, 1ull)] = i;
}

template <typename Src, typename Dst>
void launch_convert(const void* src, int64_t rows, int cols, int64_t src_ld, void* dst,
                    int64_t dst_ld, hipStream_t s) {
  hipLaunchKernelGGL((oap_convert_pad<Src, Dst>), dim3(grid_for(rows * dst_ld, 256)), dim3(256), 0,
                     s, static_cast<const Src*>(src), rows, cols, src_ld, static_cast<Dst*>(dst),
                     dst_ld);
}

}  // namespace

void convert_pad(const void* src, DType src_t, int64_t rows, int cols, int64_t src_ld, void* dst,
                 DType dst_t, int64_t dst_ld, hipStream_t s) {
  if (rows == 0) return;
  if (src_t == DType::F64 && dst_t == DType::F32)
    launch_convert<double, float>(src, rows, cols, src_ld, dst, dst_ld, s);
  else if (src_t == DType::F32 && dst_t == DType::F32)
    launch_convert<float, float>(src, rows, cols, src_ld, dst, dst_ld, s);
  else if (src_t == DType::F64 && dst_t == DType::BF16)
    launch_convert<double, __bf16>(src, rows, cols, src_ld, dst, dst_ld, s);
  else if (src_t == DType::F32 && dst_t == DType::BF16)
    launch_convert<float, __bf16>(src, rows, cols, src_ld, dst, dst_ld, s);
  else if (src_t == DType::F64 && dst_t == DType::F64)
    launch_convert<double, double>(src, rows, cols, src_ld, dst, dst_ld, s);
  else if (src_t == DType::F32 && dst_t == DType::F64)
    launch_convert<float, double>(src, rows, cols, src_ld, dst, dst_ld, s);
  else
    OAP_THROW(ConfigError, "convert_pad: unsupported " << dtype_name(src_t) << " -> "
                                                       << dtype_name(dst_t));
  OAP_HIP_CHECK(hipGetLastError());
}

void column_absmax(const void* xv, DType t, int64_t rows, int cols, int64_t ld, float* out,
                   hipStream_t s) {
  if (rows == 0) return;
  OAP_CHECK(t == DType::F32 || t == DType::BF16, "column_absmax: f32 or bf16 rows");
  const bool aligned = (reinterpret_cast<uintptr_t>(xv) & 15) == 0;
  const int grid = static_cast<int>(rows < 2048 ? rows : 2048);
  if (t == DType::BF16) {
    if (ld % 8 == 0 && ld / 8 <= 256 && aligned) {
      hipLaunchKernelGGL(oap_column_absmax8_bf16, dim3(2048), dim3(256), 0, s,
                         static_cast<const bf16x8*>(xv), rows, static_cast<int>(ld / 8), cols,
                         out);
    } else {
      hipLaunchKernelGGL(oap_column_absmax<__bf16>, dim3(grid), dim3(256), 0, s,
                         static_cast<const __bf16*>(xv), rows, cols, ld, out);
    }
    OAP_HIP_CHECK(hipGetLastError());
    return;
  }
  const float* x = static_cast<const float*>(xv);
  if (ld % 4 == 0 && ld / 4 <= 256 && aligned) {
    hipLaunchKernelGGL(oap_column_absmax4, dim3(2048), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(x), rows, static_cast<int>(ld / 4), cols,
                       out);
    OAP_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(oap_column_absmax<float>, dim3(grid), dim3(256), 0, s, x, rows, cols, ld,
                     out);
  OAP_HIP_CHECK(hipGetLastError());
}

int row_sqnorm_partials(const float* x, int64_t rows, int cols, int64_t ld, double* part,
                        hipStream_t s) {
  const bool aligned = reinterpret_cast<uintptr_t>(x) % 16 == 0;
  if (rows <= 0 || ld % 4 != 0 || ld / 4 > 256 || !aligned) return -1;
  hipLaunchKernelGGL(oap_row_sqnorm_partials4, dim3(kSqnormBlocks), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(x), rows, static_cast<int>(ld / 4), cols,
                     part);
  OAP_HIP_CHECK(hipGetLastError());
  return kSqnormBlocks;
}

void synth_blobs(void* x, DType t, int64_t rows, int cols, int64_t ld, int64_t row0, int ncenters,
                 float box, float sigma, uint64_t seed, hipStream_t s) {
  if (rows == 0) return;
  OAP_CHECK(t == DType::F32 || t == DType::BF16, "synth_blobs: f32 or bf16 rows");
  const dim3 grid(grid_for(rows * ld, 256));
  if (t == DType::BF16)
    hipLaunchKernelGGL(oap_synth_blobs<__bf16>, grid, dim3(256), 0, s, static_cast<__bf16*>(x),
                       rows, cols, ld, row0, ncenters, box, sigma, seed);
  else
    hipLaunchKernelGGL(oap_synth_blobs<float>, grid, dim3(256), 0, s, static_cast<float*>(x),
                       rows, cols, ld, row0, ncenters, box, sigma, seed);
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

int reduce_sum_f32(const float* v, int64_t n, double* slab, hipStream_t s) {
  const int grid = 256;
  hipLaunchKernelGGL(oap_reduce_sum_f32, dim3(grid), dim3(256), 0, s, v, n, slab);
  OAP_HIP_CHECK(hipGetLastError());
  return grid;
}

void sum_f64(const double* in, int m, double* out, hipStream_t s) {
  hipLaunchKernelGGL(oap_sum_f64, dim3(1), dim3(64), 0, s, in, m, out);
  OAP_HIP_CHECK(hipGetLastError());
}

void gather_rows(const void* x, DType t, int64_t ld, int cols, const int64_t* idx, int64_t m,
                 float* out, hipStream_t s) {
  if (m == 0) return;
  const dim3 grid(grid_for(m * cols, 256));
  if (t == DType::BF16)
    hipLaunchKernelGGL(oap_gather_rows<__bf16>, grid, dim3(256), 0, s,
                       static_cast<const __bf16*>(x), ld, cols, idx, m, out);
  else
    hipLaunchKernelGGL(oap_gather_rows<float>, grid, dim3(256), 0, s,
                       static_cast<const float*>(x), ld, cols, idx, m, out);
  OAP_HIP_CHECK(hipGetLastError());
}

void compact_flags(const int32_t* flag, int64_t n, int64_t* out_idx, unsigned long long* counter,
                   hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(oap_compact_flags, dim3(grid_for(n, 256)), dim3(256), 0, s, flag, n,
                     out_idx, counter);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
