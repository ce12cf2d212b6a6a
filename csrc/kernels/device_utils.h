// Device-side helpers shared by the HIP kernels (wave64 reductions, hashing RNG, bf16 splits).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels/rng.h"

namespace oap {
namespace kern {

// Workgroup barrier that waits for this wave's LDS operations only.  __syncthreads() adds a
// workgroup-scope release fence, which on gfx9-family waitcnt semantics (vmcnt counts loads AND
// stores) drains every outstanding global load — it defeats register prefetch of the next
// chunk's rows across the barrier.  Use this where the barrier only orders LDS traffic.
__device__ inline void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned long long u64;

// The value of lane l ^ 32 (the other half of the wave), as __shfl_xor(v, 32): one
// v_permlane32_swap (a VALU op) instead of an LDS ds_bpermute round trip
// (checked on gfx950 by tools/probes/permlane32_probe.hip).
__device__ inline int xor32_i(int v) {
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (threadIdx.x & 32) ? p[0] : p[1];
}
__device__ inline float xor32_f(float v) { return __int_as_float(xor32_i(__float_as_int(v))); }

__device__ inline double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__device__ inline float wave_sum_f32(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__device__ inline float wave_max_f32(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// x = hi + lo + O(2^-18 |x|): the 2-term bf16 split used by the "bf16x3" MFMA products.
__device__ inline void bf16_split(float x, __bf16& hi, __bf16& lo) {
  hi = static_cast<__bf16>(x);
  lo = static_cast<__bf16>(x - static_cast<float>(hi));
}

inline int grid_for(int64_t n, int block, int cap = 8192) {
  int64_t g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

}  // namespace kern
}  // namespace oap
