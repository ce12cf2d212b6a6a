// Device helpers shared by the K-Means assign kernels (kmeans_assign.hip: the general fused
// kernel; kmeans_lloyd.hip: the lean tier-1 Lloyd kernel).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels/device_utils.h"

namespace oap {
namespace kern {
namespace kmdev {

__host__ __device__ inline size_t round16(size_t v) { return (v + 15) / 16 * 16; }
__host__ __device__ inline int stride_bf16(int dp) { return dp + 8; }  // (dp+8)/8 odd slots
__host__ __device__ inline int stride_f32(int dp) { return dp + 4; }   // (dp+4)/4 odd slots

// Raw buffer resource over [base, base + bytes) (gfx9 dword3 0x00020000).  Loads / stores
// through it at an out-of-range offset read 0 / are dropped by the buffer unit, so a per-lane
// predicate becomes an offset instead of a branch: the instruction is issued on every path,
// the count of vector-memory operations per loop trip stays fixed, and the compiler's wait for
// an older prefetch can stay partial (s_waitcnt vmcnt counts in issue order; a conditional
// store makes it fall back to vmcnt(0) — a wait for this tile's own stores).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kBufOff = 0x80000000u;
__device__ inline __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), static_cast<short>(0),
                                           static_cast<int>(bytes), 0x00020000);
}
__device__ inline void buf_store_b32(__amdgpu_buffer_rsrc_t rs, uint32_t off, int v, bool on) {
  __builtin_amdgcn_raw_buffer_store_b32(v, rs, on ? off : kBufOff, 0, 0);
}
__device__ inline void buf_store_f2(__amdgpu_buffer_rsrc_t rs, uint32_t off, float2 v, bool on) {
  const u32x2 w = {__float_as_uint(v.x), __float_as_uint(v.y)};
  __builtin_amdgcn_raw_buffer_store_b64(w, rs, on ? off : kBufOff, 0, 0);
}
__device__ inline int buf_load_b32(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool on) {
  return __builtin_amdgcn_raw_buffer_load_b32(rs, on ? off : kBufOff, 0, 0);
}

// v_med3_i32 as a pure operation (schedulable: no volatile)
__device__ inline int med3_i32_pure(int a, int b, int c) {
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ inline int med3_i32(int a, int b, int c) {
  int r;
  asm volatile("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// The lane's slice of one 32-row tile: features f = 16s + 8h + j (s < KS, j < 8) of row r.
// f32 tables keep the fp32 values; bf16 tables keep the raw bf16 vectors, which are already
// the MFMA B operand (and exact: bf16 -> fp32 is a shift).
template <int KS, bool XB>
struct Frag;
template <int KS>
struct Frag<KS, false> {
  float v[KS][8];
  __device__ float at(int s, int j) const { return v[s][j]; }
};
template <int KS>
struct Frag<KS, true> {
  bf16x8 v[KS];
  __device__ float at(int s, int j) const { return static_cast<float>(v[s][j]); }
};

// Exact fp32 argmin over kpad centroids for the lane's row (both halves get the result).
template <int KS, class F>
__device__ inline void exact_argmin(const float* __restrict__ cbase, int stride, const F& x,
                                    const float* __restrict__ cn, int kpad, int d, int r, int h,
                                    int& bidx) {
  float best = INFINITY;
  bidx = 0x7fffffff;
  for (int c0 = 0; c0 < kpad; c0 += 32) {
    f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float* cp = cbase + size_t(c0 + r) * stride + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (16 * s + 4 * q < d) {  // wave-uniform: skip all-padding groups
          float4 a4 = *reinterpret_cast<const float4*>(cp + 16 * s + 4 * q);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, x.at(s, 4 * q + 0), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, x.at(s, 4 * q + 1), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, x.at(s, 4 * q + 2), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, x.at(s, 4 * q + 3), acc, 0, 0, 0);
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
  if (ob < best || (ob == best && oi < bidx)) bidx = oi;
}

// ---- Refined tier-1 deferral test (image passes; kmeans_lean_img.hip and kmeans_lloyd.hip's
// image branch, bitwise the same).  The lean kernels' tier-1 bound tt prices the fp16 rounding of
// both operands at its worst case: a cross term 2^-8 beta max|c| |beta x|.  The operand image
// also carries each row's actual rounding residual |e_x| = |fp16(beta x) - beta x| (rounded up)
// in a pad slot (DP - kResidSlotOff: the plane is 0 there, so no product sees it), and every
// workgroup computes 2 r, r = max_c |fp16(-2 beta c) - (-2 beta c)| (plane_resid2).  With T the
// tier-1 value and D the exact alpha^2 distance, for any center c against the pick c1
//   |(D(c) - T(c)) - (D(c1) - T(c1))| <= 2 |e_x| |beta (c - c1)| + 2 r |X| + rest,
//   |beta (c - c1)| <= sqrt(D(c)) + sqrt(D(c1)),   D <= T + tt,   |X| <= |beta x| + |e_x|,
// where rest is tt without its cross term (bias pairs, accumulation, subnormals, key truncation).
// T - 2 |e_x| sqrt(T + tt) increases with T (tt >= 5e-5 |beta x|^2 >> |e_x|^2), so the test at the
// second-best key value b2 covers every other center.  On overlapping blobs (headline) this
// halves the rows the worst-case test defers; only waves holding such a row evaluate it.
constexpr int kResidSlots = 16;   // LDS: per-wave partial maxima (<= 16 waves per workgroup)
constexpr int kResidSlotOff = 5;  // image slot DP - 5 (h = 1 lanes, element 3 of step KS - 1)

// 2 max |fp16(-2 alpha c_f) - (-2 alpha c_f)|_2 over this wave's centers (c = tid, tid + nt, ..;
// each difference is exact in fp32), rounded up; every lane gets the wave's value
__device__ inline float plane_resid2(const float* __restrict__ centers, int dp, int k, int d,
                                     float alpha, int tid, int nt) {
  float m = 0.f;
  for (int c = tid; c < k; c += nt) {
    float e2 = 0.f;
#pragma unroll 8
    for (int f = 0; f < d; ++f) {
      const float p = -2.f * alpha * centers[size_t(c) * dp + f];
      const float e = static_cast<float>(static_cast<_Float16>(p)) - p;
      e2 = fmaf(e, e, e2);
    }
    m = fmaxf(m, e2);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  return 2.f * __builtin_amdgcn_sqrtf(m * 1.0001f) * 1.001f + 1e-30f;
}

// fp16 upper bound of a residual norm given an fp32 upper bound of it
__device__ inline _Float16 resid_f16_norm_up(float nrm) {
  return static_cast<_Float16>(nrm * 1.001f + 6e-8f);
}

// the refined bound (see above): b1 <= b2 the tier-1 keys' values, tt the worst-case bound, rest
// tt without its cross term, nx2 |beta x|^2 (bias pair), exn >= |e_x|, r2 = 2 r
__device__ inline float refined_tt(float b1, float b2, float tt, float rest, float nx2, float exn,
                                   float r2) {
  const float xn = __builtin_amdgcn_sqrtf(nx2) * 1.001f + exn;
  const float s2 = __builtin_amdgcn_sqrtf(fmaxf(b2, 0.f) + tt);
  const float s1 = __builtin_amdgcn_sqrtf(fmaxf(b1, 0.f) * 1.0005f + tt);
  return (2.f * exn * (s1 + s2) + r2 * xn + rest) * 1.0001f;
}

template <int KS>
__device__ inline void load_row8(const float* __restrict__ p, float (&dst)[KS][8]) {
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float4 v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
      dst[s][4 * q + 0] = v.x;
      dst[s][4 * q + 1] = v.y;
      dst[s][4 * q + 2] = v.z;
      dst[s][4 * q + 3] = v.w;
    }
}

}  // namespace kmdev
}  // namespace kern
}  // namespace oap
