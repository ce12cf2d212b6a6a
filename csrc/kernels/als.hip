// Implicit-feedback ALS: per-row normal equations + blocked Cholesky solve, one wave per row.
//
// The numerical spec is Spark's computeFactors (mllib-dal/src/main/scala/org/apache/spark-3.1.1/
// ml/recommendation/ALS.scala:1718-1800): for destination row u with ratings (i, r_ui)
//   A = Y^T Y + sum_i c1 y_i y_i^T + lambda * n_u * I,   c1 = alpha |r_ui|,
//   b = sum_{r_ui > 0} (1 + c1) y_i,                     n_u = #{r_ui > 0},
// solved by Cholesky (CholeskySolver, :757-788).  It replaces the reference's oneDAL
// implicit_als step4Local (native/ALSDALImpl.cpp:301-316).
//
// MI355X mapping (one 64-thread workgroup = one wave per row, rows from an atomic work queue):
//  * Gramian: sum_i c1 y_i y_i^T is a small SYRK over the row's gathered factors on
//    v_mfma_f32_16x16x4_f32 (exact fp32 products), lower 16x16 tiles resident in accumulator
//    registers; b and n_u ride along on the VALU.  Rows longer than `long_len` ratings are split
//    into chunks whose partial (tiles, b, n_u) go to a scratch slab (oap_als_partial) and are
//    summed in chunk order by the solve kernel — power-law rows neither serialise on one wave
//    nor lose determinism.
//  * Long-row chunks (the bulk of a power-law item side) take a split-fp16 Gramian instead:
//    z = sqrt(c1) y S (S a power of two from max |rating| and max |factor|) is carried as
//    z_hi + z_lo, two fp16 values holding 22 significant bits, and z z^T as
//    hi hi^T + hi lo^T + lo hi^T on v_mfma_f32_16x16x32_f16 with fp32 accumulation: three MFMAs
//    of 16x the fp32 rate per 32 ratings instead of eight fp32 16x16x4 ones (5.3x the
//    throughput); the dropped lo lo^T and the lo rounding leave ~3 2^-22 relative per product,
//    below the fp32 accumulation error of a >4096-term sum (OAP_ALS_GRAM=fp32 restores the
//    exact-fp32 products).  The direct solve of the mid-length rows (128 < n_u <= 4096,
//    OAP_ALS_X3_MIN_LEN) takes the same Gramian at one wave per SIMD (the pipelined x3 loop
//    needs ~430 registers); shorter direct rows are Cholesky-bound and keep the fp32 16x16x4 loop
//    at two waves per SIMD (OAP_ALS_DIRECT_X3=0: every direct row).
//  * Solve: the assembled matrix goes to LDS (row stride RP+4: conflict-free MFMA fragment
//    reads) and is factored by a right-looking blocked Cholesky with 16-wide panels: the
//    diagonal block in registers (lane-per-row, cross-lane broadcasts), the panel TRSM
//    lane-per-row against broadcast LDS rows, and the trailing SYRK update on MFMA.
#include <cstdlib>

#include "kernels/als_chol.h"
#include "kernels/device_utils.h"
#include "kernels/kernels.h"
#include "runtime/common.h"
#include "runtime/knobs.h"

namespace oap {
namespace kern {

namespace {

constexpr int kAlsThreads = 64;
using als::f4;

using als::kBlkF;
using als::kBS;
using als::mi;

struct SolveArgs {
  const int64_t* rowptr;
  const int32_t* cols;
  const float* vals;
  const int32_t* rows;       // row list for this launch
  int64_t nrows;             // entries of `rows`
  const int64_t* chunk_ptr;  // long-row mode: chunks [chunk_ptr[q], chunk_ptr[q+1]) of rows[q]
  const float* partials;     // long-row mode: per chunk partial_floats<NB>() floats
  const float* src;          // [n_src][ld]
  int ld, r;
  const float* yty;          // [r][r] (implicit) or null
  float alpha, lambda;
  int implicit;
  float* dst;                // [*][ld], indexed by row id
  unsigned long long* queue;
  unsigned long long* fail;
  int ablate;  // timing ablations (OAP_ALS_ABLATE): 1 no Gramian, 2 no Cholesky, 4 no solves,
               // 8 no YtY loads
  const unsigned* absmax;  // split-fp16 direct Gramian (X3): as PartialArgs::absmax
};

struct PartialArgs {
  const int32_t* cols;
  const float* vals;
  const int64_t* chunk_begin;  // rating range of each chunk
  const int64_t* chunk_end;
  int64_t nchunks;
  const float* src;
  int ld;
  float alpha;
  int implicit;
  float* partials;
  const unsigned* absmax;  // split-fp16 path: [max |rating|, max |source factor|] (float bits)
};

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int NB>
constexpr int partial_floats() {
  return (NB * (NB + 1) / 2) * 256 + 64 * NB + 64;
}

// Gramian + b + n_u of ratings [p0, p1) of one row (lane layout of the 16x16x4 f32 MFMA).
// Ratings go kSteps x 4 at a time: lanes fetch the block's (item, rating) pairs with one load
// each (the next block's pairs are prefetched), then all k-steps' factor rows (kSteps x NB loads
// per lane) are issued before the first MFMA — more rows in flight per wave, and the
// item-index -> factor-row dependency is paid once per block.  Loads are unconditional
// (out-of-range ratings read row 0 with zero weights).  kSteps = 2 keeps the rank-100 solve
// kernel free of register spills (4 spills).
template <int NB>
__device__ inline void accumulate(const int32_t* __restrict__ cols, const float* __restrict__ vals,
                                  int64_t p0, int64_t p1, const float* __restrict__ src, int ld,
                                  float alpha, bool implicit, f4 (&acc)[NB * (NB + 1) / 2],
                                  float (&bacc)[NB], int& nexp) {
  constexpr int kSteps = 2, kBlock = 4 * kSteps;
  const int lane = als::fresh_lane(), kk = lane >> 4, c = lane & 15;
  auto fetch = [&](int64_t p, int& it, float& rv) {
    const int64_t q = p + (c & (kBlock - 1));
    const bool ok = q < p1;
    it = ok ? cols[q] : -1;
    rv = ok ? vals[q] : 0.f;
  };
  int it_n = -1;
  float rv_n = 0.f;
  if (p0 < p1) fetch(p0, it_n, rv_n);
  for (int64_t p = p0; p < p1; p += kBlock) {
    const int it_l = it_n;
    const float rv_l = rv_n;
    if (p + kBlock < p1) fetch(p + kBlock, it_n, rv_n);  // next block's pairs in flight
    float yv[kSteps][NB], rvs[kSteps];
    bool oks[kSteps];
#pragma unroll
    for (int s4 = 0; s4 < kSteps; ++s4) {
      const int item = __shfl(it_l, 4 * s4 + kk, 64);
      rvs[s4] = __shfl(rv_l, 4 * s4 + kk, 64);
      oks[s4] = item >= 0;
      const float* yrow = src + static_cast<int64_t>(oks[s4] ? item : 0) * ld + c;
#pragma unroll
      for (int f = 0; f < NB; ++f) yv[s4][f] = yrow[16 * f];
    }
#pragma unroll
    for (int s4 = 0; s4 < kSteps; ++s4) {
      const bool ok = oks[s4];
      const float rv = rvs[s4];
      float wa, wb;
      if (implicit) {
        const float c1 = alpha * fabsf(rv);
        wa = ok ? c1 : 0.f;
        wb = (ok && rv > 0.f) ? 1.f + c1 : 0.f;
        nexp += (ok && rv > 0.f && c == 0) ? 1 : 0;
      } else {  // explicit: A += y y^T, b += r y
        wa = ok ? 1.f : 0.f;
        wb = ok ? rv : 0.f;
        nexp += (ok && c == 0) ? 1 : 0;
      }
      float av[NB];
#pragma unroll
      for (int f = 0; f < NB; ++f) {
        av[f] = wa * yv[s4][f];
        bacc[f] = fmaf(wb, yv[s4][f], bacc[f]);
      }
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[bi], yv[s4][bj], acc[t], 0, 0, 0);
    }
  }
}

// accumulate() for long-row chunks: the factor rows of block p + 1 are loaded while block p's
// MFMAs run (one block ahead, double-buffered), the (item, rating) pairs two blocks ahead.  The
// unpipelined loop waited for every block's rows before its first MFMA: at one wave per SIMD
// (the partial kernel keeps 28 accumulator tiles) it stalled most of the time.
template <int NB, int kSteps>
__device__ inline void accumulate_pipe(const int32_t* __restrict__ cols,
                                       const float* __restrict__ vals, int64_t p0, int64_t p1,
                                       const float* __restrict__ src, int ld, float alpha,
                                       bool implicit, f4 (&acc)[NB * (NB + 1) / 2],
                                       float (&bacc)[NB], int& nexp) {
  constexpr int kBlock = 4 * kSteps;
  static_assert(kBlock <= 16, "pairs of one block are fetched by 16 lanes");
  const int lane = threadIdx.x, kk = lane >> 4, c = lane & 15;
  auto fetch = [&](int64_t p, int& it, float& rv) {
    const int64_t q = p + (c & (kBlock - 1));
    const bool ok = q < p1;
    it = ok ? cols[q] : -1;
    rv = ok ? vals[q] : 0.f;
  };
  auto load = [&](int it_l, float rv_l, float (&yv)[kSteps][NB], float (&rvs)[kSteps],
                  bool (&oks)[kSteps]) {
#pragma unroll
    for (int s4 = 0; s4 < kSteps; ++s4) {
      const int item = __shfl(it_l, 4 * s4 + kk, 64);
      rvs[s4] = __shfl(rv_l, 4 * s4 + kk, 64);
      oks[s4] = item >= 0;
      const float* yrow = src + static_cast<int64_t>(oks[s4] ? item : 0) * ld + c;
#pragma unroll
      for (int f = 0; f < NB; ++f) yv[s4][f] = yrow[16 * f];
    }
  };
  if (p0 >= p1) return;
  int it_b = -1;
  float rv_b = 0.f;
  fetch(p0, it_b, rv_b);
  float yc[kSteps][NB], rc[kSteps];
  bool oc[kSteps];
  load(it_b, rv_b, yc, rc, oc);
  if (p0 + kBlock < p1) fetch(p0 + kBlock, it_b, rv_b);
  for (int64_t p = p0; p < p1; p += kBlock) {
    float yn[kSteps][NB], rn[kSteps];
    bool on[kSteps];
    const bool more = p + kBlock < p1;  // wave-uniform
    if (more) load(it_b, rv_b, yn, rn, on);
    if (p + 2 * kBlock < p1) fetch(p + 2 * kBlock, it_b, rv_b);
#pragma unroll
    for (int s4 = 0; s4 < kSteps; ++s4) {
      const bool ok = oc[s4];
      const float rv = rc[s4];
      float wa, wb;
      if (implicit) {
        const float c1 = alpha * fabsf(rv);
        wa = ok ? c1 : 0.f;
        wb = (ok && rv > 0.f) ? 1.f + c1 : 0.f;
        nexp += (ok && rv > 0.f && c == 0) ? 1 : 0;
      } else {
        wa = ok ? 1.f : 0.f;
        wb = ok ? rv : 0.f;
        nexp += (ok && c == 0) ? 1 : 0;
      }
      float av[NB];
#pragma unroll
      for (int f = 0; f < NB; ++f) {
        av[f] = wa * yc[s4][f];
        bacc[f] = fmaf(wb, yc[s4][f], bacc[f]);
      }
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[bi], yc[s4][bj], acc[t], 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int s4 = 0; s4 < kSteps; ++s4) {
        rc[s4] = rn[s4];
        oc[s4] = on[s4];
#pragma unroll
        for (int f = 0; f < NB; ++f) yc[s4][f] = yn[s4][f];
      }
    }
  }
}

// Split-fp16 Gramian + b + n_u of ratings [p0, p1) (long-row chunks), in the C layout of the
// 16x16 MFMAs (the same tiles accumulate() produces).  32 ratings per step on
// v_mfma_f32_16x16x32_f16: lane (g, c) = (lane >> 4, lane & 15) holds features 16 f + c of
// ratings 8 g .. 8 g + 7, which is both the A fragment (row i = c, k = 8 g + e) and the B fragment
// (k = 8 g + e, column j = c) of z^T, so one register set per feature block serves every tile.
// The next step's factor values load into the registers the current step has just converted
// (its fp16 fragments are separate): one step of MFMA work covers the gather latency; the
// (item, rating) pairs are fetched two steps ahead.  b and n_u stay fp32 on the VALU.
template <int NB, bool PIPE = true>
__device__ inline void accumulate_x3(const int32_t* __restrict__ cols,
                                     const float* __restrict__ vals, int64_t p0, int64_t p1,
                                     const float* __restrict__ src, int ld, float alpha,
                                     bool implicit, float scale, f4 (&acc)[NB * (NB + 1) / 2],
                                     float (&bacc)[NB], int& nexp) {
  constexpr int kStep = 32;
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  auto fetch = [&](int64_t p, int& it, float& rv) {
    const int64_t q = p + (lane & 31);
    const bool ok = q < p1;
    it = ok ? cols[q] : -1;
    rv = ok ? vals[q] : 0.f;
  };
  auto load = [&](int it_l, float rv_l, float (&y)[8][NB], float (&rvs)[8], bool (&oks)[8]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int item = __shfl(it_l, 8 * g + e, 64);
      rvs[e] = __shfl(rv_l, 8 * g + e, 64);
      oks[e] = item >= 0;
      const float* yrow = src + static_cast<int64_t>(oks[e] ? item : 0) * ld + c;
#pragma unroll
      for (int f = 0; f < NB; ++f) y[e][f] = yrow[16 * f];
    }
  };
  if (p0 >= p1) return;
  int it_b = -1;
  float rv_b = 0.f;
  fetch(p0, it_b, rv_b);
  float y[8][NB], rvs[8];
  bool oks[8];
  load(it_b, rv_b, y, rvs, oks);
  if (p0 + kStep < p1) fetch(p0 + kStep, it_b, rv_b);
  for (int64_t p = p0; p < p1; p += kStep) {
    // PIPE = false (the 2-wave/SIMD direct solve: 256 registers): this step's rows load at the
    // top of the step, the y registers die into the fp16 fragments before the MFMAs
    if (!PIPE && p != p0) load(it_b, rv_b, y, rvs, oks);
    if (!PIPE && p + kStep < p1) fetch(p + kStep, it_b, rv_b);
    // weights (absent ratings: 0)
    float sq[8], wb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float rv = rvs[e];
      const bool ok = oks[e];
      float wa;
      if (implicit) {
        const float c1 = alpha * fabsf(rv);
        wa = ok ? c1 : 0.f;
        wb[e] = (ok && rv > 0.f) ? 1.f + c1 : 0.f;
        nexp += (ok && rv > 0.f && c == 0) ? 1 : 0;
      } else {
        wa = ok ? 1.f : 0.f;
        wb[e] = ok ? rv : 0.f;
        nexp += (ok && c == 0) ? 1 : 0;
      }
      sq[e] = sqrtf(wa) * scale;
    }
    // b on the VALU; z = sqrt(w) y S split into fp16 hi + lo fragments
    h16x8 zh[NB], zl[NB];
#pragma unroll
    for (int f = 0; f < NB; ++f) {
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        bacc[f] = fmaf(wb[e], y[e][f], bacc[f]);
        bacc[f] = fmaf(wb[e + 1], y[e + 1][f], bacc[f]);
        const f32x2 z = f32x2{y[e][f], y[e + 1][f]} * f32x2{sq[e], sq[e + 1]};
        const h16x2 hi = __builtin_convertvector(z, h16x2);
        const h16x2 lo = __builtin_convertvector(z - __builtin_convertvector(hi, f32x2), h16x2);
        zh[f][e] = hi[0];
        zh[f][e + 1] = hi[1];
        zl[f][e] = lo[0];
        zl[f][e + 1] = lo[1];
      }
    }
    // the next step's pairs and factor values are in flight under this step's MFMAs
    const bool more = p + kStep < p1;  // wave-uniform
    if (PIPE && more) load(it_b, rv_b, y, rvs, oks);
    if (PIPE && p + 2 * kStep < p1) fetch(p + 2 * kStep, it_b, rv_b);
    // hi hi^T, then hi lo^T, then lo hi^T: consecutive MFMAs never chain on one accumulator
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = 0; bj <= bi; ++bj, ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(zh[bi], zh[bj], acc[t], 0, 0, 0);
    t = 0;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = 0; bj <= bi; ++bj, ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(zh[bi], zl[bj], acc[t], 0, 0, 0);
    t = 0;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = 0; bj <= bi; ++bj, ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(zl[bi], zh[bj], acc[t], 0, 0, 0);
  }
}

// power-of-two S with max |sqrt(w) y| S <= 2^14 (fp16 hi parts stay finite, lo parts normal for
// values within 2^-17 of the largest), and 1 / S^2 — exact, so the Gramian is S-independent
__device__ inline void x3_scale(const unsigned* absmax, float alpha, bool implicit, float& s,
                                float& inv_s2) {
  const float rmax = __uint_as_float(absmax[0]), ymax = __uint_as_float(absmax[1]);
  const float bound = sqrtf(implicit ? alpha * rmax : 1.f) * ymax;
  int e = 0;
  if (bound > 0.f && bound < 3e38f) frexpf(bound, &e);  // bound < 2^e
  e = e < -40 ? -40 : (e > 40 ? 40 : e);
  s = ldexpf(1.f, 14 - e);
  inv_s2 = ldexpf(1.f, 2 * (e - 14));
}

// Partial Gramian of one long-row chunk, pipelined accumulation at one wave per SIMD (all 512
// registers: the 28 accumulator tiles plus two blocks of factor rows in flight; 2 waves/SIMD with
// 256 registers each measured slower, 170 -> 199 ms/iter; 1 wave/SIMD without the pipeline 170;
// this form 140 at 1B ratings).
template <int NB, bool X3>
__global__ __launch_bounds__(kAlsThreads, 1) void oap_als_partial(PartialArgs a) {
  constexpr int NT = NB * (NB + 1) / 2;
  const int lane = threadIdx.x;
  float s = 1.f, inv_s2 = 1.f;
  if constexpr (X3) x3_scale(a.absmax, a.alpha, a.implicit != 0, s, inv_s2);
  for (int64_t q = blockIdx.x; q < a.nchunks; q += gridDim.x) {
    f4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    float bacc[NB];
#pragma unroll
    for (int f = 0; f < NB; ++f) bacc[f] = 0.f;
    int nexp = 0;
    if constexpr (X3)
      accumulate_x3<NB>(a.cols, a.vals, a.chunk_begin[q], a.chunk_end[q], a.src, a.ld, a.alpha,
                        a.implicit != 0, s, acc, bacc, nexp);
    else
      accumulate_pipe<NB, 4>(a.cols, a.vals, a.chunk_begin[q], a.chunk_end[q], a.src, a.ld,
                             a.alpha, a.implicit != 0, acc, bacc, nexp);
    float* out = a.partials + q * partial_floats<NB>();
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) out[t * 256 + e * 64 + lane] = acc[t][e] * inv_s2;
#pragma unroll
    for (int f = 0; f < NB; ++f) out[NT * 256 + f * 64 + lane] = bacc[f];
    out[NT * 256 + NB * 64 + lane] = static_cast<float>(nexp);
  }
}

template <int NB, bool LONG, bool X3>
__global__ __launch_bounds__(kAlsThreads, X3 ? 1 : 2) void oap_als_solve(SolveArgs a) {
  static_assert(!(LONG && X3), "long rows sum precomputed partials");
  constexpr int NT = NB * (NB + 1) / 2;
  constexpr int RP = 16 * NB;
  float xs = 1.f, inv_xs2 = 1.f;
  if constexpr (X3) x3_scale(a.absmax, a.alpha, a.implicit != 0, xs, inv_xs2);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* M = lds;  // lower 16x16 blocks, packed (mi)
  float* bv = lds + NB * (NB + 1) / 2 * kBlkF;  // RP
  const int r = a.r, lane = threadIdx.x;
  // the next row's queue slot, row id and CSR bounds are fetched one row ahead (three
  // dependent round trips), each under one phase of the current row (see als_lowrank.hip)
  const int64_t last = a.nrows - 1;  // (launched with a.nrows >= 1)
  int64_t q, row, hp0 = 0, hp1 = 0;
  {
    unsigned long long q_u = 0;
    if (lane == 0) q_u = atomicAdd(a.queue, 1ull);
    q = static_cast<int64_t>(__shfl(q_u, 0, 64));
    row = a.rows[q < a.nrows ? q : last];
    if constexpr (!LONG) {
      hp0 = a.rowptr[row];
      hp1 = a.rowptr[row + 1];
    }
  }
  while (q < a.nrows) {
    unsigned long long qn_u = 0;
    if (lane == 0) qn_u = atomicAdd(a.queue, 1ull);  // (in flight under the Gramian)

    f4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    float bacc[NB];
#pragma unroll
    for (int f = 0; f < NB; ++f) bacc[f] = 0.f;
    int nexp = 0;
    if constexpr (LONG) {
      // sum the row's chunk partials in chunk order (deterministic)
      for (int64_t ch = a.chunk_ptr[q]; ch < a.chunk_ptr[q + 1]; ++ch) {
        const float* pp = a.partials + ch * partial_floats<NB>();
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[t][e] += pp[t * 256 + e * 64 + lane];
#pragma unroll
        for (int f = 0; f < NB; ++f) bacc[f] += pp[NT * 256 + f * 64 + lane];
        nexp += static_cast<int>(pp[NT * 256 + NB * 64 + lane]);
      }
    } else if (!(a.ablate & 1)) {
      if constexpr (X3) {
        accumulate_x3<NB>(a.cols, a.vals, hp0, hp1, a.src, a.ld, a.alpha,
                          a.implicit != 0, xs, acc, bacc, nexp);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] *= inv_xs2;
      } else {
        accumulate<NB>(a.cols, a.vals, hp0, hp1, a.src, a.ld, a.alpha, a.implicit != 0, acc,
                       bacc, nexp);
      }
    }
    const int64_t qn = static_cast<int64_t>(__shfl(qn_u, 0, 64));
    const int64_t rown = a.rows[qn < a.nrows ? qn : last];  // (in flight under the assembly)
#pragma unroll
    for (int f = 0; f < NB; ++f) {
      bacc[f] += __shfl_xor(bacc[f], 16, 64);
      bacc[f] += __shfl_xor(bacc[f], 32, 64);
    }
    for (int m = 32; m >= 1; m >>= 1) nexp += __shfl_xor(nexp, m, 64);
    const float lam = a.lambda * static_cast<float>(nexp);

    // ---- assemble A = Gram + YtY + lam I (padding rows/cols -> identity) into LDS
    {
      int lid = lane;  // laundered: keeps per-element addresses from being hoisted
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
            float v;
            if (i < r && j < r) {
              v = acc[t][e];
              if (a.yty && !(a.ablate & 8)) v += a.yty[i * r + j];
              if (i == j) v += lam;
            } else {
              v = (i == j) ? 1.f : 0.f;
            }
            M[mi(i, j)] = v;
          }
      if (kk == 0) {
#pragma unroll
        for (int f = 0; f < NB; ++f) bv[16 * f + c] = (16 * f + c < r) ? bacc[f] : 0.f;
      }
    }
    __syncthreads();
    int64_t p0n = 0, p1n = 0;
    if constexpr (!LONG) {  // (in flight under the Cholesky)
      p0n = a.rowptr[rown];
      p1n = a.rowptr[rown + 1];
    }
    auto advance = [&]() {
      q = qn;
      row = rown;
      hp0 = p0n;
      hp1 = p1n;
    };

    // ---- blocked right-looking Cholesky, 16-wide panels (kernels/als_chol.h)
    const bool spd = als::chol_factor<NB>(M, (a.ablate & 2) ? NB : 0);
    float* out = a.dst + row * a.ld;
    if (!spd) {
      if (lane == 0) atomicAdd(a.fail, 1ull);
      for (int i = lane; i < a.ld; i += 64) out[i] = 0.f;
      __syncthreads();
      advance();
      continue;
    }
    // ---- blocked triangular solves, right-hand side in registers: lane l holds rows l and
    // l + 64 (v0, v1).  Per 16-row block: the diagonal solve runs in registers (16 sequential
    // steps, readlane broadcasts), the off-diagonal part is one lane-parallel update — instead
    // of r sequential LDS round trips per direction.
    float v0 = bv[lane], v1 = (lane + 64 < RP) ? bv[lane + 64] : 0.f;
    als::chol_solve<NB>(M, bv, v0, v1, (a.ablate & 4) ? 0 : NB);
    if (lane < a.ld) out[lane] = lane < r ? v0 : 0.f;
    if (lane + 64 < a.ld) out[lane + 64] = lane + 64 < r ? v1 : 0.f;
    for (int i = lane + 128; i < a.ld; i += 64) out[i] = 0.f;
    __syncthreads();
    advance();
  }
}

template <int NB>
size_t solve_lds() {
  // bv: the backward solve stages all 64 lanes (at least 128 floats)
  return (size_t(NB * (NB + 1) / 2) * kBlkF + std::max(16 * NB, 128)) * sizeof(float);
}

template <int NB, bool LONG, bool X3 = false>
void launch_solve(const SolveArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_als_solve<NB, LONG, X3>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((oap_als_solve<NB, LONG, X3>), dim3(grid), dim3(kAlsThreads), solve_lds<NB>(),
                     s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

template <int NB>
void run(const AlsSolveArgs& s, int num_cus, hipStream_t st) {
  const size_t lds = solve_lds<NB>();
  const int per_cu = std::max<int>(1, std::min<int>(16, int((160 * 1024) / (lds + 512))));
  SolveArgs a{};
  a.rowptr = s.rowptr;
  a.cols = s.cols;
  a.vals = s.vals;
  a.src = s.src;
  a.ld = s.ld;
  a.r = s.r;
  a.yty = s.yty;
  a.alpha = s.alpha;
  a.lambda = s.lambda;
  a.implicit = s.implicit ? 1 : 0;
  a.dst = s.dst;
  a.fail = s.fail;
  a.ablate = int(knob_int("OAP_ALS_ABLATE"));
  // rows of the low-rank path (the tail of short_rows) are solved by als_solve_lowrank
  const int64_t n_direct = (s.lr_off[4] > s.lr_off[0]) ? s.lr_off[0] : s.n_short;
  if (n_direct > 0) {
    OAP_HIP_CHECK(hipMemsetAsync(s.queue, 0, sizeof(unsigned long long), st));
    a.rows = s.short_rows;
    a.nrows = n_direct;
    a.queue = s.queue;
    // split-fp16 Gramian for the direct rows too (OAP_ALS_DIRECT_X3=0: exact-fp32 products)
    const bool direct_x3 = knob_int("OAP_ALS_DIRECT_X3") != 0;
    a.absmax = direct_x3 ? s.absmax : nullptr;
    // the longest rows on the split-fp16 Gramian, the short tail on the fp32 one at two waves
    // per SIMD (its rows are Cholesky-bound: 30 vs 38 ms per user half at 1B ratings)
    const int64_t n_x3 =
        a.absmax ? (s.n_direct_x3 < 0 ? n_direct : std::min(n_direct, s.n_direct_x3)) : 0;
    if (n_x3 > 0) {
      a.nrows = n_x3;
      launch_solve<NB, false, true>(
          a, int(std::min<int64_t>(n_x3, int64_t(num_cus) * per_cu)), st);
    }
    a.absmax = nullptr;
    if (n_direct > n_x3) {
      OAP_HIP_CHECK(hipMemsetAsync(s.queue + 3, 0, sizeof(unsigned long long), st));
      a.rows = s.short_rows + n_x3;
      a.nrows = n_direct - n_x3;
      a.queue = s.queue + 3;
      launch_solve<NB, false, false>(
          a, int(std::min<int64_t>(n_direct - n_x3, int64_t(num_cus) * per_cu)), st);
    }
  }
  als_solve_lowrank(s, num_cus, st);
  if (s.n_long > 0) {
    PartialArgs pa{};
    pa.cols = s.cols;
    pa.vals = s.vals;
    pa.chunk_begin = s.chunk_begin;
    pa.chunk_end = s.chunk_end;
    pa.nchunks = s.n_chunks;
    pa.src = s.src;
    pa.ld = s.ld;
    pa.alpha = s.alpha;
    pa.implicit = s.implicit ? 1 : 0;
    pa.partials = s.partials;
    pa.absmax = s.absmax;
    const dim3 pgrid(int(std::min<int64_t>(s.n_chunks, int64_t(num_cus) * 8)));
    if (s.absmax)
      hipLaunchKernelGGL((oap_als_partial<NB, true>), pgrid, dim3(kAlsThreads), 0, st, pa);
    else
      hipLaunchKernelGGL((oap_als_partial<NB, false>), pgrid, dim3(kAlsThreads), 0, st, pa);
    OAP_HIP_CHECK(hipGetLastError());
    OAP_HIP_CHECK(hipMemsetAsync(s.queue + 1, 0, sizeof(unsigned long long), st));
    a.rows = s.long_rows;
    a.nrows = s.n_long;
    a.chunk_ptr = s.long_chunk_ptr;
    a.partials = s.partials;
    a.queue = s.queue + 1;
    launch_solve<NB, true>(a, int(std::min<int64_t>(s.n_long, int64_t(num_cus) * per_cu)), st);
  }
}

// max |x| as float bits (non-negative floats order as unsigned integers): one atomic per block
__global__ __launch_bounds__(256) void oap_als_absmax(const float* __restrict__ x, int64_t n,
                                                      unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  const int64_t n4 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 ? n / 4 : 0;
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n4; i += int64_t(gridDim.x) * 256) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  for (int64_t i = 4 * n4 + blockIdx.x * int64_t(256) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * 256)
    m = fmaxf(m, fabsf(x[i]));
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f) atomicMax(out, __float_as_uint(m));  // (NaN compares false: ignored)
  }
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

size_t als_partial_floats(int r) {
  switch ((r + 15) / 16) {
    case 1: return partial_floats<1>();
    case 2: return partial_floats<2>();
    case 3: return partial_floats<3>();
    case 4: return partial_floats<4>();
    case 5: return partial_floats<5>();
    case 6: return partial_floats<6>();
    case 7: return partial_floats<7>();
    default: return partial_floats<8>();
  }
}

void als_solve(const AlsSolveArgs& s, int num_cus, hipStream_t st) {
  OAP_CHECK(s.r >= 1 && s.r <= als_max_rank(), "GPU ALS supports rank <= " << als_max_rank());
  OAP_CHECK(s.ld % 16 == 0 && s.ld >= s.r, "ALS factor stride must be a multiple of 16 >= rank");
  switch ((s.r + 15) / 16) {
    case 1: run<1>(s, num_cus, st); break;
    case 2: run<2>(s, num_cus, st); break;
    case 3: run<3>(s, num_cus, st); break;
    case 4: run<4>(s, num_cus, st); break;
    case 5: run<5>(s, num_cus, st); break;
    case 6: run<6>(s, num_cus, st); break;
    case 7: run<7>(s, num_cus, st); break;
    default: run<8>(s, num_cus, st); break;
  }
}

void als_absmax(const float* x, int64_t n, unsigned* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(oap_als_absmax, dim3(grid_for((n + 3) / 4, 256, 2048)), dim3(256), 0, s, x,
                     n, out);
  OAP_HIP_CHECK(hipGetLastError());
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
