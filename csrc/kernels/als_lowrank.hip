// Implicit ALS, short rows: the normal equations solved through their low-rank structure.
//
// Spark's per-row system (ALS.scala:1718-1800, see kernels/als.hip) is
//   A = Y^T Y + lambda n_u I + Y_u^T C_u Y_u,   b = Y_u^T w_u,   w_i = (1 + c_i) [r_i > 0],
// with Y_u the n x r block of the row's source factors and C_u = diag(alpha |r_i|).  For a row
// with n < r ratings, A is a diagonal matrix plus a rank-n update once the factors are expressed
// in the eigenbasis of Y^T Y = Q Lambda Q^T (computed once per half iteration on the host, the
// source factors rotated once: Yq = Y Q):
//   A_q = D + Yq_u^T C Yq_u,  D = Lambda + lambda n_u I  (diagonal, per row only through n_u).
// With W = Yq_u D^{-1/2} (n x r) and S = C^{1/2} the system is D^{1/2} (I + W^T S^2 W) D^{1/2}, and
// the Woodbury identity turns its r x r Cholesky into an n x n one:
//   g = D^{-1/2} b_q = W^T w,   M = I + S W W^T S  (n x n, SPD, eigenvalues >= 1),
//   x_q = D^{-1/2} (g - W^T S M^{-1} S W g),   x = Q x_q  (the back-rotation, kernel below).
// Rows with n <= 64 ratings (the bulk of a user side at 1B ratings: 50 per user) take this path:
// the Gramian is n^2 r instead of n r^2 MACs, the Cholesky n^3/3 instead of r^3/3, and the LDS
// image of M is 10 blocks (11 KB) instead of 28 (30 KB), so 3x the rows are resident per CU.
// Error: M is well conditioned (cond = 1 + |SW|^2), the normwise error is of the order of the
// direct solve's (cond(A) eps); tests/test_als_gpu.py compares both paths with an fp64 solve.
//
// MI355X mapping, one wave per row from an atomic queue (one launch per n-class NBN = ceil(n/16),
// so M has no padding blocks beyond the row's own):
//  * lane (c, kk) loads W fragments W[16 bi + c][16 q + 4 kk + e] as float4s of rotated factor
//    rows (every k-order is a valid MFMA k-order for W W^T: A and B fragments index k the same);
//  * M tiles on v_mfma_f32_16x16x4_f32 (exact fp32 products), scaled by s_i s_j and written to
//    the packed-lower LDS image (kernels/als_chol.h), padding rows (s = 0) are identity;
//  * the blocked Cholesky and both triangular solves of kernels/als_chol.h at NB = NBN;
//  * g, S W g and W^T S s are fragment-local FMAs plus cross-lane (DPP) reductions.
#include <cstdlib>

#include "kernels/als_chol.h"
#include "kernels/device_utils.h"
#include "kernels/kernels.h"
#include "runtime/common.h"
#include "runtime/knobs.h"

namespace oap {
namespace kern {

namespace {

using als::f4;
constexpr int kRS = 20;  // conflict-free block rows (als_chol.h): occupancy is register-bound here

struct LowRankArgs {
  const int64_t* rowptr;
  const int32_t* cols;
  const float* vals;
  const int32_t* rows;  // rows of this launch (each with <= 16 NBN ratings)
  int64_t nrows;
  const float* src;  // rotated source factors [n_src][ld] (columns >= r zero)
  const float* eig;  // [ld] eigenvalues of Y^T Y (padding columns 1)
  int ld;
  float alpha, lambda;
  float* out;  // [nrows][ld] rotated solutions, by position in `rows`
  unsigned long long* queue;
  unsigned long long* fail;
  int ablate;  // timing ablations (OAP_ALS_ABLATE): 16 no M MFMAs, 32 no Cholesky / solves,
               // 64 no second factor read
};

template <int CTRL>
__device__ inline float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// sum over the 16 lanes of a row group (c), every lane gets it (bitwise the same): DPP
// quad_perm xor 1, xor 2, row_half_mirror, row_mirror — four VALU adds, no LDS crossbar
__device__ inline float xor_sum16(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}

template <int NBR, int NBN, int OCC>
__global__ __launch_bounds__(64, OCC) void oap_als_lowrank(LowRankArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* M = lds;                                 // n x n, packed lower blocks
  float* bv = lds + als::packed_floats<NBN, kRS>();  // 64 floats (the backward solve: 64 lanes)
  float* gs = bv + 64;                            // 16 NBR floats: g while W is not resident
  float* dhs = gs + 16 * NBR;                     // 16 NBR floats: D^{-1/2}
  const int ld = a.ld;

  // Row headers run one row ahead: the queue pop, the row id, its CSR bounds and its (item,
  // rating) pairs are four dependent memory round trips.  Each level of the NEXT row is issued
  // during one phase of the current row (D^{-1/2}, the two W halves, the Cholesky) and consumed
  // in the next, so only the factor-row gathers stay exposed.  Loads are unconditional (indices
  // clamped) so no branch makes the compiler drain the memory counter.
  const int64_t last = a.nrows - 1;  // (launched with a.nrows >= 1)
  int64_t q, hp1;
  int hit;
  float hrv;
  int64_t hp0;
  {
    const int lane = als::fresh_lane();
    unsigned long long q_u = 0;
    if (lane == 0) q_u = atomicAdd(a.queue, 1ull);
    q = static_cast<int64_t>(__shfl(q_u, 0, 64));
    const int64_t row = a.rows[q < a.nrows ? q : last];
    hp0 = a.rowptr[row];
    hp1 = a.rowptr[row + 1];
    const int64_t ql = hp0 + (lane < int(hp1 - hp0) ? lane : 0);
    hit = a.cols[ql];
    hrv = a.vals[ql];
  }
  while (q < a.nrows) {
    // lane masks recomputed per row (kernels/als_chol.h: fresh_lane)
    const int lane = als::fresh_lane(), kk = lane >> 4, c = lane & 15;
    const int n = static_cast<int>(hp1 - hp0);  // <= 16 NBN (host-checked)
    unsigned long long qn_u = 0;
    if (lane == 0) qn_u = atomicAdd(a.queue, 1ull);  // the next row's slot (in flight)

    // per-rating scalars, lane l = rating l (lanes >= n: weight 0)
    const int it = lane < n ? hit : 0;
    const float rv = lane < n ? hrv : 0.f;
    const float cw = a.alpha * fabsf(rv);
    const float sc = sqrtf(cw);
    const bool pos = lane < n && rv > 0.f;
    const float wb = pos ? 1.f + cw : 0.f;
    const int nexp = __popcll(__ballot(pos));
    const float lam = a.lambda * static_cast<float>(nexp);

    // D^{-1/2} at the fragment columns k = 16 q + 4 kk + e, staged in LDS (registers are the
    // scarce resource here)
    bool okd = true;
    if (c == 0) {
#pragma unroll
      for (int qb = 0; qb < NBR; ++qb) {
        const float4 ev = *reinterpret_cast<const float4*>(a.eig + 16 * qb + 4 * kk);
        const float d4[4] = {ev.x + lam, ev.y + lam, ev.z + lam, ev.w + lam};
        float o4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          okd = okd && d4[e] > 0.f;
          o4[e] = __builtin_amdgcn_rsqf(fmaxf(d4[e], 1e-30f));
        }
        *reinterpret_cast<float4*>(dhs + 16 * qb + 4 * kk) =
            make_float4(o4[0], o4[1], o4[2], o4[3]);
      }
    }
    const bool fail_d = __ballot(!okd) != 0;
    __syncthreads();
    const int64_t qn = static_cast<int64_t>(__shfl(qn_u, 0, 64));
    const int64_t rown = a.rows[qn < a.nrows ? qn : last];  // (in flight under the first half)
    auto dh4 = [&](int qb) { return *reinterpret_cast<const float4*>(dhs + 16 * qb + 4 * kk); };
    // W fragments (rotated factors scaled by D^{-1/2}), g = W^T w (to LDS), the M tiles and
    // S W g, accumulated over two halves of the fragment columns: half of W in registers at a
    // time keeps the kernel at 3 waves per SIMD
    constexpr int NT = NBN * (NBN + 1) / 2;
    constexpr int QH = (NBR + 1) / 2;
    f4 macc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) macc[t] = f4{0.f, 0.f, 0.f, 0.f};
    float hp[NBN];
#pragma unroll
    for (int bi = 0; bi < NBN; ++bi) hp[bi] = 0.f;
    auto half = [&](auto q0c) {
      constexpr int q0 = decltype(q0c)::value;
      constexpr int QN = q0 == 0 ? QH : NBR - QH;
      float W[NBN][QH][4];
      float g[QH][4];
#pragma unroll
      for (int qb = 0; qb < QN; ++qb)
#pragma unroll
        for (int e = 0; e < 4; ++e) g[qb][e] = 0.f;
#pragma unroll
      for (int bi = 0; bi < NBN; ++bi) {
        const int i = 16 * bi + c;
        const int item = __shfl(it, i, 64);
        const float w_i = __shfl(wb, i, 64);
        const float* yrow = a.src + static_cast<int64_t>(item) * ld + 4 * kk + 16 * q0;
        float4 y[QH];
#pragma unroll
        for (int qb = 0; qb < QN; ++qb) y[qb] = *reinterpret_cast<const float4*>(yrow + 16 * qb);
#pragma unroll
        for (int qb = 0; qb < QN; ++qb) {
          const float yv[4] = {y[qb].x, y[qb].y, y[qb].z, y[qb].w};
          const float4 d = dh4(q0 + qb);
          const float dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            W[bi][qb][e] = yv[e] * dv[e];
            g[qb][e] = fmaf(w_i, W[bi][qb][e], g[qb][e]);
          }
        }
      }
#pragma unroll
      for (int qb = 0; qb < QN; ++qb) {
#pragma unroll
        for (int e = 0; e < 4; ++e) g[qb][e] = xor_sum16(g[qb][e]);
        if (c == 0)  // g leaves the registers (read back at the end)
          *reinterpret_cast<float4*>(gs + 16 * (q0 + qb) + 4 * kk) =
              make_float4(g[qb][0], g[qb][1], g[qb][2], g[qb][3]);
      }
      int t = 0;
      if (!(a.ablate & 16))
#pragma unroll
      for (int bi = 0; bi < NBN; ++bi)
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++t)
#pragma unroll
          for (int qb = 0; qb < QN; ++qb)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              macc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(W[bi][qb][e], W[bj][qb][e], macc[t],
                                                             0, 0, 0);
#pragma unroll
      for (int bi = 0; bi < NBN; ++bi)
#pragma unroll
        for (int qb = 0; qb < QN; ++qb)
#pragma unroll
          for (int e = 0; e < 4; ++e) hp[bi] = fmaf(W[bi][qb][e], g[qb][e], hp[bi]);
    };
    half(std::integral_constant<int, 0>{});
    const int64_t p0n = a.rowptr[rown], p1n = a.rowptr[rown + 1];  // (under the second half)
    if constexpr (NBR > QH) half(std::integral_constant<int, QH>{});

    // M = I + S W W^T S into LDS (tile (bi, bj): lane holds rows 16 bi + 4 kk + e, column
    // 16 bj + c)
    {
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < NBN; ++bi) {
        float si[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) si[e] = __shfl(sc, 16 * bi + 4 * kk + e, 64);
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++t) {
          const float sj = __shfl(sc, 16 * bj + c, 64);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ii = 16 * bi + 4 * kk + e, jj = 16 * bj + c;
            M[als::mi<kRS>(ii, jj)] = si[e] * sj * macc[t][e] + (ii == jj ? 1.f : 0.f);
          }
        }
      }
    }
    // h = S W g (vec layout: lane l holds h_l, i.e. row block kk, row c)
    float h = 0.f;
#pragma unroll
    for (int bi = 0; bi < NBN; ++bi) {
      float part = hp[bi];
      part += __shfl_xor(part, 16, 64);
      part += __shfl_xor(part, 32, 64);
      if (bi == kk) h = part;
    }
    h *= sc;  // lane l: s_l
    __syncthreads();
    // the next row's (item, rating) pairs, in flight under the Cholesky
    const int64_t qln = p0n + (lane < int(p1n - p0n) ? lane : 0);
    const int itn = a.cols[qln];
    const float rvn = a.vals[qln];
    auto advance = [&]() {
      q = qn;
      hp0 = p0n;
      hp1 = p1n;
      hit = itn;
      hrv = rvn;
    };

    const bool spd = (a.ablate & 32) ? true : als::chol_factor<NBN, kRS>(M);
    float* out = a.out + q * ld;
    if (!spd || fail_d) {
      if (lane == 0) atomicAdd(a.fail, 1ull);
      for (int k = lane; k < ld; k += 64) out[k] = 0.f;
      __syncthreads();
      advance();
      continue;
    }
    float v1 = 0.f;
    if (!(a.ablate & 32)) als::chol_solve<NBN, kRS>(M, bv, h, v1);
    const float ss = h * sc;  // S s, lane l = element l

    // x_q = D^{-1/2} (g - W^T S s) = D^{-1/2} (g - D^{-1/2} Yq_u^T S s): the factor rows again
    // (L2-resident), unscaled
    float t[NBR][4];
#pragma unroll
    for (int qb = 0; qb < NBR; ++qb)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[qb][e] = 0.f;
#pragma unroll
    for (int bi = 0; bi < ((a.ablate & 64) ? 0 : NBN); ++bi) {
      const int i = 16 * bi + c;
      const float s_i = __shfl(ss, i, 64);
      const int item = __shfl(it, i, 64);
      const float* yrow = a.src + static_cast<int64_t>(item) * ld + 4 * kk;
#pragma unroll
      for (int qb = 0; qb < NBR; ++qb) {
        const float4 y = *reinterpret_cast<const float4*>(yrow + 16 * qb);
        t[qb][0] = fmaf(y.x, s_i, t[qb][0]);
        t[qb][1] = fmaf(y.y, s_i, t[qb][1]);
        t[qb][2] = fmaf(y.z, s_i, t[qb][2]);
        t[qb][3] = fmaf(y.w, s_i, t[qb][3]);
      }
    }
#pragma unroll
    for (int qb = 0; qb < NBR; ++qb) {
      const float4 d = dh4(qb);
      const float dv[4] = {d.x, d.y, d.z, d.w};
      float xv[4];
      const float4 gq = *reinterpret_cast<const float4*>(gs + 16 * qb + 4 * kk);
      const float gv[4] = {gq.x, gq.y, gq.z, gq.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) xv[e] = dv[e] * (gv[e] - dv[e] * xor_sum16(t[qb][e]));
      if (c == 0)
        *reinterpret_cast<float4*>(out + 16 * qb + 4 * kk) =
            make_float4(xv[0], xv[1], xv[2], xv[3]);
    }
    __syncthreads();
    advance();
  }
}

template <int NBR, int NBN, int OCC = (NBN >= 4 ? 2 : 3)>
void launch_lowrank(const LowRankArgs& a, int num_cus, hipStream_t s) {
  constexpr size_t lds = (als::packed_floats<NBN, kRS>() + 64 + 32 * NBR) * sizeof(float);
  const int per_cu = std::max<int>(1, std::min<int>(16, int((160 * 1024) / (lds + 512))));
  const int grid = int(std::min<int64_t>(a.nrows, int64_t(num_cus) * per_cu));
  hipLaunchKernelGGL((oap_als_lowrank<NBR, NBN, OCC>), dim3(grid), dim3(64), lds, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

template <int NBR>
void lowrank_classes(const AlsSolveArgs& s, int num_cus, hipStream_t st) {
  LowRankArgs a{};
  a.rowptr = s.rowptr;
  a.cols = s.cols;
  a.vals = s.vals;
  a.src = s.lr_src;
  a.eig = s.lr_eig;
  a.ld = s.ld;
  a.alpha = s.alpha;
  a.lambda = s.lambda;
  a.fail = s.fail;
  a.ablate = int(knob_int("OAP_ALS_ABLATE"));
  // waves/SIMD of the 33-48-rating class (timing experiments)
  const int lr3_occ = int(knob_int("OAP_ALS_LR3_OCC"));
  // class j: rows [lr_off[j], lr_off[j+1]) of short_rows hold 16 (4 - j) - 15 .. 16 (4 - j) ratings
  for (int j = 0; j < 4; ++j) {
    const int64_t b = s.lr_off[j], e = s.lr_off[j + 1];
    if (e <= b) continue;
    a.rows = s.short_rows + b;
    a.nrows = e - b;
    a.out = s.lr_scratch + (b - s.lr_off[0]) * s.ld;
    a.queue = s.queue + 4 + j;
    OAP_HIP_CHECK(hipMemsetAsync(a.queue, 0, sizeof(unsigned long long), st));
    switch (j) {
      case 0: launch_lowrank<NBR, 4>(a, num_cus, st); break;
      case 1:
        if (lr3_occ == 2)
          launch_lowrank<NBR, 3, 2>(a, num_cus, st);
        else if (lr3_occ == 4)
          launch_lowrank<NBR, 3, 4>(a, num_cus, st);
        else
          launch_lowrank<NBR, 3>(a, num_cus, st);
        break;
      case 2: launch_lowrank<NBR, 2>(a, num_cus, st); break;
      default: launch_lowrank<NBR, 1>(a, num_cus, st); break;
    }
  }
}

// out[orow(i)] = in[irow(i)] R for n rows of ld floats (R: ld x ld row-major, in LDS).  256
// threads: 64 rows per tile in LDS (stride ld + 1: conflict-free column reads), thread (row,
// column group) accumulates ld / 4 outputs against broadcast rows of R.
template <int CW>
__global__ __launch_bounds__(256) void oap_als_rotate(const float* __restrict__ in,
                                                      const int32_t* __restrict__ in_rows,
                                                      float* __restrict__ out,
                                                      const int32_t* __restrict__ out_rows,
                                                      int64_t n, const float* __restrict__ R) {
  constexpr int LD = 4 * CW, XS = LD + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Rs = lds;            // LD x LD
  float* Xs = lds + LD * LD;  // 64 x XS
  const int t = threadIdx.x;
  for (int i = t; i < LD * LD / 4; i += 256)
    reinterpret_cast<float4*>(Rs)[i] = reinterpret_cast<const float4*>(R)[i];
  const int rl = t & 63, cg = t >> 6;
  for (int64_t r0 = int64_t(blockIdx.x) * 64; r0 < n; r0 += int64_t(gridDim.x) * 64) {
    __syncthreads();
    for (int i = t; i < 64 * (LD / 4); i += 256) {
      const int rr = i / (LD / 4), c4 = i % (LD / 4);
      const int64_t gi = r0 + rr;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gi < n) {
        const int64_t src_row = in_rows ? in_rows[gi] : gi;
        v = *reinterpret_cast<const float4*>(in + src_row * LD + 4 * c4);
      }
      float* xd = Xs + rr * XS + 4 * c4;
      xd[0] = v.x;
      xd[1] = v.y;
      xd[2] = v.z;
      xd[3] = v.w;
    }
    __syncthreads();
    float acc[CW];
#pragma unroll
    for (int j = 0; j < CW; ++j) acc[j] = 0.f;
    const float* xr = Xs + rl * XS;
#pragma unroll 2
    for (int k = 0; k < LD; ++k) {
      const float xv = xr[k];
      const float* rr = Rs + k * LD + cg * CW;
#pragma unroll
      for (int j = 0; j < CW; j += 4) {
        const float4 rv = *reinterpret_cast<const float4*>(rr + j);
        acc[j] = fmaf(xv, rv.x, acc[j]);
        acc[j + 1] = fmaf(xv, rv.y, acc[j + 1]);
        acc[j + 2] = fmaf(xv, rv.z, acc[j + 2]);
        acc[j + 3] = fmaf(xv, rv.w, acc[j + 3]);
      }
    }
    const int64_t gi = r0 + rl;
    if (gi < n) {
      const int64_t dst_row = out_rows ? out_rows[gi] : gi;
      float* o = out + dst_row * LD + cg * CW;
#pragma unroll
      for (int j = 0; j < CW; j += 4)
        *reinterpret_cast<float4*>(o + j) = make_float4(acc[j], acc[j + 1], acc[j + 2], acc[j + 3]);
    }
  }
}

// The same product on the f32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32 products, the
// VALU form's rate per clock but without its per-FMA LDS broadcast reads): 256 threads, a
// 64-row tile in LDS, wave w owns rows 16 w .. 16 w + 15 and all NB column blocks (NB
// accumulators of 4), R stays in LDS for the whole launch.
template <int NB>
__global__ __launch_bounds__(256) void oap_als_rotate_mfma(const float* __restrict__ in,
                                                           const int32_t* __restrict__ in_rows,
                                                           float* __restrict__ out,
                                                           const int32_t* __restrict__ out_rows,
                                                           int64_t n, const float* __restrict__ R) {
  constexpr int LD = 16 * NB, XS = LD + 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Rs = lds;            // LD x LD, row k = input feature
  float* Xs = lds + LD * LD;  // 64 x XS
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i16 = lane & 15, kq = lane >> 4;
  for (int i = t; i < LD * LD / 4; i += 256)
    reinterpret_cast<float4*>(Rs)[i] = reinterpret_cast<const float4*>(R)[i];
  for (int64_t r0 = int64_t(blockIdx.x) * 64; r0 < n; r0 += int64_t(gridDim.x) * 64) {
    __syncthreads();
    for (int i = t; i < 64 * (LD / 4); i += 256) {
      const int rr = i / (LD / 4), c4 = i % (LD / 4);
      const int64_t gi = r0 + rr;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gi < n) {
        const int64_t src_row = in_rows ? in_rows[gi] : gi;
        v = *reinterpret_cast<const float4*>(in + src_row * LD + 4 * c4);
      }
      float* xd = Xs + rr * XS + 4 * c4;
      xd[0] = v.x;
      xd[1] = v.y;
      xd[2] = v.z;
      xd[3] = v.w;
    }
    __syncthreads();
    f4 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};
    const float* xa = Xs + (16 * wave + i16) * XS + kq;  // A: row i16 of the wave, k = 4 ks + kq
    const float* rb = Rs + kq * LD + i16;                // B: k = 4 ks + kq, column 16 b + i16
#pragma unroll 4
    for (int ks = 0; ks < LD / 4; ++ks) {
      const float av = xa[4 * ks];
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, rb[4 * ks * LD + 16 * b], acc[b], 0, 0,
                                                      0);
    }
    // C/D layout: lane holds column 16 b + i16 of rows 4 kq + e of the wave's 16
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t gi = r0 + 16 * wave + 4 * kq + e;
      if (gi < n) {
        const int64_t dst_row = out_rows ? out_rows[gi] : gi;
        float* o = out + dst_row * LD + i16;
#pragma unroll
        for (int b = 0; b < NB; ++b) o[16 * b] = acc[b][e];
      }
    }
  }
}

template <int NB>
void launch_rotate_mfma(const float* in, const int32_t* in_rows, float* out,
                        const int32_t* out_rows, int64_t n, const float* R, int num_cus,
                        hipStream_t s) {
  constexpr int LD = 16 * NB;
  const size_t lds = size_t(LD * LD + 64 * (LD + 1)) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_als_rotate_mfma<NB>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int grid = int(std::min<int64_t>((n + 63) / 64, int64_t(num_cus) * 2));
  hipLaunchKernelGGL(oap_als_rotate_mfma<NB>, dim3(grid), dim3(256), lds, s, in, in_rows, out,
                     out_rows, n, R);
  OAP_HIP_CHECK(hipGetLastError());
}

template <int CW>
void launch_rotate(const float* in, const int32_t* in_rows, float* out, const int32_t* out_rows,
                   int64_t n, const float* R, int num_cus, hipStream_t s) {
  constexpr int LD = 4 * CW;
  const size_t lds = size_t(LD * LD + 64 * (LD + 1)) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_als_rotate<CW>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int grid = int(std::min<int64_t>((n + 63) / 64, int64_t(num_cus) * 2));
  hipLaunchKernelGGL(oap_als_rotate<CW>, dim3(grid), dim3(256), lds, s, in, in_rows, out, out_rows,
                     n, R);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace

int als_lowrank_max_len() { return 64; }

void als_solve_lowrank(const AlsSolveArgs& s, int num_cus, hipStream_t st) {
  const int64_t n = s.lr_off[4] - s.lr_off[0];
  if (n <= 0) return;
  OAP_CHECK(s.implicit && s.lr_src && s.lr_eig && s.lr_back && s.lr_scratch,
            "low-rank ALS path needs the rotated sources, eigenvalues and scratch");
  switch (s.ld / 16) {
    case 1: lowrank_classes<1>(s, num_cus, st); break;
    case 2: lowrank_classes<2>(s, num_cus, st); break;
    case 3: lowrank_classes<3>(s, num_cus, st); break;
    case 4: lowrank_classes<4>(s, num_cus, st); break;
    case 5: lowrank_classes<5>(s, num_cus, st); break;
    case 6: lowrank_classes<6>(s, num_cus, st); break;
    case 7: lowrank_classes<7>(s, num_cus, st); break;
    default: lowrank_classes<8>(s, num_cus, st); break;
  }
  // back to the original basis, scattered to the destination rows
  als_rotate(s.lr_scratch, nullptr, s.dst, s.short_rows + s.lr_off[0], n, s.lr_back, s.ld,
             num_cus, st);
}

void als_rotate(const float* in, const int32_t* in_rows, float* out, const int32_t* out_rows,
                int64_t n, const float* R, int ld, int num_cus, hipStream_t s) {
  if (n <= 0) return;
  OAP_CHECK(ld % 16 == 0 && ld >= 16 && ld <= 128,
            "als_rotate: ld must be 16..128, multiple of 16");
  const bool valu = knob_on("OAP_ALS_ROTATE_VALU");
  if (!valu) {
    switch (ld / 16) {
      case 1: launch_rotate_mfma<1>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
      case 2: launch_rotate_mfma<2>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
      case 3: launch_rotate_mfma<3>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
      case 4: launch_rotate_mfma<4>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
      case 5: launch_rotate_mfma<5>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
      case 6: launch_rotate_mfma<6>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
      case 7: launch_rotate_mfma<7>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
      default: launch_rotate_mfma<8>(in, in_rows, out, out_rows, n, R, num_cus, s); return;
    }
  }
  switch (ld / 16) {
    case 1: launch_rotate<4>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
    case 2: launch_rotate<8>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
    case 3: launch_rotate<12>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
    case 4: launch_rotate<16>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
    case 5: launch_rotate<20>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
    case 6: launch_rotate<24>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
    case 7: launch_rotate<28>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
    default: launch_rotate<32>(in, in_rows, out, out_rows, n, R, num_cus, s); break;
  }
}

}  // namespace kern
}  // namespace oap
