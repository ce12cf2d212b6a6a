// One-wave blocked Cholesky factorisation and triangular solves of a small SPD matrix held in LDS
// as packed lower 16x16 blocks.  Shared by the ALS normal-equation solve (kernels/als.hip, the
// r x r system of a long row) and the low-rank Woodbury solve (kernels/als_lowrank.hip, the
// n x n capacitance system of a short row).
#pragma once

#include "kernels/device_utils.h"

namespace oap {
namespace kern {
namespace als {

typedef float f4 __attribute__((ext_vector_type(4)));

// LDS image: only the lower 16x16 blocks, packed (block (bi, bj), bi >= bj, at bi (bi + 1) / 2 +
// bj), dense 16-float rows and a 16-byte pad per block (consecutive blocks start on different
// banks).  28 blocks at rank 100 = 29 KB per row instead of 52 KB for the full square: 5 rows per
// CU.  Occupancy beats bank conflicts here: 20-float (conflict-free) rows fit only 4 rows per CU
// and ran 15% slower (0.200 vs 0.173 s/iter, 50M ratings, rank 100).
constexpr int kBS = 16, kBlkF = 16 * kBS + 4;
// RS: float stride of a block row.  16 packs tightest (the direct r x r solve is LDS-bound: 5
// rows per CU); 20 makes the lane-per-row float4 accesses conflict-free (rows 80 B apart land on
// distinct 4-bank groups) where occupancy is bound by registers anyway (the low-rank solve).
template <int RS>
constexpr int blk_floats() {
  return 16 * RS + 4;
}
template <int RS = kBS>
__device__ inline int mi(int i, int j) {
  const int bi = i >> 4, bj = j >> 4;
  return (bi * (bi + 1) / 2 + bj) * blk_floats<RS>() + (i & 15) * RS + (j & 15);
}
template <int NB, int RS = kBS>
constexpr int packed_floats() {
  return NB * (NB + 1) / 2 * blk_floats<RS>();
}

// Right-looking blocked Cholesky, 16-wide panels: the diagonal block in registers (lane-per-row,
// cross-lane broadcasts), the panel TRSM lane-per-row against broadcast LDS rows, the trailing
// SYRK update on v_mfma_f32_16x16x4_f32 with fragments straight from LDS.  Returns false (and
// stops) at the first non-positive pivot.  `first` > 0 skips panels (timing ablation).
// The lane id laundered through an empty asm: the lane masks derived from it (lane > j, lane ==
// j, ... for every unrolled j) are then recomputed where they are used instead of being hoisted
// out of the caller's row loop into hundreds of SGPR pairs (spilled to VGPR lanes and read back
// with v_readlane + hazard nops on every use).
__device__ inline int fresh_lane() {
  int lane = static_cast<int>(threadIdx.x);
  asm volatile("" : "+v"(lane));
  return lane;
}

// One step of the diagonal block's factorisation, lane (mod 16) = row: the pivot and column J of
// L come from DPP row broadcasts (v_mov_b32_dpp row_newbcast, lane K of every 16-lane row to that
// row) — a plain VALU operand, where v_readlane round-trips each value through an SGPR (with
// its hazard wait) — 16 broadcasts a step instead of 16 readlanes.  Every 16-lane row of the
// wave holds a copy of the block (rows of lane & 15); only lanes 0..15 store it.
template <int J>
__device__ inline float row_bcast(float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + J, 0xF, 0xF, false));
}
// t[K] -= lij L[K][J] as ONE instruction: v_fmac_f32 with the DPP broadcast on its first source
// (lane K of the row's t[J]) — the compiler keeps a v_mov_b32_dpp apart from the FMA that uses
// it.  fma(b, -lij, t) is bitwise fma(-lij, b, t).  The caller waits 2 states after writing tj
// (VALU write -> DPP read); the updates write other registers than they broadcast.
template <int J, int K>
__device__ inline void diag_update(float (&t)[16], float nlij, float tj) {
  if constexpr (K < 16) {
    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(t[K])
                 : "v"(tj), "v"(nlij), "i"(K));
    diag_update<J, K + 1>(t, nlij, tj);
  }
}
template <int J>
__device__ inline void diag_steps(float (&t)[16], int rl, bool& ok) {
  if constexpr (J < 16) {
    const float piv = row_bcast<J>(t[J]);
    ok = ok && (piv > 0.f);
    // (v_sqrt_f32, 1 ulp: the IEEE-exact sqrtf expands to ~10 VALU on the serial chain)
    const float dj = __builtin_amdgcn_sqrtf(fmaxf(piv, 1e-30f)), inv = __builtin_amdgcn_rcpf(dj);
    t[J] = (rl > J) ? t[J] * inv : (rl == J ? dj : t[J]);
    const float nlij = (rl > J) ? -t[J] : 0.f;
    if constexpr (J + 1 < 16) {
      const float tj = t[J];
      asm volatile("s_nop 1" ::"v"(tj));  // (VALU write -> DPP read: 2 wait states)
      diag_update<J, J + 1>(t, nlij, tj);
    }
    diag_steps<J + 1>(t, rl, ok);
  }
}

template <int NB, int RS = kBS>
__device__ inline bool chol_factor(float* M, int first = 0) {
  constexpr int RP = 16 * NB;
  const int lane = fresh_lane();
  for (int jb = first; jb < NB; ++jb) {
    const int o = 16 * jb;
    // (1) diagonal block: lanes 0..15 own its rows, in registers (copies in the other rows)
    float t[16];
    const int rl = lane & 15;
    {
#pragma unroll
      for (int m = 0; m < 16; m += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&M[mi<RS>(o + rl, o + m)]);
        t[m] = v.x;
        t[m + 1] = v.y;
        t[m + 2] = v.z;
        t[m + 3] = v.w;
      }
    }
    bool ok = true;
    diag_steps<0>(t, rl, ok);
    if (!ok) return false;
    if (lane < 16) {
#pragma unroll
      for (int m = 0; m < 16; m += 4)
        *reinterpret_cast<float4*>(&M[mi<RS>(o + lane, o + m)]) =
            make_float4(t[m], t[m + 1], t[m + 2], t[m + 3]);
    }
    __syncthreads();
    if (jb + 1 == NB) break;
    // (2) panel TRSM: rows below solve x L_jj^T = a, lane-per-row, L_jj rows broadcast
    for (int i = o + 16 + lane; i < RP; i += 64) {
      float x[16];
#pragma unroll
      for (int m = 0; m < 16; m += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&M[mi<RS>(i, o + m)]);
        x[m] = v.x;
        x[m + 1] = v.y;
        x[m + 2] = v.z;
        x[m + 3] = v.w;
      }
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) {
        float lrow[16];
#pragma unroll
        for (int m = 0; m < 16; m += 4) {
          const float4 v = *reinterpret_cast<const float4*>(&M[mi<RS>(o + cc, o + m)]);
          lrow[m] = v.x;
          lrow[m + 1] = v.y;
          lrow[m + 2] = v.z;
          lrow[m + 3] = v.w;
        }
        float s = x[cc];
#pragma unroll
        for (int m = 0; m < cc; ++m) s = fmaf(-x[m], lrow[m], s);
        x[cc] = s * __builtin_amdgcn_rcpf(lrow[cc]);
      }
#pragma unroll
      for (int m = 0; m < 16; m += 4)
        *reinterpret_cast<float4*>(&M[mi<RS>(i, o + m)]) =
            make_float4(x[m], x[m + 1], x[m + 2], x[m + 3]);
    }
    __syncthreads();
    // (3) trailing update T[ib][kb] -= P_ib P_kb^T on MFMA (fragments straight from LDS)
    {
      const int kk = lane >> 4, c = lane & 15;
      for (int ib = jb + 1; ib < NB; ++ib) {
        float pa[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) pa[s4] = -M[mi<RS>(16 * ib + c, o + 4 * s4 + kk)];
        for (int kb = jb + 1; kb <= ib; ++kb) {
          f4 cacc;
#pragma unroll
          for (int e = 0; e < 4; ++e) cacc[e] = M[mi<RS>(16 * ib + 4 * kk + e, 16 * kb + c)];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const float pb = M[mi<RS>(16 * kb + c, o + 4 * s4 + kk)];
            cacc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[s4], pb, cacc, 0, 0, 0);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) M[mi<RS>(16 * ib + 4 * kk + e, 16 * kb + c)] = cacc[e];
        }
      }
    }
    __syncthreads();
  }
  return true;
}

// Diagonal-block steps of the triangular solves.  Step J's value z_J = vd / L_JJ is meaningful at
// lane base + J and reaches the block's other rows by a DPP row broadcast (the block occupies one
// 16-lane row), fused into the update as ONE v_fmac_f32_dpp: vd += m_J z_J with the per-lane
// coefficient m_J = -L[row][J] below the diagonal, 1 on it (where vd was zeroed first: vd = z_J)
// and 0 elsewhere — three VALU a step (multiply, select, fused update) instead of six.  The
// reciprocals and coefficients are formed before the chain.  (fma(-l, z, v) is bitwise the
// original update; a zero coefficient leaves vd exactly.)
template <int J>
__device__ inline void solve_steps_fwd(const float (&rt)[16], const float (&m)[16], float& vd,
                                       int rl) {
  if constexpr (J < 16) {
    const float zl = vd * rt[J];
    vd = (rl == J) ? 0.f : vd;
    asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(vd)
                 : "v"(zl), "v"(m[J]), "i"(J));
    solve_steps_fwd<J + 1>(rt, m, vd, rl);
  }
}
template <int J>
__device__ inline void solve_steps_bwd(const float (&rt)[16], const float (&m)[16], float& vd,
                                       int rl) {
  if constexpr (J >= 0) {
    const float xl = vd * rt[J];
    vd = (rl == J) ? 0.f : vd;
    asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(vd)
                 : "v"(xl), "v"(m[J]), "i"(J));
    solve_steps_bwd<J - 1>(rt, m, vd, rl);
  }
}

// L L^T x = b with the factor from chol_factor.  Right-hand side in registers: lane l holds rows
// l and l + 64 (v0, v1; v1 only when NB > 4).  Per 16-row block the diagonal solve runs in
// registers (16 sequential steps, readlane broadcasts) and the off-diagonal part is one
// lane-parallel update — instead of r sequential LDS round trips per direction.  `bv`: RP floats
// of LDS scratch.  `nsolve` < NB skips blocks (timing ablation).
template <int NB, int RS = kBS>
__device__ inline void chol_solve(const float* M, float* bv, float& v0, float& v1,
                                  int nsolve = NB) {
  constexpr int RP = 16 * NB;
  const int lane = fresh_lane();
  // forward: L z = b
#pragma unroll
  for (int jb = 0; jb < nsolve; ++jb) {
    const int o = 16 * jb, base = o & 63, rl = lane - base;
    const bool mine = rl >= 0 && rl < 16;
    const int rr = mine ? rl : 0;
    float t[16];
#pragma unroll
    for (int m = 0; m < 16; m += 4) {
      const float4 q = *reinterpret_cast<const float4*>(&M[mi<RS>(o + rr, o + m)]);
      t[m] = q.x;
      t[m + 1] = q.y;
      t[m + 2] = q.z;
      t[m + 3] = q.w;
    }
    float vd = (o < 64) ? v0 : v1;
    // the serial chain on the block's own 16-lane row (DPP row broadcasts), then z to every lane
    // (lane base + j holds z_j) by independent readlanes off the chain
    {
      float rt[16], m[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        // (rows of other blocks: a zero reciprocal broadcasts z = 0, so their zero coefficient
        // leaves them bitwise untouched; 1/0 there would broadcast inf and 0 * inf = NaN)
        rt[j] = mine ? __builtin_amdgcn_rcpf(t[j]) : 0.f;
        m[j] = rl == j ? 1.f : ((mine && rl > j) ? -t[j] : 0.f);
      }
      solve_steps_fwd<0>(rt, m, vd, rl);
    }
    float z[16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      z[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vd), base + j));
    if (o < 64) v0 = vd;
    else v1 = vd;
    if (jb + 1 < NB) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = lane + 64 * h;
        if (i >= o + 16 && i < RP) {
          float acc2 = 0.f;
#pragma unroll
          for (int m = 0; m < 16; m += 4) {
            const float4 q = *reinterpret_cast<const float4*>(&M[mi<RS>(i, o + m)]);
            acc2 = fmaf(q.x, z[m], acc2);
            acc2 = fmaf(q.y, z[m + 1], acc2);
            acc2 = fmaf(q.z, z[m + 2], acc2);
            acc2 = fmaf(q.w, z[m + 3], acc2);
          }
          if (h == 0) v0 -= acc2;
          else v1 -= acc2;
        }
      }
    }
  }
  // backward: L^T x = z
#pragma unroll
  for (int jb = nsolve - 1; jb >= 0; --jb) {
    const int o = 16 * jb, base = o & 63, rl = lane - base;
    const bool mine = rl >= 0 && rl < 16;
    float vd = (o < 64) ? v0 : v1;
    if (jb + 1 < NB) {
      // z_{o+m} -= sum_{i >= o+16} L[i][o+m] x_i: x staged in LDS, 4 row groups per column
      bv[lane] = v0;
      if (lane + 64 < RP) bv[lane + 64] = v1;
      __syncthreads();
      const int m = lane & 15, g = lane >> 4;
      float part = 0.f;
      for (int i = o + 16 + g; i < RP; i += 4) part = fmaf(M[mi<RS>(i, o + m)], bv[i], part);
      part += __shfl_xor(part, 16, 64);
      part += __shfl_xor(part, 32, 64);
      const float sub = __shfl(part, (lane - base) & 15, 64);
      if (mine) vd -= sub;
      __syncthreads();
    }
    // diagonal block: lane base + p holds column p of L_jj
    float c[16];
    const int cp = mine ? rl : 0;
#pragma unroll
    for (int mm = 0; mm < 16; ++mm) c[mm] = M[mi<RS>(o + mm, o + cp)];
    {
      float rt[16], m[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        rt[j] = mine ? __builtin_amdgcn_rcpf(c[j]) : 0.f;
        m[j] = rl == j ? 1.f : ((mine && rl < j) ? -c[j] : 0.f);
      }
      solve_steps_bwd<15>(rt, m, vd, rl);
    }
    if (o < 64) v0 = vd;
    else v1 = vd;
  }
}

}  // namespace als
}  // namespace kern
}  // namespace oap
