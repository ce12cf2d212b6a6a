// oap_kmeans_assign_mfma — the fused K-Means hot kernel for MI355X (gfx950, CDNA4).
//
// One launch per Lloyd iteration replaces oneDAL's step1Local (mllib-dal/src/main/native/
// KMeansDALImpl.cpp:70-77): distance cross-term on the matrix cores, argmin in
// registers, exact per-row cost, and per-cluster fixed-point sums/counts.
//
// * Layout: a wave owns a 32-row tile; lane (r = l&31, h = l>>5) holds features f = 16s + 8h + j
//   (s < KS, j < 8) of row r in registers.  Centroids are the MFMA A operand, staged ONCE per
//   workgroup in LDS with an odd-16B-slot row stride (conflict-free ds_read_b128); data rows are
//   the B operand straight from registers.  The 32x32 accumulator holds one data row x 16
//   centroids per lane, so the argmin is a per-lane scan plus one cross-half exchange.
// * Fast path: the cross term x.c on the bf16 matrix cores as a 3-product split
//   (x_hi c_hi + x_hi c_lo + x_lo c_hi, operands split as hi + lo bf16, fp32 accumulation):
//   3 x v_mfma_f32_32x32x16_bf16 replace 8 x v_mfma_f32_32x32x2_f32 per 16 features.  The split's
//   error is bounded by 4.6e-5 |x||c| per distance; every tile holding a row whose best/2nd-best
//   gap is inside that bound (+ the fp32 path's own bound) is re-decided by the exact-fp32 MFMA
//   pass, so assignments are IDENTICAL to the exact kernel (tested bitwise) at bf16-split speed.
// * Exact path (PRECISE and refinement): v_mfma_f32_32x32x2_f32 in the same feature order.
// * Exact per-row cost |x - c_best|^2 from the fp32 center; in the fast path the c_best rows are
//   fetched from L2 one tile ahead (software pipelined) so their latency hides under the next
//   tile's MFMAs.
// * Centroid sums in FIXED POINT: v = rint(x * 2^e_f) is an integer; the per-workgroup LDS
//   accumulator adds these integers as doubles (ds_add_f64) — exact while |partial| < 2^53,
//   which the driver's choice of e_f guarantees — so the order of the LDS atomics cannot change a
//   bit.  The flush converts to int64 and adds across workgroups, ranks (RCCL) in integer
//   arithmetic: results are bitwise identical for any schedule and any world size.
// * Persistent grid (>= 256 workgroups of 512 threads, one per CU: 2 waves per SIMD so one wave's
//   VALU epilogue overlaps the other's MFMAs), register prefetch two tiles ahead.
// * f32 or bf16 row storage (bf16: half the HBM bytes, 2 MFMAs per k-step, exact operands).
// * Pruning (Hamerly-style bounds, exact): each row keeps an upper bound u on its distance to its
//   center and a lower bound l on its distance to every other center.  When the centers move,
//   u grows by its center's drift and l shrinks by the largest drift (triangle inequality, fp32
//   rounding folded into rounded-up drifts and a margin wider than two candidates' fp32
//   evaluation error).  A tile whose rows all keep l^2 - u^2 > margin provably keeps every label
//   — the exact-fp32 argmin cannot change — so it skips the MFMA distance work and goes straight
//   to the exact cost and the accumulation.  Bounds are refreshed from the top-2 keys of every
//   tile that does run.  Chunked (large-k) passes: the seed pass computes the exact distance to
//   the old label and writes the per-row verdict; passes skip tiles whose rows all passed and
//   merge a running lower bound over the non-best candidates for the rest.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "kernels/device_utils.h"
#include "kernels/kmeans_frag.h"
#include "kernels/kmeans_internal.h"

namespace oap {
namespace kern {

namespace {

using namespace kmdev;

constexpr int kThreads = kAssignThreads;
constexpr int kWaves = kThreads / 64;

struct Smem {
  size_t planes, cn, dr, sc, acc, cnt, wcost, pref, total;
};
// lds_acc: LDS counters (+ the fp64 fixed-point sum accumulator when lds_sums).
__host__ __device__ inline Smem smem_plan(int dp, int kpad, int k, int d, bool precise,
                                          bool lds_acc, bool lds_sums = true) {
  Smem m;
  size_t off = 0;
  m.planes = 0;
  off += precise ? size_t(kpad) * stride_f32(dp) * 4 : size_t(2) * kpad * stride_bf16(dp) * 2;
  off = round16(off);
  m.cn = off;
  off = round16(off + size_t(kpad) * 4);
  m.dr = off;  // per-center drift (pruning)
  off = round16(off + size_t(kpad) * 4);
  m.sc = off;
  off = round16(off + size_t(dp) * 4);
  m.acc = off;
  if (lds_acc && lds_sums)
    off += size_t(k) * (d | 1) * 8;  // odd row stride => conflict-free ds_add_f64
  off = round16(off);
  m.cnt = off;
  if (lds_acc) off += size_t(k) * 4;
  off = round16(off);
  m.wcost = off;
  off += kWaves * 8;
  off = round16(off);
  m.pref = off;  // row-list mode: sub-segment prefix sums
  off += (kDeferSubs + 1) * 4;
  m.total = round16(off);
  return m;
}

// Capacity of one workgroup's deferral segment: the most tiles a workgroup of the persistent
// grid visits.
__host__ __device__ inline int64_t defer_segment(int64_t ntiles, int64_t grid) {
  const int64_t stride = grid * kWaves;
  return (ntiles + stride - 1) / stride * kWaves;
}

// BIAS (fast path): padding features carry the norms through the MFMAs so accumulators start at
// zero and the chunk loop reads only the operand fragments from LDS (no norm loads / seeding
// VALU).  f32 rows: x' = [x, 1, |x|^2], c' = [-2c, |c|^2, 1] (d + 2 <= 16*KS; |x|^2 is split
// hi/lo like every other feature).  bf16 rows: x' = [x, 1, hi(|x|^2), lo(|x|^2)],
// c' = [-2c, |c|^2, 1, 1] (d + 3 <= 16*KS) — x is exact in bf16, so each k-step needs only the
// two products x c_hi + x c_lo.
//
// XB (bf16 storage): rows are bf16 (row stride a.ld elements, multiple of 8).  Half the HBM
// bytes of f32 and 2 instead of 3 MFMAs per k-step; the refinement bound of the f32 split still
// holds (the bf16 products have strictly less error), so assignments equal an exact fp32
// evaluation of the bf16 data.
template <int KS, bool PRECISE, bool LDSACC, bool BIAS, bool XB, bool DEEP>
__global__ __launch_bounds__(kThreads, 2) void oap_kmeans_assign_mfma(KMeansAssignArgs a) {
  constexpr int DP = 16 * KS;
  // DEEP: three rotating tiles (prefetch two ahead); else two (prefetch one ahead).
  using F = Frag<KS, XB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int kpad = a.kpad, k = a.k, d = a.d;
  const Smem L = smem_plan(DP, kpad, k, d, PRECISE, LDSACC, a.sums_too);
  const int sb = stride_bf16(DP), s32 = stride_f32(DP);
  __bf16* ph = reinterpret_cast<__bf16*>(smem + L.planes);
  __bf16* pl = ph + size_t(kpad) * sb;
  float* p32 = reinterpret_cast<float*>(smem + L.planes);
  float* cn = reinterpret_cast<float*>(smem + L.cn);
  float* dr_l = reinterpret_cast<float*>(smem + L.dr);
  float* sc_l = reinterpret_cast<float*>(smem + L.sc);
  double* acc_l = reinterpret_cast<double*>(smem + L.acc);
  unsigned* cnt_l = reinterpret_cast<unsigned*>(smem + L.cnt);
  double* wcost = reinterpret_cast<double*>(smem + L.wcost);
  const int tid = threadIdx.x;
  const bool accumulate = a.accumulate && !a.merge && !(a.ablate & 1);
  const bool do_cost = !(a.ablate & 2);

  // ---- stage centroids (+ norms, fixed-point scales) once per workgroup
  for (int idx = tid; idx < kpad * DP; idx += kThreads) {
    const int c = idx / DP, f = idx - c * DP;
    const float v = a.centers[idx];
    if constexpr (PRECISE) {
      p32[c * s32 + f] = v;
    } else {
      __bf16 hi, lo;
      float w = -2.f * v;  // exact scaling: split(-2c) == -2 split(c)
      if (BIAS && f == d) w = (c < k) ? a.cnorm[c] : 1e30f;
      if (BIAS && f == d + 1) w = 1.f;
      if (BIAS && XB && f == d + 2) w = 1.f;
      bf16_split(w, hi, lo);
      ph[c * sb + f] = hi;
      pl[c * sb + f] = lo;
    }
  }
  // padded centroids get a huge FINITE norm: their keys must never be NaN bit patterns
  for (int c = tid; c < kpad; c += kThreads) cn[c] = (c < k) ? a.cnorm[c] : 1e30f;
  // Pruning (see the header): single launches test each row's bounds against the drift of its
  // own center; chunked passes only read the seed pass's per-row verdict.
  // row-list (refine) mode: this workgroup's segment of deferred rows, 32 per position
  const int32_t* rlist = a.row_list ? a.row_list + blockIdx.x * a.row_seg_cap : nullptr;
  unsigned* s_pref = reinterpret_cast<unsigned*>(smem + L.pref);
  if (rlist && tid == 0) {
    s_pref[0] = 0u;
    for (int w = 0; w < a.row_subs; ++w)
      s_pref[w + 1] = s_pref[w] + a.row_count[blockIdx.x * kDeferSubs + w];
  }
  const bool prune_single = !PRECISE && a.bounds && a.drift && !a.merge && !rlist;
  const bool prune_merge = !PRECISE && a.bounds && a.drift && a.merge;
  const bool need_meta =
      (!PRECISE && a.bounds && (a.drift || a.merge) && !rlist) || (rlist && a.delta);
  if (prune_single)
    for (int c = tid; c < kpad; c += kThreads) dr_l[c] = (c < k) ? a.drift[a.base + c] : 0.f;
  for (int f = tid; f < DP; f += kThreads)
    sc_l[f] = (a.scale && a.sums_too && f < d) ? a.scale[f] : 0.f;
  if (LDSACC && accumulate) {
    if (a.sums_too)
      for (int i = tid; i < k * (d | 1); i += kThreads) acc_l[i] = 0.0;
    for (int i = tid; i < k; i += kThreads) cnt_l[i] = 0u;
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t rcnt = rlist ? int64_t(s_pref[a.row_subs]) : 0;
  const int64_t rsub = rlist ? a.row_seg_cap / a.row_subs : 0;
  float thr1 = 0.f, thr0 = 0.f, cmax = 0.f;
  if constexpr (!PRECISE) {
    cmax = a.cstat ? a.cstat[0] : 0.f;
    thr1 = 1.25e-4f * cmax;  // 2 candidates x (bf16 split + accumulation) + fp32-path bound
    // bias feature: |c|^2 enters as a bf16 hi/lo pair (error <= 2^-18 |c|^2 per candidate)
    thr0 = (BIAS ? 1e-5f : 2e-6f) * cmax * cmax + 1e-30f;
  }
  const float dmax = prune_single ? a.drift_max[0] : 0.f;
  // fp32 evaluation error of two candidates' distances, relative to |x|^2 + cmax^2 (+ rounding
  // of the bound arithmetic): a bound gap wider than this decides the exact-fp32 argmin too
  const float mrel = 4e-7f * float(d + 8);
  const float ueps = 1.f + 1e-6f + 6e-8f * float(d + 4);  // direct-form |x - c|^2 rounding
  unsigned long long n_pruned = 0;
  unsigned n_exact = 0;  // row-list mode: rows this wave sent to the exact pass
  double my_cost = 0.0;

  // Bounds update carried into finish(): single launch: l = the row's new lower bound (distance);
  // merge: l / lo = lower bounds (squared) on every candidate of the chunk / on all but the
  // first key's (launch-local index i1), lin = running bound from earlier passes, yin = the seed's
  // verdict (kept).
  struct BUpd {
    float l = 0.f, lo = 0.f, lin = INFINITY, yin = -1.f;
    int i1 = -1;
    bool same = false;  // pruned row: its stored label is already right
    int old = -1;       // delta mode: the row's label from the previous iteration
  };

  // fixed-point accumulation of one row into cluster b (neg: subtract it)
  auto add_row = [&](const F& xv, int b, bool neg) {
    const float sgn = neg ? -1.f : 1.f;
    if constexpr (LDSACC) {
      if (h == 0) atomicAdd(&cnt_l[b], neg ? 0xffffffffu : 1u);
      if (!a.sums_too) return;
      double* ap = acc_l + b * (d | 1) + 8 * h;
      // k-steps below KS-1 are all real features (KS = ceil(d/16)): no per-element guards
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f0 = 16 * s + 8 * h;
        const float4 s0 = *reinterpret_cast<const float4*>(sc_l + f0);
        const float4 s1 = *reinterpret_cast<const float4*>(sc_l + f0 + 4);
        const float scv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        if (s < KS - 1 || d == DP) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            atomicAdd(ap + 16 * s + j, sgn * static_cast<double>(rintf(xv.at(s, j) * scv[j])));
        } else {
          const int nv = d - f0;  // real features of this lane's half of the last k-step
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nv)
              atomicAdd(ap + 16 * s + j, sgn * static_cast<double>(rintf(xv.at(s, j) * scv[j])));
        }
      }
    } else {
      if (h == 0) atomicAdd(&a.counts[b], neg ? ~0ull : 1ull);
      if (a.sums_too) {
        u64* gp = a.sums + size_t(b) * d;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int f = 16 * s + 8 * h + j;
            if (f < d) {
              const long long qv = static_cast<long long>(sgn * rintf(xv.at(s, j) * sc_l[f]));
              atomicAdd(gp + f, static_cast<u64>(qv));
            }
          }
      }
    }
  };

  // ---- per-row epilogue: exact cost, outputs, fixed-point accumulation
  auto finish = [&](const F& xv, const float (&cv)[KS][8], int b, int64_t row, bool valid,
                    const BUpd& bu) {
    float part = 0.f;  // padded features are zero in both operands
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = xv.at(s, j) - cv[s][j];
          part = fmaf(e, e, part);
        }
    const float rowcost = part + __shfl_xor(part, 32, 64);
    if (!valid) return;
    if (h == 0) {
      if (a.merge) {
        // (cost, index) order: lowest index wins exact ties whatever the chunk order / seed
        const float md = a.mindist[row];
        const int lab = a.labels[row];
        const bool take = rowcost < md || (rowcost == md && a.base + b < lab);
        if (take) {
          a.mindist[row] = rowcost;
          a.labels[row] = a.base + b;
        }
        if (!PRECISE && a.bounds) {
          // running bound over every candidate except the row's best: when this chunk wins, the
          // displaced best (exact md) joins and the pick leaves; otherwise the best may itself
          // sit in this chunk (seeded label, a deferred re-run) and must be left out
          const int best = take ? b : lab - a.base;
          const float ch = (best == bu.i1) ? bu.lo : bu.l;
          const float lo = take ? fminf(bu.lin, fminf(md, ch)) : fminf(bu.lin, ch);
          reinterpret_cast<float2*>(a.bounds)[row] = make_float2(lo, bu.yin);
        }
      } else {
        if (a.labels && !bu.same) a.labels[row] = a.base + b;
        if (a.mindist) a.mindist[row] = rowcost;
        if (!PRECISE && a.bounds)
          reinterpret_cast<float2*>(a.bounds)[row] =
              make_float2(sqrtf(rowcost) * ueps + 1e-30f, bu.l);
      }
      my_cost += double(rowcost);
    }
    if (!accumulate) return;
    // delta mode: a row that keeps its label contributes nothing; a moved row adds +x to its new
    // and -x to its old cluster (integer-valued fixed point, so exactly the full recount)
    if (a.delta) {
      if (bu.same || bu.old == b || bu.old < 0) return;
      add_row(xv, b, false);
      add_row(xv, bu.old, true);
    } else {
      add_row(xv, b, false);
    }
  };

  const int64_t ntiles_all = (a.n + 31) / 32;
  // Positions walk every tile, the seed's list of active tiles (one list, grid-strided), or —
  // seg_list — this workgroup's own segment of a deferral list (see defer_list below).
  const int64_t seg_cap = defer_segment(ntiles_all, gridDim.x);
  const int32_t* list =
      a.tile_list ? a.tile_list + (a.seg_list ? blockIdx.x * seg_cap : 0) : nullptr;
  const int64_t ntiles = rlist         ? (rcnt + 31) / 32
                         : !a.tile_list ? ntiles_all
                         : a.seg_list  ? int64_t(a.tile_count[blockIdx.x])
                                       : int64_t(*a.tile_count);
  const bool local_seg = a.seg_list || rlist;
  const int64_t stride = local_seg ? int64_t(kWaves) : int64_t(gridDim.x) * kWaves;
  int64_t t = local_seg ? int64_t(wave) : int64_t(blockIdx.x) * kWaves + wave;
  // the row a lane works on at position tt (clamped to a real row; valid_of tells if it counts)
  auto row_of = [&](int64_t tt) -> int64_t {
    if (rlist) {  // (an empty segment still prefetches: row 0 is a real row)
      if (rcnt == 0) return int64_t(0);
      int64_t i = tt * 32 + r;
      i = i < rcnt ? i : rcnt - 1;
      int w = 0;
      while (w + 1 < a.row_subs && int64_t(s_pref[w + 1]) <= i) ++w;
      return int64_t(rlist[w * rsub + (i - int64_t(s_pref[w]))]);
    }
    const int64_t row = tt * 32 + r;
    return row < a.n ? row : a.n - 1;
  };
  auto valid_of = [&](int64_t tt) { return rlist ? tt * 32 + r < rcnt : tt * 32 + r < a.n; };
  auto tile_of = [&](int64_t q) -> int64_t {
    if (!list) return q;  // (past the end: load_tile clamps the rows)
    return q < ntiles ? int64_t(list[q]) : ntiles_all - 1;
  };
  // deferral: one list segment + counter per workgroup (no single hot counter)
  auto defer_tile = [&](int64_t tile) {
    if (lane == 0) {
      const unsigned i = atomicAdd(a.defer_count + blockIdx.x, 1u);
      a.defer_list[blockIdx.x * seg_cap + i] = static_cast<int32_t>(tile);
    }
  };

  // Rows past n are clamped to row n-1 (their results are discarded, nothing needs zeroing);
  // only the last k-step can reach past the row stride, and it is zero-filled there.
  auto load_tile = [&](int64_t tt, F& dst) {
    const int64_t row = row_of(tt);
    if constexpr (XB) {
      const __bf16* p = static_cast<const __bf16*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f = 16 * s + 8 * h;
        if (s < KS - 1 || f < a.ld)
          dst.v[s] = *reinterpret_cast<const bf16x8*>(p + 16 * s);
        else
          dst.v[s] = bf16x8{};
      }
    } else {
      const float* p = static_cast<const float*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int f = 16 * s + 8 * h + 4 * q;
          float4 v;
          if (s < KS - 1 || f < a.ld)
            v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
          else
            v = make_float4(0.f, 0.f, 0.f, 0.f);
          dst.v[s][4 * q + 0] = v.x;
          dst.v[s][4 * q + 1] = v.y;
          dst.v[s][4 * q + 2] = v.z;
          dst.v[s][4 * q + 3] = v.w;
        }
    }
  };

  // Per-row pruning state of a tile (prefetched with the rows).
  struct Meta {
    int lab = 0;
    float bx = 0.f, by = -1.f;
  };
  auto load_meta = [&](int64_t tt, Meta& m) {
    if (!need_meta) return;
    const int64_t row = row_of(tt);
    if (!rlist) {
      const float2 b = reinterpret_cast<const float2*>(a.bounds)[row];
      m.bx = b.x;
      m.by = b.y;
    }
    if (prune_single || rlist) m.lab = a.labels[row];
  };

  // One tile: `x` holds its rows, `xn` receives the prefetch of tile `pf`.  DEEP: pf is two
  // tiles ahead and issued AFTER this tile's c_best loads — vmcnt retires in issue order, so
  // waiting for c_best never waits for the freshly issued prefetch, and each prefetch has about
  // two tile-times to land.  Otherwise pf is the next tile, issued before the MFMAs.  The loops
  // below rotate named buffers, so no register copies are needed.
  auto process = [&](const int64_t t, F& x, F& xn, const Meta& m, Meta& mn, const int64_t pf) {
    const int64_t row = row_of(t);
    const bool valid = valid_of(t);
    int bidx;
    if constexpr (PRECISE) {
      load_tile(pf, xn);  // prefetch, hidden behind this tile's MFMAs
      if (a.ablate & 8)
        bidx = r % k;  // timing ablation: no distance work
      else
        exact_argmin<KS>(p32, s32, x, cn, kpad, d, r, h, bidx);
      if (bidx >= k || bidx < 0) bidx = 0;
      float cb[KS][8];
      if (do_cost) {
        load_row8<KS>(p32 + size_t(bidx) * s32 + 8 * h, cb);
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) cb[s][j] = 0.f;
      }
      finish(x, cb, bidx, row, valid, BUpd{});
    } else {
      // merge mode: the row's best exact cost so far (earlier chunks / previous label), fetched
      // now so it has landed by the refinement decision
      float md_prev = INFINITY;
      if (a.merge && valid) md_prev = a.mindist[row];
      // MFMA B operands: xh = the row's bf16 hi part (bf16 rows: the row itself); the lo part of
      // f32 rows is built only when the 3-product tier runs.
      bf16x8 xh[KS], xl[XB ? 1 : KS];
      float nx2 = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) nx2 = fmaf(x.at(s, j), x.at(s, j), nx2);
      nx2 += __shfl_xor(nx2, 32, 64);
      // per-tile max |x|^2 (the scan's margin: conservative for every row)
      if (a.xnorm && !rlist) {
        float tmax = nx2;
#pragma unroll
        for (int m = 16; m >= 1; m >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, m, 64));
        if (lane == 0) a.xnorm[t] = tmax;
      }
      const float marg = mrel * (nx2 + cmax * cmax);
      // Pruning: a tile whose rows all keep their center provably (bounds) skips the distance
      // work; its rows still get the exact cost, outputs and accumulation from their label.
      if (prune_single || prune_merge) {
        float lk = 0.f;
        bool ok;
        if (prune_merge) {
          ok = m.by >= 0.f;  // the seed pass's verdict for this iteration
        } else {
          const float u = m.bx + dr_l[min(max(m.lab, 0), k - 1)];
          lk = m.by - dmax;
          ok = lk > 0.f && (lk - u) * (lk + u) > marg;
        }
        if (__all(!valid || ok)) {
          load_tile(pf, xn);
          load_meta(pf, mn);
          ++n_pruned;
          if (prune_merge) return;  // labels / mindist already hold the seed's exact answer
          const int b = min(max(m.lab, 0), k - 1);
          float cb[KS][8];
          load_row8<KS>(a.centers + size_t(b) * DP + 8 * h, cb);
          BUpd bu;
          bu.l = lk;
          bu.same = true;
          finish(x, cb, b, row, valid, bu);
          return;
        }
      }
      const int jb = d - 16 * (KS - 1) - 8 * h;  // lane-local slot of bias feature d (if in range)
      if constexpr (XB) {
#pragma unroll
        for (int s = 0; s < KS - 1; ++s) xh[s] = x.v[s];
        bf16x8 last = x.v[KS - 1];
        if constexpr (BIAS) {
          __bf16 nh, nl;
          bf16_split(nx2, nh, nl);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            last[j] = (j == jb) ? static_cast<__bf16>(1.f) : last[j];
            last[j] = (j == jb + 1) ? nh : last[j];
            last[j] = (j == jb + 2) ? nl : last[j];
          }
        }
        xh[KS - 1] = last;
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float v = x.v[s][j];
            if (BIAS && s == KS - 1) {
              v = (j == jb) ? 1.f : v;
              v = (j == jb + 1) ? nx2 : v;
            }
            xh[s][j] = static_cast<__bf16>(v);
          }
      }
      auto build_lo = [&]() {
        if constexpr (!XB) {
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float v = x.v[s][j];
              if (BIAS && s == KS - 1) {
                v = (j == jb) ? 1.f : v;
                v = (j == jb + 1) ? nx2 : v;
              }
              xl[s][j] = static_cast<__bf16>(v - static_cast<float>(xh[s][j]));
            }
        }
      };
      if constexpr (!DEEP) {  // prefetch, hidden behind this tile's MFMAs
        load_tile(pf, xn);
        load_meta(pf, mn);
      }

      // Accumulators are seeded with |c|^2 + |x|^2 and the planes hold -2c, so each MFMA chain
      // ends at |x - c|^2.  Top-2 tracking runs on integer KEYS: the float's bits with the low 10
      // mantissa bits replaced by the centroid index (kpad <= 1024) — int min/max give value
      // order plus lowest-index tie-break in 4 VALU ops per candidate.  Two accumulators let chunk
      // c's key epilogue (VALU) interleave with chunk c+1's MFMAs.
      //
      // Tiers (TERMS): 1 = hi x hi only (one MFMA per k-step; bound ~0.8% of |x||c|), 3 = the
      // bf16x3 split (x_hi c_hi + x_hi c_lo + x_lo c_hi; bf16 rows: x c_hi + x c_lo; bound
      // ~1e-4).  With a.fast1 the tile starts at tier 1 and only tiles holding a row whose top-2
      // gap is inside tier 1's bound run tier 3; rows still unsure after tier 3 are re-decided in
      // exact fp32.  Every tier's bound is rigorous, so the assignments never change.
      int k1 = 0x7fffffff, k2 = 0x7fffffff;
      auto mfma_chunk = [&](auto tag, int c0, f32x16& acc) {
        constexpr int T = decltype(tag)::value;
        if constexpr (!BIAS) {
          // norms first: the first MFMA needs the seeded accumulator + fragment 0 only
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float4 c4 = *reinterpret_cast<const float4*>(cn + c0 + 8 * g + 4 * h);
            acc[4 * g + 0] = c4.x + nx2;
            acc[4 * g + 1] = c4.y + nx2;
            acc[4 * g + 2] = c4.z + nx2;
            acc[4 * g + 3] = c4.w + nx2;
          }
        }
        const __bf16* ah_p = ph + size_t(c0 + r) * sb + 8 * h;
        const __bf16* al_p = pl + size_t(c0 + r) * sb + 8 * h;
        bf16x8 ah[KS], al[T == 1 ? 1 : KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          ah[s] = *reinterpret_cast<const bf16x8*>(ah_p + 16 * s);
          if constexpr (T != 1) al[s] = *reinterpret_cast<const bf16x8*>(al_p + 16 * s);
        }
        // KS = ceil(d/16): every k-step holds real features, so there is no runtime guard here
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          if (BIAS && s == 0)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], xh[s], f32x16{}, 0, 0, 0);
          else
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], xh[s], acc, 0, 0, 0);
          if constexpr (T != 1) {
            if constexpr (!XB)
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], xl[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[s], xh[s], acc, 0, 0, 0);
          }
        }
      };
      auto epilogue = [&](int c0, const f32x16& acc) {
        // chunk-local keys carry the in-chunk offset 8(e>>2)+(e&3) (an inline constant: one
        // v_and_or_b32 per candidate); the lane's chunk base c0+4h is OR-ed in once per chunk.
        // Keys are compared as signed ints (same order as the floats for the non-negative
        // distances; a tiny negative from rounding only ever looks like a near tie, which the
        // exact pass re-decides).  Integer min / med3 avoid the NaN canonicalisation that float
        // min/max would add, so the top-2 update is 3 VALU per candidate.  Four independent
        // trackers (candidates e mod 4) keep the dependency chains short.
        int t1[4], t2[4];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int off = 8 * (e >> 2) + (e & 3);
          const int key = (__float_as_int(acc[e]) & ~0x3ff) | (off & 0x3ff);
          const int t = e & 3;
          if (e < 4) {
            t1[t] = key;
            t2[t] = 0x7fffffff;
          } else {
            t2[t] = med3_i32(t1[t], t2[t], key);  // 2nd smallest of {t1, t2, key}, t1 <= t2
            t1[t] = min(t1[t], key);
          }
        }
        auto merge2 = [](int& x1, int& x2, int y1, int y2) {
          x2 = min(max(x1, y1), min(x2, y2));
          x1 = min(x1, y1);
        };
        merge2(t1[0], t2[0], t1[1], t2[1]);
        merge2(t1[2], t2[2], t1[3], t2[3]);
        merge2(t1[0], t2[0], t1[2], t2[2]);
        const int q1 = t1[0], q2 = t2[0];
        const int base = c0 + 4 * h;  // disjoint from every in-chunk offset's bits
        const int i1 = q1 | base, i2 = q2 | base;
        k2 = min(max(k1, i1), min(k2, i2));
        k1 = min(k1, i1);
      };
      auto run_tier = [&](auto tag) {
        k1 = 0x7fffffff;
        k2 = 0x7fffffff;
        if (a.ablate & 8) {
          k1 = r % k;  // timing ablation: no distance work
        } else {
          f32x16 accA, accB;
          mfma_chunk(tag, 0, accA);
          int c0 = 32;
          for (; c0 + 32 < kpad; c0 += 64) {  // branch-free body: chunk pairs
            mfma_chunk(tag, c0, accB);
            epilogue(c0 - 32, accA);
            mfma_chunk(tag, c0 + 32, accA);
            epilogue(c0, accB);
          }
          if (c0 < kpad) {  // one chunk left (wave-uniform)
            mfma_chunk(tag, c0, accB);
            epilogue(c0 - 32, accA);
            epilogue(c0, accB);
          } else {
            epilogue(c0 - 32, accA);
          }
        }
        // merge the two halves' top-2 keys
        const int o1 = __shfl_xor(k1, 32, 64), o2 = __shfl_xor(k2, 32, 64);
        k2 = min(max(k1, o1), min(k2, o2));
        k1 = min(k1, o1);
      };
      // A near tie inside this chunk only matters if the chunk can still win: in merge mode a
      // row whose chunk-best is provably worse than its best exact cost so far needs no exact
      // re-decision (every threshold bounds one candidate's error with room to spare).
      auto unsure_at = [&](float thr) {
        const float b1 = __int_as_float(k1 & ~0x3ff), b2 = __int_as_float(k2 & ~0x3ff);
        const float t = thr + 2.5e-4f * fabsf(b2);  // + key truncation
        return valid && !(a.ablate & 8) && !(b2 - b1 > t) && !(a.merge && b1 - t > md_prev);
      };
      // tier-3 bound: split + accumulation error, seed rounding
      const float thr3 = fmaf(thr1, sqrtf(nx2), thr0) + 2e-6f * nx2;
      bool unsure;
      float thr_used = thr3;  // bound of the tier that produced k1 / k2
      if (a.fast1) {
        run_tier(std::integral_constant<int, 1>{});
        // tier-1 bound, two candidates: cross term 2 x 2(2^-8 + 2^-18)|c||x|, |c|^2 bias
        // 2 x 2^-9 cmax^2, |x|^2 bias 2^-9 nx2 (cancels in the gap, not in the merge test),
        // fp32 accumulation 4e-5 (cmax^2 + nx2)
        const float cm = cmax;
        const float thrA = 0.0157f * cm * sqrtf(nx2) + 0.004f * cm * cm + 0.002f * nx2 +
                           4e-5f * (cm * cm + nx2) + 1e-30f;
        unsure = unsure_at(thrA);
        thr_used = thrA;
        if (a.defer_list && __any(unsure)) {
          defer_tile(t);
          unsure = false;  // decided after the last chunk (see KMeansAssignArgs::defer_list)
        }
        if (__any(unsure)) {
          thr_used = thr3;
          build_lo();
          run_tier(std::integral_constant<int, 3>{});
          unsure = unsure_at(thr3);
          if (lane == 0 && a.refine_tiles) atomicAdd(a.refine_tiles + 1, 1ull);
        }
      } else {
        build_lo();
        run_tier(std::integral_constant<int, 3>{});
        unsure = unsure_at(thr3);
        if (a.defer_list && __any(unsure)) {
          defer_tile(t);
          unsure = false;
        }
      }
      bidx = k1 & 0x3ff;
      bool to_exact = false;
      if (a.exact_rows && rlist) {
        // row-list mode: only the still-unsure rows go to the exact VALU pass (per-wave
        // sub-segment, filled in position order: deterministic)
        const unsigned long long um = __ballot(unsure && h == 0);
        if (um) {
          int32_t* seg = a.exact_rows + (int64_t(blockIdx.x) * kWaves + wave) * a.exact_sub_cap;
          if (unsure && h == 0)
            seg[n_exact + __popcll(um & ((1ull << lane) - 1ull))] = static_cast<int32_t>(row);
          n_exact += static_cast<unsigned>(__popcll(um));
          if (lane == 0 && a.refine_tiles) atomicAdd(a.refine_tiles, u64(__popcll(um)));
        }
        to_exact = unsure;
      } else if (__any(unsure)) {
        // rare: re-decide the whole tile exactly (bitwise the PRECISE kernel's answer)
        exact_argmin<KS>(a.centers, DP, x, cn, kpad, d, r, h, bidx);
        if (lane == 0 && a.refine_tiles) atomicAdd(a.refine_tiles, 1ull);
      }
      if (bidx >= k || bidx < 0) bidx = 0;  // only for degenerate (NaN / all-inf) inputs
      float cb[KS][8];
      if (do_cost) {
        load_row8<KS>(a.centers + size_t(bidx) * DP + 8 * h, cb);  // L2-resident
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) cb[s][j] = 0.f;
      }
      if constexpr (DEEP) {  // younger than the c_best loads (see above)
        load_tile(pf, xn);
        load_meta(pf, mn);
      }
      BUpd bu;
      if (a.delta) bu.old = min(max(m.lab, 0), k - 1);
      if (a.bounds) {
        // every candidate's true distance is >= its key - tt; the pick's rivals are the other
        // keys (the second key, or the first when the exact pass picked another center)
        const float b1 = __int_as_float(k1 & ~0x3ff), b2 = __int_as_float(k2 & ~0x3ff);
        const float tt = thr_used + 2.5e-4f * fabsf(b2) + marg;
        const float lo = ((bidx == (k1 & 0x3ff)) ? b2 : b1) - tt;
        if (a.merge) {
          bu.l = b1 - tt;
          bu.lo = b2 - tt;  // NaN (no second key) is ignored by fminf
          bu.i1 = k1 & 0x3ff;
          bu.lin = a.fresh_bound ? INFINITY : m.bx;  // the first chunk starts the bound afresh
          bu.yin = m.by;
        } else {
          bu.l = sqrtf(fmaxf(lo, 0.f)) * (1.f - 1e-6f);  // NaN (no second key) -> 0
        }
      }
      finish(x, cb, bidx, row, valid && !to_exact, bu);
    }
  };

  if constexpr (DEEP) {
    F xa, xb, xc;
    Meta ma, mb, mc;
    load_tile(tile_of(t), xa);
    load_meta(tile_of(t), ma);
    load_tile(tile_of(t + stride), xb);
    load_meta(tile_of(t + stride), mb);
    for (; t < ntiles; t += 3 * stride) {  // t is wave-uniform: every branch stays uniform
      process(tile_of(t), xa, xc, ma, mc, tile_of(t + 2 * stride));
      if (t + stride >= ntiles) break;
      process(tile_of(t + stride), xb, xa, mb, ma, tile_of(t + 3 * stride));
      if (t + 2 * stride >= ntiles) break;
      process(tile_of(t + 2 * stride), xc, xb, mc, mb, tile_of(t + 4 * stride));
    }
  } else {
    F xa, xb;
    Meta ma, mb;
    load_tile(tile_of(t), xa);
    load_meta(tile_of(t), ma);
    for (; t < ntiles; t += 2 * stride) {
      process(tile_of(t), xa, xb, ma, mb, tile_of(t + stride));
      if (t + stride >= ntiles) break;
      process(tile_of(t + stride), xb, xa, mb, ma, tile_of(t + 2 * stride));
    }
  }
  if (lane == 0 && n_pruned && a.pruned_tiles) atomicAdd(a.pruned_tiles, n_pruned);
  if (lane == 0 && a.exact_count && rlist) a.exact_count[blockIdx.x * kWaves + wave] = n_exact;

  // ---- deterministic per-block cost: fixed shuffle tree, waves in index order
  const double wsum = wave_sum_f64(my_cost);
  if (lane == 0) wcost[wave] = wsum;
  __syncthreads();
  if (tid == 0 && a.cost_slab) {
    double tot = 0.0;
    for (int w = 0; w < kWaves; ++w) tot += wcost[w];
    a.cost_slab[blockIdx.x] = tot;
  }
  if (LDSACC && accumulate) {
    for (int i = tid; a.sums_too && i < k * d; i += kThreads) {
      const int b = i / d, f = i - b * d;
      const double v = acc_l[b * (d | 1) + f];  // an exact integer, |v| < 2^53
      if (v != 0.0) atomicAdd(&a.sums[i], static_cast<u64>(static_cast<long long>(v)));
    }
    for (int i = tid; i < k; i += kThreads) {
      const int c = static_cast<int>(cnt_l[i]);  // signed: delta mode subtracts
      if (c) atomicAdd(&a.counts[i], static_cast<u64>(static_cast<long long>(c)));
    }
  }
}

// mindist[row] = |x_row - c_{labels[row]}|^2 with exactly the assign kernel's lane layout and
// fp32 summation order (so a later chunk that picks the same center computes the bitwise same
// value).  Seeds the chunked large-k passes with the previous iteration's labels.
//
// With bounds + drift it also decides pruning for the iteration's chunk passes: the row's lower
// bound on the non-label centers (the merged chunk bound of the last iteration, or the seed's own
// decayed bound for rows whose tile was skipped) minus the largest drift, against the exact
// distance just computed.  Writes bounds[row] = {unset (>= 3e38), l if the row provably keeps its
// label else -1}.
template <int KS, bool XB>
__global__ __launch_bounds__(256) void oap_kmeans_seed_mindist(KMeansAssignArgs a) {
  constexpr int DP = 16 * KS;
  using F = Frag<KS, XB>;
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (a.n + 31) / 32;
  const bool prune = a.bounds && a.drift;
  const float dmax = prune ? a.drift_max[0] : 0.f;
  const float cmax = a.cstat ? a.cstat[0] : 0.f;
  const float mrel = 4e-7f * float(a.d + 8);
  const float ueps2 = 1.f + 2e-6f + 1.2e-7f * float(a.d + 4);
  // one tile per wave step; the next tile's label, bounds and rows are prefetched while this
  // tile's center rows (L2) are fetched — issued first, so waiting for them (vmcnt retires in
  // order) never waits for the younger prefetch
  struct T {
    F x;
    int lab = 0;
    float2 bo = make_float2(0.f, -1.f);
  };
  auto load = [&](int64_t tt, T& d) {
    int64_t row = tt * 32 + r;
    row = row < a.n ? row : a.n - 1;
    d.lab = a.labels[row];
    if (a.bounds) d.bo = reinterpret_cast<const float2*>(a.bounds)[row];
    if constexpr (XB) {
      const __bf16* p = static_cast<const __bf16*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f = 16 * s + 8 * h;
        d.x.v[s] = (s < KS - 1 || f < a.ld) ? *reinterpret_cast<const bf16x8*>(p + 16 * s)
                                            : bf16x8{};
      }
    } else {
      const float* p = static_cast<const float*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int f = 16 * s + 8 * h + 4 * q;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (s < KS - 1 || f < a.ld) v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
          d.x.v[s][4 * q + 0] = v.x;
          d.x.v[s][4 * q + 1] = v.y;
          d.x.v[s][4 * q + 2] = v.z;
          d.x.v[s][4 * q + 3] = v.w;
        }
    }
  };
  auto step = [&](int64_t t, const T& c, T& nx, int64_t tn) {
    const int64_t row = t * 32 + r;
    const bool valid = row < a.n;
    int b = c.lab;
    if (b < 0 || b >= a.k) b = 0;
    float cv[KS][8];
    load_row8<KS>(a.centers + size_t(b) * DP + 8 * h, cv);
    load(tn, nx);
    float part = 0.f, px = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = c.x.at(s, j);
        const float e = xv - cv[s][j];
        part = fmaf(e, e, part);
        px = fmaf(xv, xv, px);
      }
    const float rowcost = part + __shfl_xor(part, 32, 64);
    const float nx2 = px + __shfl_xor(px, 32, 64);
    float2 bnew = make_float2(3.4e38f, -1.f);
    if (prune) {
      const float2 bo = c.bo;
      const float lp =
          bo.x >= 3e38f ? bo.y : fmaxf(sqrtf(fmaxf(bo.x, 0.f)) * (1.f - 1e-6f), bo.y);
      const float l = lp - dmax;
      if (l > 0.f && l * l - rowcost * ueps2 > mrel * (nx2 + cmax * cmax)) bnew.y = l;
    }
    if (valid && h == 0) {
      a.mindist[row] = rowcost;
      if (b != c.lab) a.labels[row] = b;  // labels stay (only an out-of-range one is reset)
      if (a.bounds) reinterpret_cast<float2*>(a.bounds)[row] = bnew;
    }
    if (a.tile_list && __any(valid && bnew.y < 0.f) && lane == 0)
      a.tile_list[atomicAdd(a.tile_count, 1u)] = static_cast<int32_t>(t);
  };
  const int64_t stride = int64_t(gridDim.x) * blockDim.x / 64;
  int64_t t = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
  T ta, tb;
  load(t, ta);
  for (; t < ntiles; t += 2 * stride) {  // wave-uniform trip count
    step(t, ta, tb, t + stride);
    if (t + stride >= ntiles) break;
    step(t + stride, tb, ta, t + 2 * stride);
  }
}

template <int KS, bool XB>
void launch_seed(const KMeansAssignArgs& a, hipStream_t s) {
  const int64_t tiles = (a.n + 31) / 32;
  const int grid = static_cast<int>(tiles / 4 + 1 < 8192 ? tiles / 4 + 1 : 8192);
  hipLaunchKernelGGL((oap_kmeans_seed_mindist<KS, XB>), dim3(grid), dim3(256), 0, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

template <bool XB>
void seed_xb(const KMeansAssignArgs& a, hipStream_t s) {
  switch ((a.d + 15) / 16) {
    case 1: launch_seed<1, XB>(a, s); break;
    case 2: launch_seed<2, XB>(a, s); break;
    case 3: launch_seed<3, XB>(a, s); break;
    case 4: launch_seed<4, XB>(a, s); break;
    case 5: launch_seed<5, XB>(a, s); break;
    case 6: launch_seed<6, XB>(a, s); break;
    case 7: launch_seed<7, XB>(a, s); break;
    case 8: launch_seed<8, XB>(a, s); break;
    default: OAP_THROW(ConfigError, "kmeans_seed_mindist: unsupported d=" << a.d);
  }
}

template <int KS, bool P, bool LA, bool B, bool XB, bool DEEP>
void launch4(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  const Smem L = smem_plan(16 * KS, a.kpad, a.k, a.d, P, LA, a.sums_too);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&oap_kmeans_assign_mfma<KS, P, LA, B, XB, DEEP>),
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_assign_mfma<KS, P, LA, B, XB, DEEP>), dim3(grid),
                     dim3(kThreads), L.total, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

// Prefetch depth (measured, profiles/ablate_kmeans_r24.json): one tile ahead for f32 and bf16
// rows (10.2 vs 10.4 and 8.1 vs 8.4 ms per 100M rows) — the third buffer costs more in
// register pressure than it hides.  The ablation bit 16 selects two-ahead (tuning A/B only).
template <int KS, bool P, bool LA, bool B, bool XB>
void launch3(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  constexpr bool kDeepOk = XB || KS <= 4;
  const bool deep = kDeepOk && (a.ablate & 16) != 0;
  if (deep)
    launch4<KS, P, LA, B, XB, kDeepOk>(a, grid, s);
  else
    launch4<KS, P, LA, B, XB, false>(a, grid, s);
}

template <int KS, bool XB>
void launch_ks(const KMeansAssignArgs& a, int grid, hipStream_t s, bool lds_acc) {
  if (a.precise) {
    if (lds_acc) launch3<KS, true, true, false, XB>(a, grid, s);
    else launch3<KS, true, false, false, XB>(a, grid, s);
  } else if (a.d + (XB ? 3 : 2) <= 16 * KS) {
    if (lds_acc) launch3<KS, false, true, true, XB>(a, grid, s);
    else launch3<KS, false, false, true, XB>(a, grid, s);
  } else {
    if (lds_acc) launch3<KS, false, true, false, XB>(a, grid, s);
    else launch3<KS, false, false, false, XB>(a, grid, s);
  }
}

template <bool XB>
void launch_xb(const KMeansAssignArgs& a, int grid, hipStream_t s, bool lds_acc) {
  const int dp = (a.d + 15) / 16 * 16;
  switch (dp / 16) {
    case 1: launch_ks<1, XB>(a, grid, s, lds_acc); break;
    case 2: launch_ks<2, XB>(a, grid, s, lds_acc); break;
    case 3: launch_ks<3, XB>(a, grid, s, lds_acc); break;
    case 4: launch_ks<4, XB>(a, grid, s, lds_acc); break;
    case 5: launch_ks<5, XB>(a, grid, s, lds_acc); break;
    case 6: launch_ks<6, XB>(a, grid, s, lds_acc); break;
    case 7: launch_ks<7, XB>(a, grid, s, lds_acc); break;
    case 8: launch_ks<8, XB>(a, grid, s, lds_acc); break;
    default: OAP_THROW(ConfigError, "kmeans_assign: unsupported d=" << a.d);
  }
}

// sum over rows of |x_row - c_{labels[row]}|^2: per row exactly the assign kernel's fp32 lane
// layout and summation order (bitwise its per-row cost), the centers staged in LDS (no L2 vector
// loads next to the row stream), rows prefetched two tiles ahead.  One fp64 partial per block
// (waves in index order) into slab.
template <int KS, bool XB>
__global__ __launch_bounds__(256) void oap_kmeans_label_cost(KMeansAssignArgs a, double* slab) {
  constexpr int DP = 16 * KS;
  using F = Frag<KS, XB>;
  extern __shared__ float4 dyn_lds[];
  float* cl = reinterpret_cast<float*>(dyn_lds);
  __shared__ double wsum[4];
  for (int i = threadIdx.x; i < a.k * DP / 4; i += blockDim.x)
    reinterpret_cast<float4*>(cl)[i] = reinterpret_cast<const float4*>(a.centers)[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (a.n + 31) / 32;
  struct T {
    F x;
    int lab = 0;
  };
  auto load = [&](int64_t tt, T& d) {
    int64_t row = tt * 32 + r;
    row = row < a.n ? (row < 0 ? 0 : row) : a.n - 1;
    d.lab = a.labels[row];
    if constexpr (XB) {
      const __bf16* p = static_cast<const __bf16*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f = 16 * s + 8 * h;
        d.x.v[s] = (s < KS - 1 || f < a.ld) ? *reinterpret_cast<const bf16x8*>(p + 16 * s)
                                            : bf16x8{};
      }
    } else {
      const float* p = static_cast<const float*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int f = 16 * s + 8 * h + 4 * q;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (s < KS - 1 || f < a.ld) v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
          d.x.v[s][4 * q + 0] = v.x;
          d.x.v[s][4 * q + 1] = v.y;
          d.x.v[s][4 * q + 2] = v.z;
          d.x.v[s][4 * q + 3] = v.w;
        }
    }
  };
  double my = 0.0;
  auto step = [&](int64_t t, const T& c, T& nx, int64_t tn) {
    load(tn, nx);  // prefetch: in flight while this tile computes
    const bool valid = t * 32 + r < a.n;
    int b = c.lab;
    if (b < 0 || b >= a.k) b = 0;
    float cv[KS][8];
    load_row8<KS>(cl + size_t(b) * DP + 8 * h, cv);
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = c.x.at(s, j) - cv[s][j];
        part = fmaf(e, e, part);
      }
    const float rowcost = part + __shfl_xor(part, 32, 64);
    if (valid && h == 0) my += double(rowcost);
  };
  const int64_t stride = int64_t(gridDim.x) * 4;
  int64_t t = int64_t(blockIdx.x) * 4 + wave;
  T ta, tb;
  load(t, ta);
  for (; t < ntiles; t += 2 * stride) {  // wave-uniform trip count
    step(t, ta, tb, t + stride);
    if (t + stride >= ntiles) break;
    step(t + stride, tb, ta, t + 2 * stride);
  }
  const double ws = wave_sum_f64(my);
  if (lane == 0) wsum[wave] = ws;
  __syncthreads();
  if (threadIdx.x == 0) slab[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

template <int KS, bool XB>
int launch_label_cost(const KMeansAssignArgs& a, double* slab, int max_blocks, hipStream_t s) {
  const size_t lds = size_t(a.k) * 16 * KS * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_label_cost<KS, XB>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(kLdsLimit - 1024)));
    attr_set = true;
  }
  const int64_t tiles = (a.n + 31) / 32;
  const int grid = static_cast<int>(std::min<int64_t>(tiles / 8 + 1, max_blocks));
  hipLaunchKernelGGL((oap_kmeans_label_cost<KS, XB>), dim3(grid), dim3(256), lds, s, a, slab);
  OAP_HIP_CHECK(hipGetLastError());
  return grid;
}

template <bool XB>
int label_cost_xb(const KMeansAssignArgs& a, double* slab, int max_blocks, hipStream_t s) {
  switch ((a.d + 15) / 16) {
    case 1: return launch_label_cost<1, XB>(a, slab, max_blocks, s);
    case 2: return launch_label_cost<2, XB>(a, slab, max_blocks, s);
    case 3: return launch_label_cost<3, XB>(a, slab, max_blocks, s);
    case 4: return launch_label_cost<4, XB>(a, slab, max_blocks, s);
    case 5: return launch_label_cost<5, XB>(a, slab, max_blocks, s);
    case 6: return launch_label_cost<6, XB>(a, slab, max_blocks, s);
    case 7: return launch_label_cost<7, XB>(a, slab, max_blocks, s);
    case 8: return launch_label_cost<8, XB>(a, slab, max_blocks, s);
    default: OAP_THROW(ConfigError, "kmeans_label_cost: unsupported d=" << a.d);
  }
}

}  // namespace

void launch_kmeans_seed_mindist(const KMeansAssignArgs& a, hipStream_t s) {
  if (a.n == 0) return;
  OAP_CHECK(a.d <= 128 && a.labels && a.mindist, "kmeans_seed_mindist: bad arguments");
  if (a.xbf16)
    seed_xb<true>(a, s);
  else
    seed_xb<false>(a, s);
}

int launch_kmeans_label_cost(const KMeansAssignArgs& a, double* slab, int max_blocks,
                             hipStream_t s) {
  OAP_CHECK(a.d <= 128 && a.labels && a.centers && a.n > 0, "kmeans_label_cost: bad arguments");
  if (size_t(a.k) * kmeans_dp(a.d) * sizeof(float) > kLdsLimit - 1024) return -1;
  return a.xbf16 ? label_cost_xb<true>(a, slab, max_blocks, s)
                 : label_cost_xb<false>(a, slab, max_blocks, s);
}

int kmeans_mfma_kmax(int d, bool precise) {
  if (d > 128) return 0;
  const int dp = (d + 15) / 16 * 16;
  int kp = 32;
  if (smem_plan(dp, kp, 0, d, precise, false).total > kLdsLimit) return 0;
  while (smem_plan(dp, kp + 32, 0, d, precise, false).total <= kLdsLimit) kp += 32;
  return precise ? kp : (kp < 1024 ? kp : 1024);  // fast path keys carry a 10-bit index
}

int kmeans_mfma_grid(int64_t n, int num_cus) {
  const int64_t tiles = (n + 31) / 32;
  const int64_t want = (tiles + kWaves - 1) / kWaves;
  const int64_t cap = num_cus > 256 ? num_cus : 256;
  return static_cast<int>(want < cap ? (want < 1 ? 1 : want) : cap);
}

void kmeans_defer_layout(int64_t n, int num_cus, int* grid, int64_t* seg_cap) {
  *grid = kmeans_mfma_grid(n, num_cus);
  *seg_cap = defer_segment((n + 31) / 32, *grid);
}

void launch_kmeans_assign_mfma(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  const int dp = (a.d + 15) / 16 * 16;
  const bool acc = a.accumulate && !a.merge;
  const bool lds_acc =
      acc && smem_plan(dp, a.kpad, a.k, a.d, a.precise, true, a.sums_too).total <= kLdsLimit;
  if (a.xbf16)
    launch_xb<true>(a, grid, s, lds_acc);
  else
    launch_xb<false>(a, grid, s, lds_acc);
}

}  // namespace kern
}  // namespace oap
