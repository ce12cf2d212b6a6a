// oap_kmeans_lloyd_t1 — the lean Lloyd-iteration kernel for MI355X (gfx950, CDNA4).
//
// One pass over the local rows per Lloyd iteration (the reference's hot loop
// is oneDAL's step1Local, mllib-dal/src/main/native/KMeansDALImpl.cpp:70-77): distances on the
// fp16 matrix cores, top-2 argmin in registers, exact fp32 per-row cost, fixed-point per-cluster
// sums in LDS.  It evaluates ONE product per k-step (tier 1) and never escalates a 32-row tile:
// a row whose top-2 gap is inside the tier's rigorous error bound is appended to its wave's
// segment of a deferral list and left untouched; oap_kmeans_exact_rows then re-decides exactly
// those rows with the exact fp32 MFMA argmin (v_mfma_f32_32x32x2_f32) and accumulates them.  So
// assignments are identical to an exact fp32 evaluation while the hot pass keeps a fixed,
// branch-free instruction stream whatever the data's share of near ties.
//
// Design points (CDNA4):
// * A wave owns a 32-row tile: lane (r = l & 31, h = l >> 5) holds features 16s + 8h + j of row
//   r.  The centroid plane (fp16 of -2 alpha c, plus bias features) is the MFMA A operand,
//   staged once per workgroup in LDS with an odd 16-byte-slot stride (conflict-free
//   ds_read_b128); rows (fp16 of alpha x) are the B operand straight from registers.
// * fp16, not bf16: 11 significant bits make tier 1's bound 8x tighter than bf16 at the same
//   MFMA rate (v_mfma_f32_32x32x16_f16), so several times fewer rows are deferred on
//   overlapping clusters.  alpha is a power of two with alpha * max|c| <= 2^8 (exact scaling),
//   so centers and typical rows sit in fp16's normal range; a row too large for it
//   (alpha^2 |x|^2 >= 2^20) is simply deferred.
// * Bias features carry both norms through the MFMA as hi/lo pairs scaled by 2^-4:
//   x' = [alpha x, 0.., 16, 16, hi, lo (alpha^2 |x|^2 / 16)], c' = [-2 alpha c, 0.., hi, lo
//   (alpha^2 |c|^2 / 16), 16, 16] (the four bias slots are the last four of the k-steps), so the
//   accumulator ends at alpha^2 |x - c|^2 with no seeding VALU and only the cross term carrying
//   fp16 error.
// * Only the fp16 plane lives in LDS: the fixed-point fp64 accumulator fits beside it and the
//   workgroup has 16 waves (4 per SIMD), so one wave's VALU epilogue, another's MFMAs and a
//   third's HBM loads overlap.
// * Each workgroup owns a contiguous range of ceil(tiles / grid) tiles (never more rows than
//   kmeans_rows_per_block_bound assumes: fixed-point exactness).  Delta passes read the
//   workgroup's own segment of the scan's tile list (oap_kmeans_lean_scan), so no counter is
//   shared by the whole grid.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <type_traits>

#include "kernels/kmeans_frag.h"
#include "kernels/kmeans_internal.h"
#include "runtime/knobs.h"

namespace oap {
namespace kern {

namespace {

using namespace kmdev;

// the kernel's helper lambdas share its argument block by reference: one of them left out of
// line (several call sites) would force a private copy of LeanArgs into scratch
#define OAP_AI __attribute__((always_inline))

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr float kBiasUnit = 16.f;  // bias features' unit (2^4)

// The kernel's own compact argument block (fewer SGPRs than KMeansAssignArgs).
struct LeanArgs {
  const void* x;
  const float* centers;
  const float* cnorm;
  const float* cstat;
  const float* scale;
  u64* sums;
  u64* counts;
  double* cost_slab;
  int32_t* labels;
  float* mindist;
  float2* bounds;
  float* xnorm;
  const int32_t* tile_list;   // delta: [grid][tiles_per_block] segments
  const unsigned* tile_count;  // delta: [grid]
  int32_t* defer_rows;
  unsigned* defer_row_count;
  u64* deferred_rows;
  int64_t n, seg_cap, tiles_per_block;
  int ld, d, k, kpad;
  int accumulate, sums_too, delta;
  int ablate;  // timing ablations only: 1 no accumulate, 2 no cost, 8 no distance, 16 no loads,
               // 32 minimal epilogue
  int refine;  // image passes: the refined deferral test (kmeans_frag.h refined_tt)
  // centroid-chunked pass (KMeansAssignArgs::chunk_mode): running top-2 keys per row, the
  // chunk's first global center, the global k, every center (the final chunk's exact cost)
  int2* keys;
  const float* centers_all;
  int kbase, kglob, chunk_mode;
  // resident fp16 operand image (f32 rows, KMeansAssignArgs::ximg): 1 = this full pass writes
  // it (and its scale), 2 = this pass reads it instead of the f32 rows
  _Float16* ximg;
  float* img_beta;
  int img_mode;
  // full passes over the rows: per-workgroup sum |x|^2 (fp64, exact squares) and the
  // provisional fixed-point bound check (KMeansAssignArgs::sq_slab / bound_flag / bound_inf)
  double* sq_slab;
  unsigned* bound_flag;
  float bound_inf;
  const int* halt;  // batched fits: set once the fit converged (the pass then does nothing)
};

struct LeanSmem {
  size_t plane, sc, acc, cnt, mv, wcost, wsq, total;
};

constexpr int kMoveCap = 64;  // per-wave staging slots for moved rows (delta passes)

__host__ __device__ inline LeanSmem lean_plan(int dp, int kpad, int k, int d, bool acc, bool sums,
                                              int waves, bool delta) {
  LeanSmem m;
  size_t off = 0;
  m.plane = 0;
  off = round16(size_t(kpad) * stride_bf16(dp) * 2);  // fp16 plane, same 2-byte layout
  m.sc = off;  // scales [dp], then per-wave 2 max |e_c| (kmdev::plane_resid2)
  off = round16(off + size_t(dp + kResidSlots) * 4);
  m.acc = off;
  if (acc && sums) off += size_t(k) * (d | 1) * 8;  // odd row stride: conflict-free ds_add_f64
  off = round16(off);
  m.cnt = off;
  if (acc) off += size_t(k) * 4;
  off = round16(off);
  m.mv = off;  // delta: per wave kMoveCap (row, new | old << 16) pairs
  if (acc && delta) off += size_t(waves) * kMoveCap * 8;
  m.wcost = off;
  off += size_t(waves) * 8;
  m.wsq = off;
  off += size_t(waves) * 8;
  m.total = round16(off);
  return m;
}

// alpha: power of two with alpha * cmax <= 2^8 (cmax = max |c|)
__device__ inline float lean_alpha(float cmax) {
  const float c = fmaxf(cmax, 1e-30f);
  return exp2f(floorf(log2f(256.f / c)));
}

__device__ inline void split_f16(float v, _Float16& hi, _Float16& lo) {
  hi = static_cast<_Float16>(v);
  lo = static_cast<_Float16>(v - static_cast<float>(hi));
}

// PF: 0 = no prefetch; 1 = double-buffered rows (prefetch the next tile into a second register
// set); 2 = the next tile is loaded into the current tile's registers as soon as its fp16
// operands are built, and the current tile is re-read (L2 / Infinity Cache) for the cost and
// the accumulation — a prefetch that costs no extra registers across the MFMA phase.
// COST: compute each row's exact cost (|x - c|^2 in fp32, direct form) and mindist; without it
// the row's f32 values are not needed after its fp16 operands are built (rows that accumulate
// re-read theirs), so PF 2 can reuse their registers, and the bounds' upper half comes from the
// tier-1 distance plus its error bound.
// SG: all KS fragment reads of a chunk in flight before its first MFMA.
// (Measured dead ends, in git history: two chunks per step, software-pipelined fragment reads,
// an accumulator-pipelined chunk loop (config 5: 293 vs 290 ms/iter, profiles/r5/
// cfg5_r5h_v12.json), a register-resident plane at 2 waves/SIMD (6% slower, profiles/r3/
// lean_variants_r3n_v11.json).)
template <int KS, bool XB, int WAVES, int PF, bool COST, bool SG = false>
__global__ __launch_bounds__(WAVES * 64, 1) void oap_kmeans_lloyd_t1(LeanArgs a) {
  constexpr int DP = 16 * KS;
  constexpr int NT = WAVES * 64;
  // image passes: tiles of operands in flight per wave (3 waves/SIMD have the registers for 2)
  constexpr int PD = WAVES == 12 ? 2 : 1;
  using F = Frag<KS, XB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (a.halt && *a.halt) return;
  const int kpad = a.kpad, k = a.k, d = a.d;
  // chunked passes: keys carry global center indices (kbase + in-chunk offset, < 1024); the
  // first and middle chunks only merge into the running keys, the last one finishes the rows
  const int kglob = a.chunk_mode ? a.kglob : k, kbase = a.chunk_mode ? a.kbase : 0;
  const float* cen_all = a.chunk_mode ? a.centers_all : a.centers;
  const bool keys_in = a.chunk_mode >= 2, keys_out = a.chunk_mode == 1 || a.chunk_mode == 2;
  const bool accumulate = a.accumulate != 0;
  const bool do_acc = accumulate && !(a.ablate & 1);
  const bool do_cost = !(a.ablate & 2);
  const bool do_dist = !(a.ablate & 8);
  const LeanSmem L = lean_plan(DP, kpad, k, d, accumulate, a.sums_too != 0, WAVES, a.delta != 0);
  const int sb = stride_bf16(DP);
  _Float16* ph = reinterpret_cast<_Float16*>(smem + L.plane);
  float* sc_l = reinterpret_cast<float*>(smem + L.sc);
  double* acc_l = reinterpret_cast<double*>(smem + L.acc);
  unsigned* cnt_l = reinterpret_cast<unsigned*>(smem + L.cnt);
  int2* mv_l = reinterpret_cast<int2*>(smem + L.mv) + (threadIdx.x >> 6) * kMoveCap;
  double* wcost = reinterpret_cast<double*>(smem + L.wcost);
  double* wsq = reinterpret_cast<double*>(smem + L.wsq);
  const int tid = threadIdx.x;
  const float cmax = a.cstat[0];
  float alpha = lean_alpha(cmax);
  // The operand image holds fp16(beta x) for a scale beta fixed when it was written (a quarter
  // of that pass's alpha: 4x headroom for the rows and 16x for later centers).  A pass reads it
  // only while the plane at that scale stays representable (beta max|c| <= 2^9: -2 beta c and
  // beta^2 |c|^2 / 16 inside fp16); otherwise it reads the f32 rows as usual.
  bool use_img = false;
  if constexpr (!XB && PF == 2 && !COST) {
    if (a.img_mode == 2 || a.img_mode == 3) {
      const float bt = a.img_beta[0];
      use_img = bt * cmax <= 512.f;
      if (use_img) alpha = bt;
      // img_mode 3: the f32-row fallback of oap_kmeans_lean_img (kmeans_lean_img.hip), which
      // ran this pass already whenever the image is usable
      if (use_img && a.img_mode == 3) return;
    }
  }
  const float a2 = alpha * alpha;
  const float inv_a2 = 1.f / a2;  // (a power of two: multiplying is the division, bitwise)
  const float beta_w = 0.25f * alpha;  // the scale a writing pass gives the image
  if (a.img_mode == 1 && blockIdx.x == 0 && tid == 0) a.img_beta[0] = beta_w;
  // (deferred_rows[2]: passes that actually read the image)
  if (use_img && blockIdx.x == 0 && tid == 0 && a.deferred_rows)
    atomicAdd(a.deferred_rows + 2, 1ull);

  // ---- stage c' = [-2 alpha c, 0 .., hi, lo (alpha^2 |c|^2 / 16), 16, 16] (fp16) once per
  // workgroup; the four bias features sit in the LAST four slots (DP - 4 .. DP - 1, d <= DP - 4
  // by the choice of KS), i.e. in the h = 1 lanes' j = 4..7 of the last k-step for every d: the
  // per-tile operand build then patches two fixed dwords instead of testing every slot against
  // a lane-dependent position (24 hoisted lane masks -> SGPR spills -> v_readlane per use)
  // (unconditional loads, unrolled: a thread's loads in flight together)
#pragma unroll 4
  for (int idx = tid; idx < kpad * DP; idx += NT) {
    const int c = idx / DP, f = idx - c * DP;
    const float cv = a.centers[idx], cnv = a.cnorm[c];
    _Float16 v;
    if (f < d) {
      v = static_cast<_Float16>(-2.f * alpha * cv);
    } else if (f == DP - 4 || f == DP - 3) {
      _Float16 hi, lo;
      // padded centers: the largest finite bias (their distance never wins)
      split_f16((c < k) ? a2 * cnv * (1.f / kBiasUnit) : 60000.f, hi, lo);
      v = (f == DP - 4) ? hi : lo;
    } else {
      v = static_cast<_Float16>(f >= DP - 2 ? kBiasUnit : 0.f);
    }
    ph[c * sb + f] = v;
  }
  for (int f = tid; f < DP; f += NT) sc_l[f] = (a.scale && a.sums_too && f < d) ? a.scale[f] : 0.f;
  // image passes: the plane's largest rounding residual for the refined deferral test
  // (kmeans_frag.h refined_tt), per wave
  // (and the image-writing pass, at its own alpha: its residuals are computed for the image)
  const bool refine = !XB && a.refine &&
                      (use_img ? d <= DP - kResidSlotOff : COST && a.img_mode == 1);
  if (refine) {
    const float r2w = plane_resid2(a.centers, DP, k, d, alpha, tid, NT);
    if ((tid & 63) == 0) sc_l[DP + (tid >> 6)] = r2w;
  }
  if (accumulate) {
    if (a.sums_too)
      for (int i = tid; i < k * (d | 1); i += NT) acc_l[i] = 0.0;
    for (int i = tid; i < k; i += NT) cnt_l[i] = 0u;
  }
  __syncthreads();

  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (uniform)
  const int r = lane & 31, h = lane >> 5;
  // tier-1 bound on two candidates' distance error (alpha^2 units): the cross term
  // 2 x 2 x 2^-10 |alpha c||alpha x| (fp16 products), fp16 subnormals d 2^-14, the bias pairs
  // 2^-21 (|c|^2 + |x|^2), fp32 accumulation 4e-5 (cmax^2 + |x|^2), plus the key truncation
  const float cm_s = alpha * cmax;
  // bf16 rows are exact in fp16 (8 significant bits, alpha a power of two; subnormal and
  // out-of-range rows are covered by thr_k / deferred), so only the centers' fp16 rounding
  // enters the cross term: half the f32-row coefficient (2 x 2^-10 instead of 2 x 2 x 2^-10)
  const float thr_c = (XB ? 0.0020f : 0.0040f) * cm_s;
  // (subnormals: 1.25 d 2^-14 — the image is fp16(alpha x) / 4, rounded twice where subnormal)
  const float thr_k = 6e-5f * cm_s * cm_s + float(d) * 7.8e-5f + 1e-30f;
  const float mrel = 4e-7f * float(d + 8);                // fp32 evaluation margin (bounds)
  float r2max = 0.f;
  if (refine)
    for (int w = 0; w < WAVES; ++w) r2max = fmaxf(r2max, sc_l[DP + w]);
  r2max = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(r2max)));
  // direct-form |x - c|^2 rounding; the bound square roots are v_sqrt_f32 (1 ulp: inside the
  // 1e-6 relative widening of both bounds)
  const float ueps = 1.f + 1e-6f + 6e-8f * float(d + 4);
  const int64_t ntiles_all = (a.n + 31) / 32;
  const bool listed = a.tile_list != nullptr;
  const int64_t T = a.tiles_per_block;
  const int64_t t0 = int64_t(blockIdx.x) * T;  // this workgroup's first tile
  const int64_t npos = listed ? int64_t(a.tile_count[blockIdx.x])
                              : (t0 < ntiles_all ? (ntiles_all - t0 < T ? ntiles_all - t0 : T) : 0);
  const int32_t* seg = listed ? a.tile_list + blockIdx.x * T : nullptr;
  const int64_t stride = WAVES;
  int64_t t = wave;
  // deferral: each wave owns a sub-segment of its workgroup's segment, filled in tile order, so
  // the list (and everything the exact pass sums over it) is deterministic
  const int64_t sub_cap = a.seg_cap / WAVES;
  int32_t* dseg = a.defer_rows + blockIdx.x * a.seg_cap + wave * sub_cap;
  unsigned n_def = 0;  // wave-uniform
  // per-row outputs through buffer resources over this workgroup's rows (listed tiles are the
  // workgroup's own too): predicated by offset, issued on every path (see buf_rsrc)
  const int64_t row0 = t0 * 32;
  const int64_t wrows = row0 < a.n ? (a.n - row0 < T * 32 ? a.n - row0 : T * 32) : 0;
  const __amdgpu_buffer_rsrc_t rs_lab =
      buf_rsrc(a.labels ? a.labels + row0 : nullptr, a.labels ? uint32_t(wrows * 4) : 0u);
  const __amdgpu_buffer_rsrc_t rs_bnd =
      buf_rsrc(a.bounds ? a.bounds + row0 : nullptr, a.bounds ? uint32_t(wrows * 8) : 0u);
  const __amdgpu_buffer_rsrc_t rs_def = buf_rsrc(dseg, uint32_t(sub_cap * 4));
  const __amdgpu_buffer_rsrc_t rs_md =
      buf_rsrc(a.mindist ? a.mindist + row0 : nullptr, a.mindist ? uint32_t(wrows * 4) : 0u);
  const __amdgpu_buffer_rsrc_t rs_xn =
      buf_rsrc(a.xnorm ? a.xnorm + t0 : nullptr, a.xnorm ? uint32_t((wrows + 31) / 32 * 4) : 0u);
  double my_cost = 0.0;
  double my_sq = 0.0;  // sum of the fp32 |x|^2 of this lane's rows (sq_slab)
  float my_nx2max = 0.f;  // largest fp32 |x|^2 of its rows (bound_flag[1])

  auto tile_of = [&](int64_t q) OAP_AI -> int64_t {
    if (npos == 0) return 0;  // (prefetch of an empty range: any real tile)
    q = q < npos ? q : npos - 1;
    if (!listed) return t0 + q;
    // (scalar load: the index is wave-uniform, and a vector load here would be the youngest
    // memory op, so the wait for it would also wait for the prefetch)
    typedef const int32_t __attribute__((address_space(4)))* seg_cptr;
    const int64_t tl = int64_t(((seg_cptr)(seg))[q]);
    return tl < 0 ? 0 : (tl < ntiles_all ? tl : ntiles_all - 1);
  };
  auto load_row = [&](int64_t row, F& dst) OAP_AI {
    if (a.ablate & 16) {  // timing ablation: no row loads (synthetic values)
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          uint32_t hsh = uint32_t(row) * 2654435761u ^ uint32_t(16 * s + j) * 2246822519u;
          hsh ^= hsh >> 15;
          hsh *= 2654435761u;
          const float v = float(hsh >> 8) * (20.f / 16777216.f) - 10.f;
          if constexpr (XB)
            dst.v[s][j] = static_cast<__bf16>(v);
          else
            dst.v[s][j] = v;
        }
      return;
    }
    if constexpr (XB) {
      const __bf16* p = static_cast<const __bf16*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f = 16 * s + 8 * h;
        dst.v[s] = (s < KS - 1 || f < a.ld) ? *reinterpret_cast<const bf16x8*>(p + 16 * s)
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
          dst.v[s][4 * q + 0] = v.x;
          dst.v[s][4 * q + 1] = v.y;
          dst.v[s][4 * q + 2] = v.z;
          dst.v[s][4 * q + 3] = v.w;
        }
    }
  };
  auto load_tile = [&](int64_t tile, F& dst) OAP_AI {
    const int64_t row = tile * 32 + r;
    load_row(row < a.n ? row : a.n - 1, dst);
  };
  // image layout: row-major [row][16 KS halves] (the MFMA B operand of each row: k-step s,
  // half h at halves 16 s + 8 h) — a row is one 16 KS-half record, so a listed (gathered) row
  // costs whole cache lines (kmeans_lean_img.hip's row-list passes)
  auto img_frag = [&](int64_t tile, int s) OAP_AI -> f16x8* {
    return reinterpret_cast<f16x8*>(a.ximg) + (tile * 32 + r) * (2 * KS) + 2 * s + h;
  };
  auto load_img = [&](int64_t tile, f16x8 (&dst)[KS]) OAP_AI {
#pragma unroll
    for (int s = 0; s < KS; ++s) dst[s] = *img_frag(tile, s);
  };

  // fixed-point accumulation of one row into cluster b (neg: subtract it)
  // fixed-point accumulation of one row: +x into cluster b, and -x into cluster bo when bo >= 0
  // (a moved row of a delta pass: the integers are formed once for both)
  auto add_row2 = [&](const F& xv, int b, int bo) OAP_AI {
    if (h == 0) {
      atomicAdd(&cnt_l[b], 1u);
      if (bo >= 0) atomicAdd(&cnt_l[bo], 0xffffffffu);
    }
    if (!a.sums_too) return;
    double* ap = acc_l + b * (d | 1) + 8 * h;
    double* aq = acc_l + (bo >= 0 ? bo : 0) * (d | 1) + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int f0 = 16 * s + 8 * h;
      const float4 s0 = *reinterpret_cast<const float4*>(sc_l + f0);
      const float4 s1 = *reinterpret_cast<const float4*>(sc_l + f0 + 4);
      const float scv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      // k-steps below KS-1 hold real features only (KS = ceil((d+4)/16)); the last one d - f0
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (s < KS - 1 || j < d - f0) {
          const double v = static_cast<double>(rintf(xv.at(s, j) * scv[j]));
          atomicAdd(ap + 16 * s + j, v);
          if (bo >= 0) atomicAdd(aq + 16 * s + j, -v);
        }
    }
  };
  auto add_row = [&](const F& xv, int b) OAP_AI { add_row2(xv, b, -1); };

  // delta passes: a tile's few moved rows would each cost the whole wave 2 KS x 8 predicated
  // LDS atomics; instead they are staged in the wave's LDS slots and accumulated 32 at a time
  // with every lane busy (rows re-read from L2: their tile was just streamed)
  unsigned n_mv = 0;  // wave-uniform
  u64 moved_total = 0;
  auto flush_moved = [&](unsigned cnt) OAP_AI {  // accumulate staged entries [0, min(cnt, 32))
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool on = unsigned(r) < cnt;
    const int2 e = mv_l[on ? r : 0];
    if (on) {
      F xr;
      load_row(int64_t(e.x), xr);
      add_row2(xr, e.y & 0xffff, e.y >> 16);
    }
    if (cnt > 32) {  // slide the rest down (read all before any write: in-order LDS)
      const int2 rest = mv_l[32 + r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (h == 0 && unsigned(r) < cnt - 32) mv_l[r] = rest;
    }
    moved_total += cnt < 32 ? cnt : 32;
  };

  // fp16 operand of s * x with the bias slots [16, 16, hi, lo (s^2 |x|^2 / 16)] (nx2 = |x|^2)
  auto build_operand = [&](const F& x, float s_, float nx2, f16x8 (&out)[KS]) OAP_AI {
    _Float16 nh, nl;
    split_f16(s_ * s_ * nx2 * (1.f / kBiasUnit), nh, nl);
    const _Float16 unit = static_cast<_Float16>(kBiasUnit);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      f16x8 v;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {  // v_pk_mul_f32 + v_cvt_pk_f16_f32 (RNE): 1 op / value
        const f32x2 p = f32x2{x.at(s, j), x.at(s, j + 1)} * s_;
        const f16x2 q = __builtin_convertvector(p, f16x2);
        v[j] = q[0];
        v[j + 1] = q[1];
      }
      if (s == KS - 1) {  // h = 1 lanes: slots 4..7 = [16, 16, hi, lo] (x is 0 there)
        v[4] = h ? unit : v[4];
        v[5] = h ? unit : v[5];
        v[6] = h ? nh : v[6];
        v[7] = h ? nl : v[7];
      }
      out[s] = v;
    }
  };

  // img_t: std::true_type — the operands come from the resident image (xi: this tile's, xin:
  // where the next tile's are loaded once xi is copied), the f32 rows are read only by the
  // accumulation
  auto process = [&](auto img_t, const int64_t pos, const int64_t tile, F& x, F& xn,
                     const int64_t pf, f16x8 (&xi)[KS], f16x8 (&xin)[KS]) OAP_AI {
    constexpr bool IMG = decltype(img_t)::value;
    const int64_t row = tile * 32 + r;
    const bool valid = pos < npos && row < a.n;
    if constexpr (!IMG && PF == 1) load_tile(tile_of(pf), xn);  // next tile: in flight
    // running pair of a chunked pass (one half takes it: no duplicate), merged after the chunk
    // loop — loaded here, ahead of the next tile's prefetch, so no wait in the loop covers the
    // prefetch (s_waitcnt vmcnt counts in issue order)
    int2 kin = make_int2(0x7fffffff, 0x7fffffff);
    if (!IMG && keys_in && h == 0 && valid) kin = a.keys[row];
    const uint32_t roff = uint32_t(row - row0);  // (valid rows: this workgroup's)
    // image passes are always delta passes of a single-launch fit: no chunk keys, no timing
    // ablations — compile-time constants there (fewer live uniform switches)
    const bool dl = IMG || a.delta;
    int old = buf_load_b32(rs_lab, roff * 4, dl && valid);
    old = (dl && valid) ? old : -1;
    // MFMA B operand: fp16 of alpha x with the bias slots [16, 16, hi, lo (alpha^2 |x|^2 / 16)]
    f16x8 xh[KS];
    float nx2_s;
    float e2a = 0.f;  // (image-writing passes: the row's alpha-scale rounding residual^2)
    if constexpr (IMG) {
#pragma unroll
      for (int s = 0; s < KS; ++s) xh[s] = xi[s];
      if constexpr (PD == 2) {  // xi takes the next tile's (landed or in flight), xin pf's
#pragma unroll
        for (int s = 0; s < KS; ++s) xi[s] = xin[s];
      }
      load_img(tile_of(pf), xin);  // operands PD tiles ahead (PD 1: xin is xi): in flight
      // alpha^2 |x|^2 from the bias pair (h = 1 lanes' slots 6, 7 of the last k-step)
      const float mine = kBiasUnit * (static_cast<float>(xh[KS - 1][6]) +
                                      static_cast<float>(xh[KS - 1][7]));
      const float other = xor32_f(mine);
      nx2_s = h ? mine : other;
    } else {
      float nx2 = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) nx2 = fmaf(x.at(s, j), x.at(s, j), nx2);
      nx2 += xor32_f(nx2);
      // the row's fp32 |x|^2 (a chain of <= 8 KS + 1 roundings) summed in fp64: the final cost's
      // sum_i |x_i|^2 at the per-row accuracy of the cost pass it replaces, for one add a tile
      // (exact fp64 squares cost this pass ~10%: +1 ms at the headline)
      if (a.sq_slab && valid && h == 0) my_sq += static_cast<double>(nx2);
      // provisional fixed-point bounds: a value at or beyond the smallest column bound makes
      // the host check the column maxima (max3 chains with |.| modifiers: 16 VALU a tile)
      if (a.bound_flag) {
        float m = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; j += 2)
            m = fmaxf(m, fmaxf(fabsf(x.at(s, j)), fabsf(x.at(s, j + 1))));
        if (valid && !(m < a.bound_inf)) atomicOr(a.bound_flag, 1u);
        my_nx2max = fmaxf(my_nx2max, valid ? nx2 : 0.f);
      }
      // per-tile max |x|^2 (the delta scan's pruning margin): the reduction only where it is
      // asked for, the store predicated by offset (issued on every path, see buf_rsrc)
      float tmax = nx2;
      if (a.xnorm) {
#pragma unroll
        for (int m = 16; m >= 1; m >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, m, 64));
      }
      buf_store_b32(rs_xn, uint32_t(tile - t0) * 4u, __float_as_int(tmax),
                    a.xnorm && lane == 0 && pos < npos);
      nx2_s = a2 * nx2;
      build_operand(x, alpha, nx2, xh);
      if constexpr (!XB && COST) {  // (full passes compute the cost)
        if (a.img_mode == 1 && pos < npos) {  // write the image (every lane of a real tile)
          // The decision operand's rounding residual |fp16(alpha x) - alpha x|^2 (exact
          // differences, packed fp32 squares; the bias slots of the last k-step excluded) refines
          // this pass's deferral test and bounds the image's: the image is xh / 4 = fp16(beta x)
          // exactly wherever beta x is a normal fp16 (elsewhere one more rounding, <= 2^-25 a
          // feature), its residual norm <= |e_alpha| / 4 + d 2^-25 — into the pad slot DP - 5.
          f32x2 e2v = {0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
              const f32x2 p = f32x2{x.at(s, j), x.at(s, j + 1)} * alpha;
              const f32x2 q = (s == KS - 1 && j >= 4)
                                  ? __builtin_convertvector(__builtin_convertvector(p, f16x2),
                                                            f32x2)
                                  : f32x2{static_cast<float>(xh[s][j]),
                                          static_cast<float>(xh[s][j + 1])};
              const f32x2 e = q - p;
              e2v = e * e + e2v;
            }
          const float e2p = e2v[0] + e2v[1];
          e2a = e2p + xor32_f(e2p);
          const bool wres = d <= DP - kResidSlotOff;
          const _Float16 rs16 = resid_f16_norm_up(
              0.25f * __builtin_amdgcn_sqrtf(e2a * 1.0001f) * 1.000001f + float(d) * 3e-8f);
          _Float16 nh, nl;
          split_f16(beta_w * beta_w * nx2 * (1.f / kBiasUnit), nh, nl);
          const _Float16 quarter = static_cast<_Float16>(0.25f);
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            f16x8 v = xh[s] * quarter;
            if (s == KS - 1) {
              v[3] = (h && wres) ? rs16 : v[3];
              v[4] = h ? static_cast<_Float16>(kBiasUnit) : v[4];
              v[5] = h ? static_cast<_Float16>(kBiasUnit) : v[5];
              v[6] = h ? nh : v[6];
              v[7] = h ? nl : v[7];
            }
            *img_frag(tile, s) = v;
          }
        }
      }
    }
    if constexpr (!IMG && PF == 2) load_tile(tile_of(pf), x);  // x now carries the next tile
    // ---- tier 1: one fp16 product per k-step; top-2 on integer keys (the distance's bits with
    // the low 10 mantissa bits replaced by the in-chunk offset; value order, lowest index first)
    int k1 = 0x7fffffff, k2 = 0x7fffffff;
    auto mfma_chunk = [&](int c0, f32x16& acc) OAP_AI {
      const _Float16* ap = ph + size_t(c0 + r) * sb + 8 * h;
      f16x8 av[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) av[s] = *reinterpret_cast<const f16x8*>(ap + 16 * s);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[0], xh[0], f32x16{}, 0, 0, 0);
#pragma unroll
      for (int s = 1; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s], xh[s], acc, 0, 0, 0);
      if constexpr (SG) {
        // all KS fragment reads in flight before the first MFMA (the default schedule reuses
        // one register quad and waits on each read in turn)
        __builtin_amdgcn_sched_group_barrier(0x100, KS, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
      }
    };
    auto epilogue = [&](int c0, const f32x16& acc) OAP_AI {
      if (!IMG && (a.ablate & 32)) {  // timing ablation: one op per chunk
        k1 = min(k1, (__float_as_int(acc[0]) & ~0x3ff) | (c0 + 4 * h));
        return;
      }
      // padded centers carry the largest finite bias: they never win, so no chunk needs a
      // branch for them.  Keys (one v_and_or each) fold into the chunk's top-2 two at a time:
      // with t1 <= t2, the smallest of {t1, t2, a, b} is min3(t1, a, b) and the second smallest
      // min(t2, med3(t1, a, b)) — 3 VALU per 2 keys (the old 4-lane tree took 4 per 2 keys
      // plus 12 to merge its lanes)
      int key[16];
#pragma unroll
      for (int e = 0; e < 16; ++e)
        key[e] = (__float_as_int(acc[e]) & ~0x3ff) | (8 * (e >> 2) + (e & 3));
      int t1 = min(key[0], key[1]), t2 = max(key[0], key[1]);
#pragma unroll
      for (int e = 2; e < 16; e += 2) {
        t2 = min(t2, med3_i32_pure(t1, key[e], key[e + 1]));
        t1 = min(min(t1, key[e]), key[e + 1]);
      }
      const int base = c0 + 4 * h + (IMG ? 0 : kbase);  // disjoint from every in-chunk offset
      const int i1 = t1 | base, i2 = t2 | base;
      k2 = min(max(k1, i1), min(k2, i2));
      k1 = min(k1, i1);
    };
    bool unsure;
    float b1 = 0.f, b2 = 0.f, tt = 0.f;
    if (IMG || do_dist) {
      int c0 = 0;
      for (; c0 < kpad; c0 += 32) {  // other waves' MFMAs overlap this epilogue
        f32x16 acc;
        mfma_chunk(c0, acc);
        epilogue(c0, acc);
      }
      k2 = min(max(k1, kin.x), min(k2, kin.y));  // (top-2 of the union: order-free)
      k1 = min(k1, kin.x);
      const int o1 = xor32_i(k1), o2 = xor32_i(k2);
      k2 = min(max(k1, o1), min(k2, o2));
      k1 = min(k1, o1);
      if (!IMG && keys_out) {  // not the last chunk: carry the pair to the next one
        if (h == 0 && valid) a.keys[row] = make_int2(k1, k2);
        return;
      }
      b1 = __int_as_float(k1 & ~0x3ff);
      b2 = __int_as_float(k2 & ~0x3ff);
      tt = fmaf(thr_c, __builtin_amdgcn_sqrtf(nx2_s), thr_k) + 5e-5f * nx2_s +
           2.5e-4f * fabsf(b2);
      // rows beyond fp16's comfortable range (alpha |x| >= 2^10) are always re-decided
      unsure = valid && (!(b2 - b1 > tt) || !(nx2_s < 1048576.f));
      // image passes: the refined test on the row's own residual (kmeans_frag.h refined_tt;
      // wave-uniform: the residual's exchange needs both halves)
      if ((IMG || (COST && !XB)) && refine && __ballot(unsure) != 0ull) {
        float exn;
        if constexpr (IMG) {
          const float em = static_cast<float>(xh[KS - 1][3]);
          const float eo = xor32_f(em);
          exn = h ? em : eo;
        } else {
          exn = __builtin_amdgcn_sqrtf(e2a * 1.0001f) * 1.001f + 1e-30f;
        }
        const float rest = thr_k + 5e-5f * nx2_s + 2.5e-4f * fabsf(b2);
        const float tr = refined_tt(b1, b2, tt, rest, nx2_s, exn, r2max);
        unsure = unsure && !(b1 >= 0.f && b2 - b1 > tr && nx2_s < 1048576.f);
      }
    } else {
      k1 = r % k;
      b2 = 3e38f;
      unsure = false;
    }
    // ---- defer unsure rows to the exact re-decision (wave-private sub-segment, in order)
    const unsigned long long um = __ballot(unsure && h == 0);
    buf_store_b32(rs_def, (n_def + __popcll(um & ((1ull << lane) - 1ull))) * 4u,
                  static_cast<int32_t>(row), unsure && h == 0);
    n_def += static_cast<unsigned>(__popcll(um));
    const bool done = valid && !unsure;
    int b = k1 & 0x3ff;
    b = (b < (IMG ? k : kglob)) ? b : 0;  // only for degenerate (NaN / all-inf) inputs
    const bool acc_row = done && (IMG ? accumulate : do_acc) && (!dl || (old >= 0 && old != b));
    if (dl) {  // stage moved rows (wave-private slots, in row order)
      const unsigned long long mm = __ballot(acc_row && h == 0);
      if (mm) {
        if (acc_row && h == 0)
          mv_l[n_mv + __popcll(mm & ((1ull << lane) - 1ull))] =
              make_int2(static_cast<int>(row), b | (min(old, k - 1) << 16));
        n_mv += static_cast<unsigned>(__popcll(mm));
        if (n_mv >= 32) {
          flush_moved(n_mv);
          n_mv -= 32;
        }
      }
    }
    if constexpr (COST) {
      F xr_buf;
      if constexpr (PF == 2) load_tile(tile, xr_buf);  // re-read this tile (cache-resident)
      const F& xr = (PF == 2) ? xr_buf : x;
      float cb[KS][8];
      if (do_cost) {
        load_row8<KS>(cen_all + size_t(b) * DP + 8 * h, cb);  // L2-resident; lands under adds
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) cb[s][j] = 0.f;
      }
      if (acc_row && !a.delta) add_row(xr, b);
      float part = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = xr.at(s, j) - cb[s][j];
          part = fmaf(e, e, part);
        }
      const float rowcost = part + xor32_f(part);
      const bool out = done && h == 0;
      buf_store_b32(rs_lab, roff * 4, b, out);
      // every other candidate's alpha^2 distance is >= b2 - tt; back to data units
      const float lo = (b2 - (tt + mrel * (nx2_s + cm_s * cm_s))) * inv_a2;
      buf_store_f2(rs_bnd, roff * 8,
                   make_float2(__builtin_amdgcn_sqrtf(rowcost) * ueps + 1e-30f,
                               __builtin_amdgcn_sqrtf(fmaxf(lo, 0.f)) * (1.f - 1e-6f)),
                   out);
      buf_store_b32(rs_md, roff * 4, __float_as_int(rowcost), out);
      if (out) my_cost += double(rowcost);
    } else {
      if (acc_row && !dl) {  // only rows that add re-read (x may hold the next tile)
        F xr;
        if constexpr (PF == 2)
          load_tile(tile, xr);
        else
          xr = x;
        add_row(xr, b);
      }
      const bool out = done && h == 0;
      buf_store_b32(rs_lab, roff * 4, b, out);
      // the pick's alpha^2 distance is <= b1 + tt, every other one >= b2 - tt
      const float mg = mrel * (nx2_s + cm_s * cm_s);
      const float up = (b1 + tt + mg) * inv_a2, lo = (b2 - (tt + mg)) * inv_a2;
      buf_store_f2(rs_bnd, roff * 8,
                   make_float2(
                       __builtin_amdgcn_sqrtf(fmaxf(up, 0.f)) * (1.f + 1e-6f) + 1e-30f,
                       __builtin_amdgcn_sqrtf(fmaxf(lo, 0.f)) * (1.f - 1e-6f)),
                   out);
    }
  };

  const std::false_type rows_t{};
  f16x8 no_img[KS];  // (unused by the f32-row passes)
  if (use_img) {
    // image passes: the tile's operand fragments are copied out of the load registers (KS x 4
    // moves) and the next tile's loads go straight into them, in flight under this tile (one
    // call site: a ping-pong of two register sets needs two inlined copies of the pass body)
    if constexpr (!XB && PF == 2 && !COST) {
      F unused;
      f16x8 ia[KS], ib[KS];
      load_img(tile_of(t), ia);
      if constexpr (PD == 2) load_img(tile_of(t + stride), ib);
      for (; t < npos; t += stride)  // t is wave-uniform: every branch stays uniform
        process(std::true_type{}, t, tile_of(t), unused, unused, t + PD * stride, ia,
                PD == 2 ? ib : ia);
    }
  } else if constexpr (PF == 1) {
    F xa, xb;
    load_tile(tile_of(t), xa);
    for (; t < npos; t += 2 * stride) {  // t is wave-uniform: every branch stays uniform
      process(rows_t, t, tile_of(t), xa, xb, t + stride, no_img, no_img);
      if (t + stride >= npos) break;
      process(rows_t, t + stride, tile_of(t + stride), xb, xa, t + 2 * stride, no_img, no_img);
    }
  } else if constexpr (PF == 2) {
    F xa;
    load_tile(tile_of(t), xa);
    for (; t < npos; t += stride)
      process(rows_t, t, tile_of(t), xa, xa, t + stride, no_img, no_img);
  } else {
    F xa;
    int64_t tl = tile_of(t);
    for (; t < npos; t += stride) {
      const int64_t tcur = tl;
      load_tile(tcur, xa);
      tl = tile_of(t + stride);  // listed passes: the next tile index lands under this tile
      process(rows_t, t, tcur, xa, xa, 0, no_img, no_img);
    }
  }

  if (n_mv) flush_moved(n_mv);
  // ---- deterministic per-block cost (fixed shuffle tree, waves in index order), flushes
  const double wsum = wave_sum_f64(my_cost);
  const double wsq_sum = a.sq_slab ? wave_sum_f64(my_sq) : 0.0;
  if (a.bound_flag) {  // the rows' largest norm (non-negative floats order as their bits)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) my_nx2max = fmaxf(my_nx2max, __shfl_xor(my_nx2max, m, 64));
    if (lane == 0 && my_nx2max > 0.f) atomicMax(a.bound_flag + 1, __float_as_uint(my_nx2max));
  }
  if (lane == 0) {
    wcost[wave] = wsum;
    wsq[wave] = wsq_sum;
    a.defer_row_count[blockIdx.x * kDeferSubs + wave] = n_def;
    if (a.deferred_rows && n_def) atomicAdd(a.deferred_rows, u64(n_def));
    if (a.deferred_rows && moved_total) atomicAdd(a.deferred_rows + 1, moved_total);
  }
  __syncthreads();
  if (tid == 0 && a.cost_slab) {
    double tot = 0.0;
    for (int w = 0; w < WAVES; ++w) tot += wcost[w];
    a.cost_slab[blockIdx.x] = tot;
  }
  if (tid == 0 && a.sq_slab) {
    double tot = 0.0;
    for (int w = 0; w < WAVES; ++w) tot += wsq[w];
    a.sq_slab[blockIdx.x] = tot;
  }
  if (accumulate) {
    for (int i = tid; a.sums_too && i < k * d; i += NT) {
      const int c = i / d, f = i - c * d;
      const double v = acc_l[c * (d | 1) + f];  // an exact integer, |v| < 2^53
      if (v != 0.0) atomicAdd(&a.sums[i], static_cast<u64>(static_cast<long long>(v)));
    }
    for (int i = tid; i < k; i += NT) {
      const int c = static_cast<int>(cnt_l[i]);  // signed: delta mode subtracts
      if (c) atomicAdd(&a.counts[i], static_cast<u64>(static_cast<long long>(c)));
    }
  }
}

template <int KS, bool XB, int WAVES, int PF, bool COST, bool SG = false>
void launch_lean(const LeanArgs& a, int grid, hipStream_t s) {
  const LeanSmem L =
      lean_plan(16 * KS, a.kpad, a.k, a.d, a.accumulate, a.sums_too, WAVES, a.delta != 0);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&oap_kmeans_lloyd_t1<KS, XB, WAVES, PF, COST, SG>),
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_lloyd_t1<KS, XB, WAVES, PF, COST, SG>), dim3(grid),
                     dim3(WAVES * 64), L.total, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

// Workgroup shapes (one workgroup per CU: the LDS plan), fragment reads grouped ahead of each
// MFMA chain: variant 6, 4 waves/SIMD; variant 8, 3 waves/SIMD (rows of 7-8 k-steps, where 128
// registers spill).  With the cost the rows stay in registers; without, the next tile is
// prefetched into them (PF 2).
template <int KS, bool XB>
void launch_lean_v(const LeanArgs& a, int grid, int variant, bool cost, hipStream_t s) {
  if (variant == 8) {
    if (cost) launch_lean<KS, XB, 12, 0, true, true>(a, grid, s);
    else launch_lean<KS, XB, 12, 2, false, true>(a, grid, s);
  } else {
    if (cost) launch_lean<KS, XB, 16, 0, true, true>(a, grid, s);
    else launch_lean<KS, XB, 16, 2, false, true>(a, grid, s);
  }
}

template <bool XB>
void launch_lean_xb(const LeanArgs& a, int grid, int variant, bool cost, hipStream_t s) {
  switch ((a.d + 4 + 15) / 16) {
    case 1: launch_lean_v<1, XB>(a, grid, variant, cost, s); break;
    case 2: launch_lean_v<2, XB>(a, grid, variant, cost, s); break;
    case 3: launch_lean_v<3, XB>(a, grid, variant, cost, s); break;
    case 4: launch_lean_v<4, XB>(a, grid, variant, cost, s); break;
    case 5: launch_lean_v<5, XB>(a, grid, variant, cost, s); break;
    case 6: launch_lean_v<6, XB>(a, grid, variant, cost, s); break;
    case 7: launch_lean_v<7, XB>(a, grid, variant, cost, s); break;
    case 8: launch_lean_v<8, XB>(a, grid, variant, cost, s); break;
    default: OAP_THROW(ConfigError, "kmeans_lloyd: unsupported d=" << a.d);
  }
}

// ---------------------------------------------------------------- exact re-decision
// The rows the lean pass deferred, 32 per wave step (gathered by index), re-decided with the
// exact fp32 MFMA argmin (v_mfma_f32_32x32x2_f32, the PRECISE kernel's arithmetic: bitwise its
// answer) against fp32 centers staged in LDS, then finished as the assign kernels finish a row:
// exact cost, labels / mindist / bounds, fixed-point statistics (LDS fp64 accumulator when it
// fits, else global int64 atomics).  Rows: the lean workgroup's deferral sub-segments in order
// (deterministic).
// waves per workgroup: 16 (4 per SIMD with the one workgroup the LDS plan allows per CU) where
// the kernel fits 128 VGPRs, else 8 — the pass is latency bound, not MFMA bound
constexpr int kExactWaves = 16;  // (the most: LDS slots)
__host__ __device__ constexpr int exact_waves(int ks, bool xb) {
  return (xb ? ks <= 5 : ks <= 4) ? 16 : 8;
}

struct ExactSmem {
  size_t ct, cn, sc, acc, cnt, wc, pref, total;
  bool lds_acc;
};

__host__ __device__ inline ExactSmem exact_plan(int kpad, int k, int d, bool acc, bool sums) {
  const int dp = (d + 15) / 16 * 16;
  ExactSmem m;
  size_t off = 0;
  m.ct = 0;
  off = round16(size_t(kpad) * (dp + 4) * 4);  // row stride dp + 4: 16-byte reads spread banks
  m.cn = off;
  off = round16(off + size_t(kpad) * 4);
  m.sc = off;
  off = round16(off + size_t(dp) * 4);
  m.acc = off;
  const size_t base = off;
  size_t accb = (acc && sums) ? size_t(k) * (d | 1) * 8 : 0;
  size_t cntb = acc ? size_t(k) * 4 : 0;
  m.lds_acc = acc && round16(base + accb) + round16(cntb) + 256 <= kLdsLimit - 1024;
  if (!m.lds_acc) accb = cntb = 0;
  off = round16(off + accb);
  m.cnt = off;
  off = round16(off + cntb);
  m.wc = off;
  off += kExactWaves * 8;
  m.pref = off;
  off += (kDeferSubs + 1) * 4;
  m.total = round16(off);
  return m;
}

template <int KS, bool XB>
__global__ __launch_bounds__(exact_waves(KS, XB) * 64) void oap_kmeans_exact_rows(
    KMeansAssignArgs a) {
  constexpr int EW = exact_waves(KS, XB);
  constexpr int DP = 16 * KS;
  constexpr int CS = DP + 4;
  using F = Frag<KS, XB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (a.halt && *a.halt) return;
  const int k = a.k, d = a.d, kpad = a.kpad;
  // chunked passes: the running (best, second, index) of each deferred row lives in xstate
  // between the chunk launches; the last chunk finishes the rows against every center
  const int kglob = a.chunk_mode ? a.kglob : k;
  const bool st_in = a.chunk_mode >= 2, st_out = a.chunk_mode == 1 || a.chunk_mode == 2;
  float2* xst = reinterpret_cast<float2*>(a.xstate);  // (best, index): no bounds when chunked
  const bool accumulate = a.accumulate;
  const ExactSmem L = exact_plan(kpad, k, d, accumulate, a.sums_too);
  float* ct = reinterpret_cast<float*>(smem + L.ct);
  float* cn = reinterpret_cast<float*>(smem + L.cn);
  float* sc_l = reinterpret_cast<float*>(smem + L.sc);
  double* acc_l = reinterpret_cast<double*>(smem + L.acc);
  unsigned* cnt_l = reinterpret_cast<unsigned*>(smem + L.cnt);
  double* wc = reinterpret_cast<double*>(smem + L.wc);
  unsigned* pref = reinterpret_cast<unsigned*>(smem + L.pref);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  constexpr int NT = EW * 64;
  // (the sub-segment counts loaded in parallel, then summed in LDS: one load latency, not 16)
  if (tid < a.row_subs) pref[tid + 1] = a.row_count[blockIdx.x * kDeferSubs + tid];
  __syncthreads();
  if (tid == 0) {
    pref[0] = 0u;
    for (int w = 0; w < a.row_subs; ++w) pref[w + 1] += pref[w];
  }
  __syncthreads();
  const unsigned total = pref[a.row_subs];
  if (total == 0) {  // nothing deferred here: still write this block's (zero) cost partial
    if (tid == 0 && a.cost_slab) a.cost_slab[blockIdx.x] = 0.0;
    return;
  }
#pragma unroll 8
  for (int i = tid; i < kpad * DP; i += NT) {
    const int c = i / DP, f = i - c * DP;
    ct[c * CS + f] = a.centers[i];
  }
  for (int c = tid; c < kpad; c += NT) cn[c] = (c < k) ? a.cnorm[c] : 1e30f;
  for (int f = tid; f < DP; f += NT) sc_l[f] = (a.scale && a.sums_too && f < d) ? a.scale[f] : 0.f;
  if (L.lds_acc) {
    if (a.sums_too)
      for (int i = tid; i < k * (d | 1); i += NT) acc_l[i] = 0.0;
    for (int i = tid; i < k; i += NT) cnt_l[i] = 0u;
  }
  __syncthreads();
  const int64_t sub = a.row_seg_cap / a.row_subs;
  const float cmax = a.cstat[0];
  const float mrel = 4e-7f * float(d + 8);
  const float ueps = 1.f + 1e-6f + 6e-8f * float(d + 4);
  const int64_t ngroups = (int64_t(total) + 31) / 32;
  auto slot_at = [&](int64_t i) -> int64_t {  // list slot of this workgroup's i-th row (clamped)
    i = i < int64_t(total) ? i : int64_t(total) - 1;
    int w = 0;
    while (w + 1 < a.row_subs && int64_t(pref[w + 1]) <= i) ++w;
    return int64_t(blockIdx.x) * a.row_seg_cap + w * sub + (i - pref[w]);
  };
  auto row_at = [&](int64_t i) -> int64_t {  // i-th deferred row of this workgroup (clamped)
    return int64_t(a.row_list[slot_at(i)]);
  };
  auto load_rows = [&](int64_t g, F& dst) {
    const int64_t row = row_at(g * 32 + r);
    if constexpr (XB) {
      const __bf16* p = static_cast<const __bf16*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f = 16 * s + 8 * h;
        dst.v[s] = (s < KS - 1 || f < a.ld) ? *reinterpret_cast<const bf16x8*>(p + 16 * s)
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
          dst.v[s][4 * q + 0] = v.x;
          dst.v[s][4 * q + 1] = v.y;
          dst.v[s][4 * q + 2] = v.z;
          dst.v[s][4 * q + 3] = v.w;
        }
    }
  };
  auto add_row = [&](const F& xv, int b, bool neg) {
    if (L.lds_acc) {
      if (h == 0) atomicAdd(&cnt_l[b], neg ? 0xffffffffu : 1u);
    } else if (h == 0) {
      atomicAdd(&a.counts[b], neg ? ~0ull : 1ull);
    }
    if (!a.sums_too) return;
    const float sgn = neg ? -1.f : 1.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 16 * s + 8 * h + j;
        if (f < d) {
          const float q = sgn * rintf(xv.at(s, j) * sc_l[f]);
          if (L.lds_acc)
            atomicAdd(acc_l + b * (d | 1) + f, static_cast<double>(q));
          else
            atomicAdd(&a.sums[size_t(b) * d + f], static_cast<u64>(static_cast<long long>(q)));
        }
      }
  };
  double my_cost = 0.0;
  // the previous labels of a group's rows (delta passes), gathered with its rows: a group ahead
  auto load_old = [&](int64_t gg) -> int {
    const int64_t ii = gg * 32 + r;
    return (a.delta && ii < int64_t(total)) ? a.labels[row_at(ii)] : -1;
  };
  F xa, xb;
  int64_t g = wave;
  load_rows(g, xa);
  int olda = load_old(g);
  for (; g < ngroups; g += EW) {  // wave-uniform
    const int64_t i = g * 32 + r;
    const bool valid = i < int64_t(total);
    const int64_t row = row_at(i);
    F& x = xa;
    load_rows(g + EW, xb);  // next group: in flight under this one's MFMAs
    const int oldb = load_old(g + EW);
    // exact argmin with the best and second-best exact distances (the second for the bounds)
    float best = INFINITY, second = INFINITY;
    int bidx = 0x7fffffff;
    const int64_t slot = slot_at(i);
    if (st_in && h == 0 && valid) {  // one half starts from the running state (no duplicate)
      const float2 st = xst[slot];
      best = st.x;
      bidx = __float_as_int(st.y);
    }
    for (int c0 = 0; c0 < kpad; c0 += 32) {
      f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const float* cp = ct + size_t(c0 + r) * CS + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (16 * s + 4 * q < d) {  // wave-uniform: skip all-padding groups (as exact_argmin)
            const float4 a4 = *reinterpret_cast<const float4*>(cp + 16 * s + 4 * q);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, x.at(s, 4 * q + 0), acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, x.at(s, 4 * q + 1), acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, x.at(s, 4 * q + 2), acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, x.at(s, 4 * q + 3), acc, 0, 0, 0);
          }
        }
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const float4 c4 = *reinterpret_cast<const float4*>(cn + c0 + 8 * gq + 4 * h);
        const float cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float dist = fmaf(-2.f, acc[4 * gq + q], cv[q]);
          if (dist < best) {
            second = best;
            best = dist;
            bidx = a.base + c0 + 8 * gq + 4 * h + q;
          } else if (dist < second) {
            second = dist;
          }
        }
      }
    }
    {
      const float ob = __shfl_xor(best, 32, 64), os = __shfl_xor(second, 32, 64);
      const int oi = __shfl_xor(bidx, 32, 64);
      const bool take = ob < best || (ob == best && oi < bidx);
      second = take ? fminf(best, os) : fminf(second, ob);
      if (take) {
        best = ob;
        bidx = oi;
      }
    }
    if (st_out) {  // not the last chunk: carry the state to the next one
      if (valid && h == 0) xst[slot] = make_float2(best, __int_as_float(bidx));
      xa = xb;
      olda = oldb;
      continue;
    }
    const int b = (bidx >= 0 && bidx < kglob) ? bidx : 0;
    const int old = valid ? olda : -1;
    // exact cost and |x|^2 in the assign kernels' lane order
    float part = 0.f, px = 0.f;
    const float* cb = a.chunk_mode ? a.centers_all + size_t(b) * DP + 8 * h
                                   : ct + size_t(b) * CS + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = x.at(s, j) - cb[16 * s + j];
        part = fmaf(e, e, part);
        px = fmaf(x.at(s, j), x.at(s, j), px);
      }
    const float rowcost = part + __shfl_xor(part, 32, 64);
    const float nx2 = px + __shfl_xor(px, 32, 64);
    if (valid && accumulate && !(a.delta && (old == b || old < 0))) {
      add_row(x, b, false);
      if (a.delta) add_row(x, min(old, k - 1), true);
    }
    if (valid && h == 0) {
      if (a.labels) a.labels[row] = b;
      if (a.mindist) a.mindist[row] = rowcost;
      if (a.bounds) {
        const float marg = mrel * (nx2 + cmax * cmax);
        reinterpret_cast<float2*>(a.bounds)[row] =
            make_float2(sqrtf(rowcost) * ueps + 1e-30f,
                        sqrtf(fmaxf(second + nx2 - 2.f * marg, 0.f)) * (1.f - 1e-6f));
      }
      my_cost += double(rowcost);
    }
    xa = xb;
    olda = oldb;
  }
  const double ws = wave_sum_f64(my_cost);
  if (lane == 0) wc[wave] = ws;
  __syncthreads();
  if (tid == 0 && a.cost_slab) {
    double tot = 0.0;
    for (int w = 0; w < EW; ++w) tot += wc[w];
    a.cost_slab[blockIdx.x] = tot;
  }
  if (L.lds_acc) {
    for (int i = tid; a.sums_too && i < k * d; i += NT) {
      const int c = i / d, f = i - c * d;
      const double v = acc_l[c * (d | 1) + f];  // an exact integer
      if (v != 0.0) atomicAdd(&a.sums[i], static_cast<u64>(static_cast<long long>(v)));
    }
    for (int i = tid; i < k; i += NT) {
      const int c = static_cast<int>(cnt_l[i]);
      if (c) atomicAdd(&a.counts[i], static_cast<u64>(static_cast<long long>(c)));
    }
  }
}

// ---- the exact re-decision by candidates (f32 rows, single-launch passes) ------------------
// The same decision as oap_kmeans_exact_rows, bitwise, at a fraction of its matrix work: a
// deferred row's exact argmin can only be a center whose tier-1 distance lies within the tier's
// pair error bound tt of the tier-1 best (the bound the lean pass deferred it by; kmeans_lloyd
// tier-1 notes above), so this pass re-runs tier 1 for the row (fp16 MFMA, 28 products at the
// headline's shape instead of 224 f32 ones), keeps the centers with tier-1 distance <= t1 + 2 tt,
// and evaluates only those in fp32 on the VALU — as the fmaf chain v_mfma_f32_32x32x2_f32 computes
// (k = 0 product first, then k = 1, over the same (s, q, component) steps and padding skips as
// exact_argmin: bitwise the MFMA's value, tools/probes/mfma_f32_order.hip).  A row outside fp16's
// range for tier 1 (alpha^2 |x|^2 >= 2^20) evaluates every center.  The second-best distance
// for the Hamerly lower bound is min(the exact second among the candidates, best + tt / alpha^2),
// a valid lower bound for every center left out.  Accumulation, labels, bounds, cost: as
// oap_kmeans_exact_rows.
constexpr int kCandWaves = 12;  // 3 per SIMD: latency-bound rows (the row in registers twice)
constexpr int kCandList = 8;    // per-lane candidate slots (LDS); more -> the lane takes all

struct CandSmem {
  size_t plane, cn, sc, acc, cnt, wc, pref, cl, total;
  bool lds_acc;
};

__host__ __device__ inline CandSmem cand_plan(int kpad, int k, int d, bool acc, bool sums) {
  const int dp = (d + 15) / 16 * 16;
  CandSmem m;
  size_t off = 0;
  m.plane = 0;
  off = round16(size_t(kpad) * stride_bf16(dp) * 2);
  m.cn = off;
  off = round16(off + size_t(kpad) * 4);
  m.sc = off;
  off = round16(off + size_t(dp) * 4);
  m.wc = off;
  off = round16(off + kCandWaves * 8);
  m.pref = off;
  off = round16(off + (kDeferSubs + 1) * 4);
  m.cl = off;
  off = round16(off + size_t(kCandWaves) * 64 * kCandList * 4);
  m.acc = off;
  const size_t base = off;
  size_t accb = (acc && sums) ? size_t(k) * (d | 1) * 8 : 0;
  size_t cntb = acc ? size_t(k) * 4 : 0;
  m.lds_acc = acc && round16(base + accb) + round16(cntb) <= kLdsLimit - 1024;
  if (!m.lds_acc) accb = cntb = 0;
  off = round16(off + accb);
  m.cnt = off;
  off = round16(off + cntb);
  m.total = off;
  return m;
}

template <int KS>
__global__ __launch_bounds__(kCandWaves * 64) void oap_kmeans_exact_cand(KMeansAssignArgs a) {
  constexpr int EW = kCandWaves;
  constexpr int DP = 16 * KS;
  constexpr int NT = EW * 64;
  using F = Frag<KS, false>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (a.halt && *a.halt) return;
  const int k = a.k, d = a.d, kpad = a.kpad;
  const bool accumulate = a.accumulate;
  const CandSmem L = cand_plan(kpad, k, d, accumulate, a.sums_too);
  const int sb = stride_bf16(DP);
  _Float16* ph = reinterpret_cast<_Float16*>(smem + L.plane);
  float* cn = reinterpret_cast<float*>(smem + L.cn);
  float* sc_l = reinterpret_cast<float*>(smem + L.sc);
  double* acc_l = reinterpret_cast<double*>(smem + L.acc);
  unsigned* cnt_l = reinterpret_cast<unsigned*>(smem + L.cnt);
  double* wc = reinterpret_cast<double*>(smem + L.wc);
  unsigned* pref = reinterpret_cast<unsigned*>(smem + L.pref);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  int* cl = reinterpret_cast<int*>(smem + L.cl) + wave * 64 * kCandList + lane;  // [slot * 64]
  // (the sub-segment counts loaded in parallel, then summed in LDS: one load latency, not 16)
  if (tid < a.row_subs) pref[tid + 1] = a.row_count[blockIdx.x * kDeferSubs + tid];
  __syncthreads();
  if (tid == 0) {
    pref[0] = 0u;
    for (int w = 0; w < a.row_subs; ++w) pref[w + 1] += pref[w];
  }
  __syncthreads();
  const unsigned total = pref[a.row_subs];
  if (total == 0) {
    if (tid == 0 && a.cost_slab) a.cost_slab[blockIdx.x] = 0.0;
    return;
  }
  const float cmax = a.cstat[0];
  const float alpha = lean_alpha(cmax);
  const float a2 = alpha * alpha;
  const float inv_a2 = 1.f / a2;  // (a power of two)
  // the tier-1 plane exactly as the lean first pass stages it (c' = [-2 alpha c, .., hi, lo
  // (alpha^2 |c|^2 / 16), 16, 16])
  // (unconditional loads, unrolled: a thread's loads in flight together)
#pragma unroll 4
  for (int idx = tid; idx < kpad * DP; idx += NT) {
    const int c = idx / DP, f = idx - c * DP;
    const float cv = a.centers[idx], cnv = a.cnorm[c];
    _Float16 v;
    if (f < d) {
      v = static_cast<_Float16>(-2.f * alpha * cv);
    } else if (f == DP - 4 || f == DP - 3) {
      _Float16 hi, lo;
      split_f16((c < k) ? a2 * cnv * (1.f / kBiasUnit) : 60000.f, hi, lo);
      v = (f == DP - 4) ? hi : lo;
    } else {
      v = static_cast<_Float16>(f >= DP - 2 ? kBiasUnit : 0.f);
    }
    ph[c * sb + f] = v;
  }
  for (int c = tid; c < kpad; c += NT) cn[c] = (c < k) ? a.cnorm[c] : 1e30f;
  for (int f = tid; f < DP; f += NT) sc_l[f] = (a.scale && a.sums_too && f < d) ? a.scale[f] : 0.f;
  if (L.lds_acc) {
    if (a.sums_too)
      for (int i = tid; i < k * (d | 1); i += NT) acc_l[i] = 0.0;
    for (int i = tid; i < k; i += NT) cnt_l[i] = 0u;
  }
  __syncthreads();
  const int64_t sub = a.row_seg_cap / a.row_subs;
  const float cm_s = alpha * cmax;
  const float thr_c = 0.0040f * cm_s;
  const float thr_k = 6e-5f * cm_s * cm_s + float(d) * 6.2e-5f + 1e-30f;
  const float mrel = 4e-7f * float(d + 8);
  const float ueps = 1.f + 1e-6f + 6e-8f * float(d + 4);
  const int64_t ngroups = (int64_t(total) + 31) / 32;
  auto slot_at = [&](int64_t i) -> int64_t {
    i = i < int64_t(total) ? i : int64_t(total) - 1;
    int w = 0;
    while (w + 1 < a.row_subs && int64_t(pref[w + 1]) <= i) ++w;
    return int64_t(blockIdx.x) * a.row_seg_cap + w * sub + (i - pref[w]);
  };
  auto row_at = [&](int64_t i) -> int64_t { return int64_t(a.row_list[slot_at(i)]); };
  auto load_rows = [&](int64_t g, F& dst) {
    const int64_t row = row_at(g * 32 + r);
    const float* p = static_cast<const float*>(a.x) + row * a.ld + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int f = 16 * s + 8 * h + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (s < KS - 1 || f < a.ld) v = *reinterpret_cast<const float4*>(p + 16 * s + 4 * q);
        dst.v[s][4 * q + 0] = v.x;
        dst.v[s][4 * q + 1] = v.y;
        dst.v[s][4 * q + 2] = v.z;
        dst.v[s][4 * q + 3] = v.w;
      }
  };
  auto add_row = [&](const F& xv, int b, bool neg) {
    if (L.lds_acc) {
      if (h == 0) atomicAdd(&cnt_l[b], neg ? 0xffffffffu : 1u);
    } else if (h == 0) {
      atomicAdd(&a.counts[b], neg ? ~0ull : 1ull);
    }
    if (!a.sums_too) return;
    const float sgn = neg ? -1.f : 1.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 16 * s + 8 * h + j;
        if (f < d) {
          const float q = sgn * rintf(xv.at(s, j) * sc_l[f]);
          if (L.lds_acc)
            atomicAdd(acc_l + b * (d | 1) + f, static_cast<double>(q));
          else
            atomicAdd(&a.sums[size_t(b) * d + f], static_cast<u64>(static_cast<long long>(q)));
        }
      }
  };
  double my_cost = 0.0;
  // the previous labels of a group's rows (delta passes), gathered with its rows: a group ahead
  auto load_old = [&](int64_t gg) -> int {
    const int64_t ii = gg * 32 + r;
    return (a.delta && ii < int64_t(total)) ? a.labels[row_at(ii)] : -1;
  };
  F xa, xb;
  int64_t g = wave;
  load_rows(g, xa);
  int olda = load_old(g);
  for (; g < ngroups; g += EW) {  // wave-uniform
    const int64_t i = g * 32 + r;
    const bool valid = i < int64_t(total);
    const int64_t row = row_at(i);
    F& x = xa;
    load_rows(g + EW, xb);  // next group: in flight under this one
    const int oldb = load_old(g + EW);
    // the whole row in h-normalised order: x0 = features 16 s + j (j < 8), x1 = 16 s + 8 + j
    float x0[KS][8], x1[KS][8];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float o = __shfl_xor(x.v[s][j], 32, 64);
        x0[s][j] = h ? o : x.v[s][j];
        x1[s][j] = h ? x.v[s][j] : o;
      }
    // tier-1 operand (as the lean first pass builds it) and alpha^2 |x|^2 from its bias pair
    float nx2 = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) nx2 = fmaf(x.at(s, j), x.at(s, j), nx2);
    nx2 += xor32_f(nx2);
    f16x8 xh[KS];
    {
      _Float16 nh, nl;
      split_f16(alpha * alpha * nx2 * (1.f / kBiasUnit), nh, nl);
      const _Float16 unit = static_cast<_Float16>(kBiasUnit);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        f16x8 v;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const f32x2 pp = f32x2{x.at(s, j), x.at(s, j + 1)} * alpha;
          const f16x2 qq = __builtin_convertvector(pp, f16x2);
          v[j] = qq[0];
          v[j + 1] = qq[1];
        }
        if (s == KS - 1) {
          v[4] = h ? unit : v[4];
          v[5] = h ? unit : v[5];
          v[6] = h ? nh : v[6];
          v[7] = h ? nl : v[7];
        }
        xh[s] = v;
      }
    }
    const float mine =
        kBiasUnit * (static_cast<float>(xh[KS - 1][6]) + static_cast<float>(xh[KS - 1][7]));
    const float other = xor32_f(mine);
    const float nx2_s = h ? mine : other;
    auto tier1 = [&](int c0) -> f32x16 {
      f32x16 acc = f32x16{};
      const _Float16* ap = ph + size_t(c0 + r) * sb + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(
            *reinterpret_cast<const f16x8*>(ap + 16 * s), xh[s], acc, 0, 0, 0);
      return acc;
    };
    // pass 1: the tier-1 best and second of the row
    float t1 = INFINITY, t2 = INFINITY;
    for (int c0 = 0; c0 < kpad; c0 += 32) {
      const f32x16 acc = tier1(c0);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        t2 = fminf(t2, fmaxf(t1, acc[e]));
        t1 = fminf(t1, acc[e]);
      }
    }
    {
      const float o1 = xor32_f(t1), o2 = xor32_f(t2);
      t2 = fminf(fmaxf(t1, o1), fminf(t2, o2));
      t1 = fminf(t1, o1);
    }
    const float tt = fmaf(thr_c, __builtin_amdgcn_sqrtf(nx2_s), thr_k) + 5e-5f * nx2_s +
                     2.5e-4f * fabsf(t2);
    // (row-uniform: both halves hold t1, t2, nx2_s)
    const bool every = !(nx2_s < 1048576.f) || !(t1 < INFINITY) || !(tt < INFINITY);
    const float T = t1 + 2.f * tt;
    // pass 2: this lane's candidates (centers c0 + 8 g + 4 h + q of each chunk) into its slots
    int ncand = 0;
    if (!every) {
      for (int c0 = 0; c0 < kpad; c0 += 32) {
        const f32x16 acc = tier1(c0);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int c = c0 + 8 * (e >> 2) + 4 * h + (e & 3);
          if (acc[e] <= T && c < k) {
            if (ncand < kCandList) cl[ncand * 64] = c;
            ++ncand;
          }
        }
      }
    }
    const bool all_mine = every || ncand > kCandList;  // this lane evaluates all its centers
    const int my_n = !valid ? 0 : all_mine ? 16 * (kpad / 32) : ncand;
    // exact fp32 distances of the candidates, in each lane's ascending center order
    float best = INFINITY, second = INFINITY;
    int bidx = 0x7fffffff;
    for (int j = 0; __ballot(j < my_n) != 0; ++j) {  // (wave-uniform trip count)
      if (j < my_n) {
        const int c = all_mine ? 32 * (j >> 4) + 8 * ((j & 15) >> 2) + 4 * h + (j & 3)
                               : cl[j * 64];
        if (c < k) {
          const float4* cp = reinterpret_cast<const float4*>(a.centers + size_t(c) * DP);
          float acc = 0.f;
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              if (16 * s + 4 * q < d) {
                const float4 c0v = cp[4 * s + q], c1v = cp[4 * s + 2 + q];
                acc = fmaf(x1[s][4 * q + 0], c1v.x, fmaf(x0[s][4 * q + 0], c0v.x, acc));
                acc = fmaf(x1[s][4 * q + 1], c1v.y, fmaf(x0[s][4 * q + 1], c0v.y, acc));
                acc = fmaf(x1[s][4 * q + 2], c1v.z, fmaf(x0[s][4 * q + 2], c0v.z, acc));
                acc = fmaf(x1[s][4 * q + 3], c1v.w, fmaf(x0[s][4 * q + 3], c0v.w, acc));
              }
            }
          const float dist = fmaf(-2.f, acc, cn[c]);
          if (dist < best || (dist == best && c < bidx)) {
            second = best;
            best = dist;
            bidx = a.base + c;
          } else if (dist < second) {
            second = dist;
          }
        }
      }
    }
    {
      const float ob = __shfl_xor(best, 32, 64), os = __shfl_xor(second, 32, 64);
      const int oi = __shfl_xor(bidx, 32, 64);
      const bool take = ob < best || (ob == best && oi < bidx);
      second = take ? fminf(best, os) : fminf(second, ob);
      if (take) {
        best = ob;
        bidx = oi;
      }
    }
    // centers left out: exact distance > best + tt / alpha^2
    if (!every) second = fminf(second, best + tt * inv_a2);
    const int b = (bidx >= 0 && bidx < k) ? bidx : 0;
    const int old = valid ? olda : -1;
    float part = 0.f, px = 0.f;
    const float* cb = a.centers + size_t(b) * DP + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = x.at(s, j) - cb[16 * s + j];
        part = fmaf(e, e, part);
        px = fmaf(x.at(s, j), x.at(s, j), px);
      }
    const float rowcost = part + __shfl_xor(part, 32, 64);
    const float nx2e = px + __shfl_xor(px, 32, 64);
    if (valid && accumulate && !(a.delta && (old == b || old < 0))) {
      add_row(x, b, false);
      if (a.delta) add_row(x, min(old, k - 1), true);
    }
    if (valid && h == 0) {
      if (a.labels) a.labels[row] = b;
      if (a.mindist) a.mindist[row] = rowcost;
      if (a.bounds) {
        const float marg = mrel * (nx2e + cmax * cmax);
        reinterpret_cast<float2*>(a.bounds)[row] =
            make_float2(sqrtf(rowcost) * ueps + 1e-30f,
                        sqrtf(fmaxf(second + nx2e - 2.f * marg, 0.f)) * (1.f - 1e-6f));
      }
      my_cost += double(rowcost);
    }
    xa = xb;
    olda = oldb;
  }
  const double ws = wave_sum_f64(my_cost);
  if (lane == 0) wc[wave] = ws;
  __syncthreads();
  if (tid == 0 && a.cost_slab) {
    double tot = 0.0;
    for (int w = 0; w < EW; ++w) tot += wc[w];
    a.cost_slab[blockIdx.x] = tot;
  }
  if (L.lds_acc) {
    for (int i = tid; a.sums_too && i < k * d; i += NT) {
      const int c = i / d, f = i - c * d;
      const double v = acc_l[c * (d | 1) + f];
      if (v != 0.0) atomicAdd(&a.sums[i], static_cast<u64>(static_cast<long long>(v)));
    }
    for (int i = tid; i < k; i += NT) {
      const int c = static_cast<int>(cnt_l[i]);
      if (c) atomicAdd(&a.counts[i], static_cast<u64>(static_cast<long long>(c)));
    }
  }
}

template <int KS>
void launch_cand(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  const CandSmem L = cand_plan(a.kpad, a.k, a.d, a.accumulate, a.sums_too);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_exact_cand<KS>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_exact_cand<KS>), dim3(grid), dim3(kCandWaves * 64), L.total, s,
                     a);
  OAP_HIP_CHECK(hipGetLastError());
}

template <int KS, bool XB>
void launch_exact(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  const ExactSmem L = exact_plan(a.kpad, a.k, a.d, a.accumulate, a.sums_too);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_exact_rows<KS, XB>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_exact_rows<KS, XB>), dim3(grid), dim3(exact_waves(KS, XB) * 64),
                     L.total, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

template <bool XB>
void launch_exact_xb(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  switch ((a.d + 15) / 16) {
    case 1: launch_exact<1, XB>(a, grid, s); break;
    case 2: launch_exact<2, XB>(a, grid, s); break;
    case 3: launch_exact<3, XB>(a, grid, s); break;
    case 4: launch_exact<4, XB>(a, grid, s); break;
    case 5: launch_exact<5, XB>(a, grid, s); break;
    case 6: launch_exact<6, XB>(a, grid, s); break;
    case 7: launch_exact<7, XB>(a, grid, s); break;
    case 8: launch_exact<8, XB>(a, grid, s); break;
    default: OAP_THROW(ConfigError, "kmeans_exact_rows: unsupported d=" << a.d);
  }
}

// ---------------------------------------------------------------- delta scan (lean layout)
// The pruning test of every row of a lean workgroup's tile range (the assign kernels' own test,
// with the tile's largest |x|^2 in the margin — never looser per row); pruned tiles get their
// bounds advanced in place (rounded outward; no write once no center moves), the others are
// appended to that workgroup's segment of tile_list.  Scan block (b, j) covers chunks j, j + S,
// ... of lean workgroup b's range, so every counter is shared by S blocks only.
constexpr int kScanSplit = 8;

__global__ __launch_bounds__(256) void oap_kmeans_lean_scan(
    int64_t n, int k, int d, int lean_grid, int64_t tiles_per_block, float2* __restrict__ bounds,
    const int32_t* __restrict__ labels, const float* __restrict__ xnorm,
    const float* __restrict__ drift, const float* __restrict__ drift_max,
    const float* __restrict__ cstat, int32_t* __restrict__ tile_list,
    unsigned* __restrict__ tile_count, unsigned long long* __restrict__ pruned,
    const int* __restrict__ halt) {
  if (halt && *halt) return;
  __shared__ unsigned wcnt[4], wbase[4];
  __shared__ unsigned long long bpruned;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int lb = blockIdx.x % lean_grid, j = blockIdx.x / lean_grid;
  const float dmax = drift_max[0];
  const float cmax = cstat[0];
  const float mrel = 4e-7f * float(d + 8);
  const int64_t ntiles = (n + 31) / 32;
  const int64_t T = tiles_per_block;
  const int64_t t0 = int64_t(lb) * T;
  const int64_t t1 = t0 + T < ntiles ? t0 + T : ntiles;
  const int64_t nchunks = t1 > t0 ? (t1 - t0 + 7) / 8 : 0;  // a chunk = 8 tiles, 2 per wave
  int32_t* seg = tile_list + int64_t(lb) * T;
  if (threadIdx.x == 0) bpruned = 0;
  unsigned long long n_pruned = 0;
  for (int64_t c = j; c < nchunks; c += kScanSplit) {  // block-uniform trip count
    const int64_t w0 = t0 + c * 8 + 2 * wave;  // this wave's first tile
    const int64_t row = w0 * 32 + lane;
    const bool valid = w0 + h < t1 && row < n;
    bool ok = true;
    float2 bnew = make_float2(0.f, 0.f);
    if (valid) {
      const float2 b = bounds[row];
      const int lab = min(max(labels[row], 0), k - 1);
      const float u = b.x + drift[lab];
      const float lk = b.y - dmax;
      ok = lk > 0.f && (lk - u) * (lk + u) > mrel * (xnorm[row >> 5] + cmax * cmax);
      bnew = make_float2(u * (1.f + 2.5e-7f), lk * (1.f - 2.5e-7f));
    }
    const unsigned long long all_ok = __ballot(ok);
    const bool pr0 = static_cast<unsigned>(all_ok) == 0xffffffffu;
    const bool pr1 = static_cast<unsigned>(all_ok >> 32) == 0xffffffffu;
    if (dmax > 0.f && valid && (h ? pr1 : pr0)) bounds[row] = bnew;
    const bool has0 = w0 < t1, has1 = w0 + 1 < t1;
    const bool act0 = has0 && !pr0, act1 = has1 && !pr1;
    if (lane == 0) {
      wcnt[wave] = unsigned(act0) + unsigned(act1);
      n_pruned += unsigned(has0 && pr0) + unsigned(has1 && pr1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
      unsigned pos = tot ? atomicAdd(tile_count + lb, tot) : 0u;
      for (int i = 0; i < 4; ++i) {
        wbase[i] = pos;
        pos += wcnt[i];
      }
    }
    __syncthreads();
    if (lane == 0) {
      unsigned pos = wbase[wave];
      if (act0) seg[pos++] = static_cast<int32_t>(w0);
      if (act1) seg[pos] = static_cast<int32_t>(w0 + 1);
    }
  }
  if (lane == 0 && n_pruned) atomicAdd(&bpruned, n_pruned);
  __syncthreads();
  if (threadIdx.x == 0 && bpruned && pruned) atomicAdd(pruned, bpruned);
}

}  // namespace

bool kmeans_lloyd_supported(int d, int k, bool accumulate, bool sums_too) {
  if (d + 4 > 128) return false;
  const int dp = (d + 4 + 15) / 16 * 16;
  if (dp != kmeans_dp(d)) return false;  // the centroid buffer's row stride must match
  const int kpad = (k + 31) / 32 * 32;
  if (kpad > 1024) return false;  // keys carry a 10-bit index
  return lean_plan(dp, kpad, k, d, accumulate, sums_too, 16, true).total <= kLdsLimit &&
         exact_plan(kpad, k, d, accumulate, sums_too).total <= kLdsLimit;
}

int kmeans_lloyd_chunk_kmax(int d) {
  if (d + 4 > 128) return 0;
  const int dp = (d + 4 + 15) / 16 * 16;
  if (dp != kmeans_dp(d)) return 0;
  int best = 0;
  for (int kp = 32; kp <= 1024; kp += 32)
    if (lean_plan(dp, kp, kp, d, false, false, 16, false).total <= kLdsLimit) best = kp;
  return best;
}

int kmeans_exact_chunk_kmax(int d) {
  int best = 0;
  for (int kp = 32; kp <= 1024; kp += 32)
    if (exact_plan(kp, kp, d, false, false).total <= kLdsLimit) best = kp;
  return best;
}

int kmeans_lloyd_grid(int64_t n, int num_cus) {
  const int64_t tiles = (n + 31) / 32;
  const int64_t cap = num_cus > 256 ? num_cus : 256;
  return static_cast<int>(tiles < cap ? (tiles < 1 ? 1 : tiles) : cap);
}

int64_t kmeans_lloyd_tiles_per_block(int64_t n, int grid) {
  const int64_t tiles = (n + 31) / 32;
  return (tiles + grid - 1) / grid;
}

int kmeans_lloyd_waves(int variant) { return variant == 8 ? 12 : 16; }

int64_t kmeans_lloyd_seg_cap(int64_t n, int grid, int waves) {
  const int64_t per_block = kmeans_lloyd_tiles_per_block(n, grid);
  return int64_t(waves) * ((per_block + waves - 1) / waves) * 32;
}

size_t kmeans_lloyd_image_bytes(int64_t n, int d) {
  if (n <= 0 || d <= 0 || d + 4 > 128) return 0;
  const int ks = (d + 4 + 15) / 16;
  return size_t((n + 31) / 32) * size_t(ks) * 64 * 16;
}

int kmeans_lloyd(const KMeansAssignArgs& a, int grid, int variant, hipStream_t s) {
  // the chunked driver (centers_all set) pairs this pass with a chunked exact pass, so only the
  // lean plane has to fit (a single lean chunk runs as chunk_mode 0)
  const bool chunk_ok = !a.centers_all
                            ? kmeans_lloyd_supported(a.d, a.k, a.accumulate, a.sums_too)
                            : (a.kpad <= kmeans_lloyd_chunk_kmax(a.d) && !a.accumulate &&
                               !a.delta && (a.chunk_mode == 0 || a.lean_keys) &&
                               a.base + a.kpad <= 1024 && a.base % 32 == 0);
  OAP_CHECK(chunk_ok && !a.precise &&
                !a.merge && a.cstat && a.defer_rows && a.defer_row_count &&
                a.row_seg_cap == kmeans_lloyd_seg_cap(a.n, grid, kmeans_lloyd_waves(variant)) &&
                a.ld == kmeans_ld(a.d, a.xbf16),
            "kmeans_lloyd: unsupported arguments");
  OAP_CHECK(!a.delta || a.labels, "kmeans_lloyd: delta mode needs the previous labels");
  OAP_CHECK(!a.tile_list || (a.delta && a.tile_count), "kmeans_lloyd: tile list without delta");
  // the operand image: f32 rows, one launch; written by a full pass, read without the per-tile
  // |x|^2 output (that comes from the f32 rows)
  OAP_CHECK(!a.ximg || a.img_mode == 0 ||
                (!a.xbf16 && !a.centers_all && a.img_beta &&
                 (a.img_mode == 1 ? !a.tile_list && (a.cost_slab || a.mindist)
                                  : ((a.img_mode == 2 || a.img_mode == 3) && !a.xnorm &&
                                     !a.cost_slab && !a.mindist))),
            "kmeans_lloyd: bad operand-image arguments");
  if (a.n == 0) return 0;
  LeanArgs l;
  l.x = a.x;
  l.centers = a.centers;
  l.cnorm = a.cnorm;
  l.cstat = a.cstat;
  l.scale = a.scale;
  l.sums = a.sums;
  l.counts = a.counts;
  l.cost_slab = a.cost_slab;
  l.labels = a.labels;
  l.mindist = a.mindist;
  l.bounds = reinterpret_cast<float2*>(a.bounds);
  l.xnorm = a.xnorm;
  l.tile_list = a.delta ? a.tile_list : nullptr;
  l.tile_count = a.delta ? a.tile_count : nullptr;
  l.defer_rows = a.defer_rows;
  l.defer_row_count = a.defer_row_count;
  l.deferred_rows = a.deferred_rows;
  l.n = a.n;
  l.seg_cap = a.row_seg_cap;
  l.tiles_per_block = kmeans_lloyd_tiles_per_block(a.n, grid);
  l.ld = a.ld;
  l.d = a.d;
  l.k = a.k;
  l.kpad = a.kpad;
  l.accumulate = a.accumulate;
  l.sums_too = a.sums_too;
  l.delta = a.delta;
  l.ablate = a.ablate;
  l.refine = kmeans_refine_default() ? 1 : 0;
  l.keys = reinterpret_cast<int2*>(a.lean_keys);
  l.centers_all = a.centers_all;
  l.kbase = a.base;
  l.kglob = a.kglob;
  l.chunk_mode = a.chunk_mode;
  l.ximg = static_cast<_Float16*>(a.ximg);
  l.img_beta = a.img_beta;
  l.img_mode = a.ximg ? a.img_mode : 0;
  // (full passes over the rows only: the image passes never see every row's f32 values)
  const bool rows_pass = !(l.img_mode == 2 || l.img_mode == 3) && !a.tile_list && !a.delta;
  OAP_CHECK((!a.sq_slab && !a.bound_flag) || (rows_pass && a.chunk_mode <= 1),
            "kmeans_lloyd: sum |x|^2 / bound check need a full pass over the rows");
  l.sq_slab = a.sq_slab;
  l.bound_flag = a.bound_flag;
  l.bound_inf = a.bound_inf;
  l.halt = a.halt;
  // the exact per-row cost is computed when a cost or mindist is asked for
  const bool cost = a.cost_slab != nullptr || a.mindist != nullptr;
  if (a.xbf16)
    launch_lean_xb<true>(l, grid, variant, cost, s);
  else
    launch_lean_xb<false>(l, grid, variant, cost, s);
  return grid;
}

void kmeans_exact_rows(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  OAP_CHECK(a.row_list && a.row_count && a.row_seg_cap > 0 && a.row_subs >= 1 &&
                a.row_subs <= kDeferSubs && a.d <= 128 && a.cstat &&
                a.ld == kmeans_ld(a.d, a.xbf16),
            "kmeans_exact_rows: bad arguments");
  if (a.n == 0) return;
  OAP_CHECK(exact_plan(a.kpad, a.k, a.d, a.accumulate, a.sums_too).total <= kLdsLimit,
            "kmeans_exact_rows: centers exceed LDS");
  OAP_CHECK(a.chunk_mode == 0 ||
                (a.xstate && a.centers_all && !a.accumulate && !a.delta && !a.bounds),
            "kmeans_exact_rows: chunked pass needs its running state and every center");
  // the candidate form: f32 rows of a single-launch pass whose centers' tier-1 plane fits (the
  // chunked and bf16 passes keep the full MFMA sweep); OAP_KMEANS_EXACT=mfma / cand force one
  const std::string fe = knob_str("OAP_KMEANS_EXACT");  // (read per call: tests switch it)
  const bool force_mfma = !fe.empty() && fe[0] == 'm';
  // (measured: 5-10% faster per pass at 390k rows per workgroup, the headline; 20% slower at 49k,
  // the 8-GPU shard, where staging its fp16 plane and running at 8 waves do not amortise)
  const bool big = a.n >= int64_t(grid) * 131072;
  if ((big || (!fe.empty() && fe[0] == 'c')) && !force_mfma && !a.xbf16 && a.chunk_mode == 0 &&
      a.d + 4 <= 96 && a.base == 0 &&
      (a.d + 4 + 15) / 16 * 16 == kmeans_dp(a.d) &&  // (the centers' row stride)
      cand_plan(a.kpad, a.k, a.d, a.accumulate, a.sums_too).total <= kLdsLimit) {
    switch ((a.d + 4 + 15) / 16) {
      case 1: launch_cand<1>(a, grid, s); return;
      case 2: launch_cand<2>(a, grid, s); return;
      case 3: launch_cand<3>(a, grid, s); return;
      case 4: launch_cand<4>(a, grid, s); return;
      case 5: launch_cand<5>(a, grid, s); return;
      case 6: launch_cand<6>(a, grid, s); return;
      default: break;  // (KS 7, 8: the row twice in registers spills; the sweep keeps them)
    }
  }
  if (a.xbf16)
    launch_exact_xb<true>(a, grid, s);
  else
    launch_exact_xb<false>(a, grid, s);
}

void kmeans_lean_scan(int64_t n, int k, int d, int lean_grid, float* bounds,
                      const int32_t* labels, const float* xnorm, const float* drift,
                      const float* drift_max, const float* cstat, int32_t* tile_list,
                      unsigned* tile_count, unsigned long long* pruned, hipStream_t s,
                      const int* halt) {
  if (n <= 0) return;
  OAP_HIP_CHECK(hipMemsetAsync(tile_count, 0, sizeof(unsigned) * lean_grid, s));
  hipLaunchKernelGGL(oap_kmeans_lean_scan, dim3(lean_grid * kScanSplit), dim3(256), 0, s, n, k, d,
                     lean_grid, kmeans_lloyd_tiles_per_block(n, lean_grid),
                     reinterpret_cast<float2*>(bounds), labels, xnorm, drift, drift_max, cstat,
                     tile_list, tile_count, pruned, halt);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
