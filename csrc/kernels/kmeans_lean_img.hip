// oap_kmeans_lean_img — the steady-state Lloyd pass of the headline K-Means fit (gfx950, CDNA4).
//
// Every Lloyd iteration after the first of a delta-accumulating fit over f32 rows (SURVEY.md
// §2.6 K1; the reference's hot loop is oneDAL's step1Local, KMeansDALImpl.cpp:70-77) reads the
// resident fp16 operand image that the first pass wrote (kmeans_lloyd.hip, img_mode 1) instead of
// the rows: tier-1 distances on v_mfma_f32_32x32x16_f16, the top-2 per row in registers, rows
// inside the tier's rigorous error bound deferred to oap_kmeans_exact_rows, and only the rows
// whose label changed read their f32 values (fixed-point +x / -x).  It is the same arithmetic as
// oap_kmeans_lloyd_t1's image branch (labels, bounds, deferral lists and statistics are bitwise
// those of that kernel), but as its own kernel:
// * compile-time everything: no chunk keys, no cost, no timing switches, no f32-row operand
//   path — the branch-free instruction stream the general kernel could not give its image branch
//   (runtime switches, ~70 spilled SGPRs, and a join that waited vmcnt(0) on every tile: the
//   moved-row flush's row loads, younger than the next tile's image prefetch, merged into every
//   tile's wait state);
// * the moved-row flush runs at the top of a tile, before that tile's loads are issued, and
//   drains its own loads — so no tile ever waits for the prefetch it has just issued;
// * the chunk loop is software-pipelined (CFG bit 0): chunk c + 1's MFMA chain is issued before
//   chunk c's epilogue, into a second accumulator, so the matrix pipe works under the wave's
//   own VALU as well as under the other waves';
// * the last chunk folds only its real centroid groups (k = 200: 4 of 16 keys per lane);
// * labels are stored only for rows that moved (the others already hold theirs);
// * row-scan passes (RM 2) test every row's Hamerly bounds in the kernel itself: each wave scans
//   its own tiles two at a time, advances the pruned rows' bounds in place and queues the others
//   in a per-wave LDS ring, from which it forms 32-row tiles — no separate scan kernel, no row
//   list through HBM, and a pass that prunes nothing costs one 8-byte bound read per row.
// When the plane at the image's scale is not representable (beta max|c| > 2^9) the kernel does
// nothing and oap_kmeans_lloyd_t1 (img_mode 3) runs the f32-row pass instead: both test the same
// device values, so exactly one of them runs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "kernels/kmeans_frag.h"
#include "kernels/kmeans_internal.h"
#include "runtime/knobs.h"

namespace oap {
namespace kern {

namespace {

using namespace kmdev;

#define OAP_AI __attribute__((always_inline))

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr float kBias = 16.f;  // the bias features' unit (kmeans_lloyd.hip kBiasUnit)
constexpr int kMv = 64;        // per-wave LDS slots of staged moved rows
constexpr int kRing = 128;     // per-wave LDS ring of unpruned rows (row-scan passes)

struct ImgArgs {
  const f16x8* img;  // row-major [32 tiles][2 KS] fragments (k-step s, half h at 2 s + h)
  const float* img_beta;
  const float* x;  // f32 rows [n][ld] (moved rows only)
  const float* centers;
  const float* cnorm;
  const float* cstat;
  const float* scale;
  u64* sums;
  u64* counts;
  int32_t* labels;
  float2* bounds;
  const int32_t* tile_list;
  const unsigned* tile_count;
  int32_t* defer_rows;
  unsigned* defer_row_count;
  u64* stat;  // optional [deferred rows, moved rows, image passes]
  // row-scan passes: per-tile max |x|^2 (global tile index), the centers' drift [k] and its
  // maximum at [k], and the counter of pruned rows
  const float* scan_xnorm;
  const float* drift;
  u64* pruned;
  int64_t n, seg_cap, tiles_per_block;
  int ld, d, k, kpad;
  int refine;  // the refined deferral test (kmeans_frag.h refined_tt; OAP_KMEANS_REFINE=0: off)
  const int* halt;  // batched fits: set once the fit converged (the pass then does nothing)
  const int* gate;  // optional: the pass runs only when *gate == gate_on (kmeans_scan_decide)
  int gate_on;
};

struct ImgSmem {
  size_t plane, sc, acc, cnt, mv, dr, ring, total;
};

// fp16 plane; fixed-point accumulator rows of DP + 1 doubles (odd: conflict-free ds_add_f64; the
// padded features add zeros into their own columns, so the moved-row adds need no predicate)
__host__ __device__ inline ImgSmem img_plan(int dp, int kpad, int k, int waves, bool scan) {
  ImgSmem m;
  size_t off = 0;
  m.plane = 0;
  off = round16(size_t(kpad) * stride_bf16(dp) * 2);
  m.sc = off;  // scales [dp], then per-wave 2 max |e_c| (kmdev::plane_resid2)
  off = round16(off + size_t(dp + kmdev::kResidSlots) * 4);
  m.acc = off;
  off = round16(off + size_t(k) * size_t(dp + 1) * 8);
  m.cnt = off;
  off = round16(off + size_t(k) * 4);
  m.mv = off;
  off += size_t(waves) * kMv * 8;
  m.dr = off;  // (row-scan passes: the drift, then the rings)
  off = scan ? round16(off + size_t(k) * 4) : off;
  m.ring = off;
  off += scan ? size_t(waves) * kRing * 4 : 0;
  m.total = round16(off);
  return m;
}

// set bits of a wave mask below this lane (v_mbcnt_lo + v_mbcnt_hi: no per-lane mask register)
__device__ inline unsigned lanes_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32),
                                    __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), 0u));
}

// a kernel-uniform float in an SGPR (v_readfirstlane of its bits)
__device__ inline float ufl(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ inline void split_h(float v, _Float16& hi, _Float16& lo) {
  hi = static_cast<_Float16>(v);
  lo = static_cast<_Float16>(v - static_cast<float>(hi));
}

// CFG: 1 software-pipelined chunk loop (dense passes), 0 not (row-scan passes); operands one
// tile ahead.  (The timing ablation builds of rounds 3-5 — no epilogue, MFMA, plane reads, image
// loads, accumulation or stores; operands two tiles ahead — live in git history.)
// RM (row mode): 0 dense tiles of 32 consecutive rows; 2 (SCAN) the fused row scan: 32
// consecutive entries of the wave's LDS ring (the rows its Hamerly test cannot prune).
// (Measured dead ends kept in git history only: RM 1, a separate row-scan kernel writing row
// lists through HBM, 5.30 vs 5.06 ms/step; RM 3, a mover stage against the 32 centers that moved
// most, 5.52 vs 4.38 ms/step.)
template <int KS, int WAVES, int CFG, int RM>
__global__ __launch_bounds__(WAVES * 64, 1) void oap_kmeans_lean_img(ImgArgs a) {
  constexpr bool SCAN = RM == 2;
  static_assert(RM == 0 || RM == 2, "row modes: dense (0) or fused row scan (2)");
  constexpr bool PIPE = (CFG & 1) != 0;
  static_assert(CFG == 0 || CFG == 1, "configurations: 0, 1 (pipelined chunk loop)");
  constexpr int DP = 16 * KS, NT = WAVES * 64, RS = DP + 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (a.halt && *a.halt) return;
  if (a.gate && *a.gate != a.gate_on) return;
  const float cmax = a.cstat[0];
  const float alpha = a.img_beta[0];
  if (!(alpha * cmax <= 512.f)) return;  // (kmeans_lloyd img_mode 3 takes this pass)
  const int k = a.k, kpad = a.kpad, d = a.d;
  const ImgSmem L = img_plan(DP, kpad, k, WAVES, SCAN);
  constexpr int rs = RS;  // accumulator row stride (doubles)
  const int sb = stride_bf16(DP);
  _Float16* ph = reinterpret_cast<_Float16*>(smem + L.plane);
  float* sc_l = reinterpret_cast<float*>(smem + L.sc);
  double* acc_l = reinterpret_cast<double*>(smem + L.acc);
  int* cnt_l = reinterpret_cast<int*>(smem + L.cnt);
  const int tid = threadIdx.x;
  const float a2 = alpha * alpha;
  const float inv_a2 = ufl(1.f / a2);  // (a power of two)
  // ---- the plane c' = [-2 alpha c, 0 .., hi, lo (alpha^2 |c|^2 / 16), 16, 16] (kmeans_lloyd.hip)
  // (unconditional loads, unrolled: a thread's loads in flight together — centers are kpad x DP
  // and cnorm kpad, every slot addressable)
#pragma unroll 4
  for (int idx = tid; idx < kpad * DP; idx += NT) {
    const int c = idx / DP, f = idx - c * DP;
    const float cv = a.centers[idx], cnv = a.cnorm[c];
    _Float16 v;
    if (f < d) {
      v = static_cast<_Float16>(-2.f * alpha * cv);
    } else if (f == DP - 4 || f == DP - 3) {
      _Float16 hi, lo;
      split_h((c < k) ? a2 * cnv * (1.f / kBias) : 60000.f, hi, lo);
      v = (f == DP - 4) ? hi : lo;
    } else {
      v = static_cast<_Float16>(f >= DP - 2 ? kBias : 0.f);
    }
    ph[c * sb + f] = v;
  }
  for (int f = tid; f < DP; f += NT) sc_l[f] = f < d ? a.scale[f] : 0.f;
  // (the refined deferral test: the plane's largest rounding residual, per wave)
  const bool refine = a.refine && d <= DP - kResidSlotOff;
  if (refine) {
    const float r2w = plane_resid2(a.centers, DP, k, d, alpha, tid, NT);
    if ((tid & 63) == 0) sc_l[DP + (tid >> 6)] = r2w;
  }
  for (int i = tid; i < k * rs; i += NT) acc_l[i] = 0.0;
  for (int i = tid; i < k; i += NT) cnt_l[i] = 0;
  float* dr_l = reinterpret_cast<float*>(smem + L.dr);
  if constexpr (SCAN)
    for (int i = tid; i < k; i += NT) dr_l[i] = a.drift[i];
  __syncthreads();
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  int2* mv_l = reinterpret_cast<int2*>(smem + L.mv) + wave * kMv;
  // tier-1 bound (kmeans_lloyd.hip, f32 rows): cross term, subnormals, bias pairs, accumulation
  // (kernel-uniform values pinned to SGPRs: a VGPR copy each would cost the pipelined loop
  // its register headroom)
  const float cm_s = ufl(alpha * cmax);
  const float thr_c = ufl(0.0040f * cm_s);
  // (subnormals: 1.25 d 2^-14 — the image is fp16(alpha x) / 4, rounded twice where subnormal)
  const float thr_k = ufl(6e-5f * cm_s * cm_s + float(d) * 7.8e-5f + 1e-30f);
  const float mrel = ufl(4e-7f * float(d + 8));
  const float mg_c = ufl(mrel * cm_s * cm_s);
  float r2m = 0.f;
  if (refine)
    for (int w = 0; w < WAVES; ++w) r2m = fmaxf(r2m, sc_l[DP + w]);
  const float r2max = ufl(r2m);
  const int64_t ntiles_all = (a.n + 31) / 32;
  const bool listed = a.tile_list != nullptr;
  const int64_t T = a.tiles_per_block;
  const int64_t t0 = int64_t(blockIdx.x) * T;
  const int64_t dense_pos = t0 < ntiles_all ? (ntiles_all - t0 < T ? ntiles_all - t0 : T) : 0;
  const int64_t npos = listed ? int64_t(a.tile_count[blockIdx.x]) : dense_pos;
  const int32_t* seg = listed ? a.tile_list + blockIdx.x * T : nullptr;
  constexpr int64_t stride = WAVES;
  const int64_t sub_cap = a.seg_cap / WAVES;
  int32_t* dseg = a.defer_rows + blockIdx.x * a.seg_cap + wave * sub_cap;
  unsigned n_def = 0;  // wave-uniform
  const int64_t row0 = t0 * 32;
  const int64_t wrows = row0 < a.n ? (a.n - row0 < T * 32 ? a.n - row0 : T * 32) : 0;
  const __amdgpu_buffer_rsrc_t rs_lab = buf_rsrc(a.labels + row0, uint32_t(wrows * 4));
  const __amdgpu_buffer_rsrc_t rs_bnd =
      buf_rsrc(a.bounds ? a.bounds + row0 : nullptr, a.bounds ? uint32_t(wrows * 8) : 0u);
  const __amdgpu_buffer_rsrc_t rs_def = buf_rsrc(dseg, uint32_t(sub_cap * 4));
  // this workgroup's image rows (32 ceil(wrows / 32) records, < 4 GiB) and f32 rows
  const __amdgpu_buffer_rsrc_t rs_img =
      buf_rsrc(a.img + row0 * (2 * KS), uint32_t((wrows + 31) / 32 * 32 * (32 * KS)));
  const __amdgpu_buffer_rsrc_t rs_x = buf_rsrc(a.x + row0 * a.ld, uint32_t(wrows * a.ld * 4));
  const bool want_bounds = a.bounds != nullptr;
  // last chunk: its real 8-centroid groups (the earlier chunks are all real: kpad = 32 ceil(k/32))
  const int c_last = kpad - 32;
  const int ng_last = (k - c_last + 7) >> 3;  // 1..4

  auto tile_of = [&](int64_t q) OAP_AI -> int64_t {
    if (npos == 0) return 0;
    q = q < npos ? q : npos - 1;
    if (!listed) return t0 + q;
    typedef const int32_t __attribute__((address_space(4)))* seg_cptr;  // (scalar load)
    const int64_t tl = int64_t(((seg_cptr)(seg))[q]);
    return tl < 0 ? 0 : (tl < ntiles_all ? tl : ntiles_all - 1);
  };
  // one row's operand fragments (row-major image: 2 KS fragments per row) through a buffer
  // resource over this workgroup's rows: a 32-bit offset per lane instead of a 64-bit pointer
  // (the pipelined loop has no VGPRs to spare)
  auto load_img_row = [&](int64_t row, f16x8(&dst)[KS]) OAP_AI {
    const uint32_t off = uint32_t(row - row0) * uint32_t(32 * KS) + 16u * uint32_t(h);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      dst[s] = __builtin_bit_cast(
          f16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_img, off + 32u * s, 0, 0));
  };

  // ---- moved rows: staged (row, new | old << 16) in the wave's LDS slots, accumulated 32 at a
  // time with every lane busy (fixed-point +x into new, -x into old)
  unsigned n_mv = 0;  // wave-uniform
  u64 moved_total = 0;
  auto flush = [&](unsigned cnt) OAP_AI {  // entries [0, min(cnt, 32))
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool on = unsigned(r) < cnt;
    const int2 e = mv_l[on ? r : 0];
    float xv[KS][8];
    {
      // (an offset past the row's ld reads zeros: features beyond ld are padding)
      const uint32_t rb = uint32_t(int64_t(e.x) - row0) * uint32_t(a.ld) * 4u;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int f = 16 * s + 8 * h + 4 * q;
          const uint32_t off = (s < KS - 1 || f < a.ld) ? rb + uint32_t(f) * 4u : kBufOff;
          const f32x4 v = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_x, off, 0, 0));
          xv[s][4 * q + 0] = v[0];
          xv[s][4 * q + 1] = v[1];
          xv[s][4 * q + 2] = v[2];
          xv[s][4 * q + 3] = v[3];
        }
    }
    if (on) {
      const int b = e.y & 0xffff, bo = e.y >> 16;
      if (h == 0) {
        atomicAdd(&cnt_l[b], 1);
        atomicAdd(&cnt_l[bo], -1);
      }
      double* ap = acc_l + b * rs + 8 * h;
      double* aq = acc_l + bo * rs + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float4 s0 = *reinterpret_cast<const float4*>(sc_l + 16 * s + 8 * h);
        const float4 s1 = *reinterpret_cast<const float4*>(sc_l + 16 * s + 8 * h + 4);
        const float scv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // (features >= d: scale 0, a zero into a pad column)
          const double v = static_cast<double>(rintf(xv[s][j] * scv[j]));
          atomicAdd(ap + 16 * s + j, v);
          atomicAdd(aq + 16 * s + j, -v);
        }
      }
    }
    if (cnt > 32) {  // slide the rest down (read all before any write: in-order LDS)
      const int2 rest = mv_l[32 + r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (h == 0 && unsigned(r) < cnt - 32) mv_l[r] = rest;
    }
    moved_total += cnt < 32 ? cnt : 32;
    // drain the row loads here: a younger load left pending would make every later tile's
    // wait for its operand prefetch wait for it too (vmcnt counts in issue order)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  };

  // ---- one tile: X holds its operands (landed or in flight), pf receives tile pos + stride
  // row: this lane's row (-1: none); pf_row: the row whose operands go to pf (a real row)
  auto body = [&](auto pf_t, const int64_t pos, const int64_t row, const int64_t pf_row,
                  f16x8(&X)[KS], f16x8(&pf)[KS]) OAP_AI {
    constexpr bool PFON = decltype(pf_t)::value;  // (false: no next-tile prefetch)
    if (n_mv >= 32) {  // (before this tile's loads are issued)
      flush(n_mv);
      n_mv -= 32;
    }
    const bool valid = pos < npos && row >= 0 && row < a.n;
    const uint32_t roff = uint32_t(row - row0);
    int old = buf_load_b32(rs_lab, roff * 4, valid);
    if constexpr (PFON) load_img_row(pf_row, pf);
    // alpha^2 |x|^2 from the bias pair (h = 1 lanes' slots 6, 7 of the last k-step)
    const float mine =
        kBias * (static_cast<float>(X[KS - 1][6]) + static_cast<float>(X[KS - 1][7]));
    const float other = xor32_f(mine);
    const float nx2_s = h ? mine : other;
    int k1 = 0x7fffffff, k2 = 0x7fffffff;
    auto frags = [&](int c0, f16x8(&av)[KS]) OAP_AI {
      const _Float16* ap = ph + size_t(c0 + r) * sb + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) av[s] = *reinterpret_cast<const f16x8*>(ap + 16 * s);
    };
    auto chain = [&](const f16x8(&av)[KS], f32x16& acc) OAP_AI {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[0], X[0], f32x16{}, 0, 0, 0);
#pragma unroll
      for (int s = 1; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s], X[s], acc, 0, 0, 0);
    };
    // keys: the distance's bits with the low 10 mantissa bits replaced by the centroid's offset
    // (value order, lowest index first); padded centroids carry the largest finite bias and
    // never win.  NG groups of 8 centroids (4 per lane); the pair fold is 3 VALU per 2 keys.
    auto epi = [&](auto ng_t, int c0, const f32x16& acc) OAP_AI {
      constexpr int NG = decltype(ng_t)::value;
      int key[4 * NG];
#pragma unroll
      for (int e = 0; e < 4 * NG; ++e)
        key[e] = (__float_as_int(acc[e]) & ~0x3ff) | (8 * (e >> 2) + (e & 3));
      int t1 = min(key[0], key[1]), t2 = max(key[0], key[1]);
#pragma unroll
      for (int e = 2; e < 4 * NG; e += 2) {
        t2 = min(t2, med3_i32_pure(t1, key[e], key[e + 1]));
        t1 = min(min(t1, key[e]), key[e + 1]);
      }
      const int base = c0 + 4 * h;
      const int i1 = t1 | base, i2 = t2 | base;
      k2 = min(max(k1, i1), min(k2, i2));
      k1 = min(k1, i1);
    };
    auto epi_last = [&](const f32x16& acc) OAP_AI {
      switch (ng_last) {  // (wave-uniform)
        case 1: epi(std::integral_constant<int, 1>{}, c_last, acc); break;
        case 2: epi(std::integral_constant<int, 2>{}, c_last, acc); break;
        case 3: epi(std::integral_constant<int, 3>{}, c_last, acc); break;
        default: epi(std::integral_constant<int, 4>{}, c_last, acc); break;
      }
    };
    const std::integral_constant<int, 4> full{};
    f16x8 av[KS];
    if constexpr (!PIPE) {
      for (int c0 = 0; c0 < c_last; c0 += 32) {
        f32x16 acc;
        frags(c0, av);
        chain(av, acc);
        epi(full, c0, acc);
      }
      f32x16 acc;
      frags(c_last, av);
      chain(av, acc);
      epi_last(acc);
    } else {
      // chunk c's epilogue runs while chunk c + 1's MFMA chain is in the matrix pipe (its
      // fragment reads land under the tail of chunk c's chain; the fragment registers are dead
      // during the epilogue: two accumulators fit the 128-register budget without spills)
      f32x16 accA, accB;
      frags(0, av);
      chain(av, accA);
      int c0 = 0;
      bool last_in_b = false;
      while (c0 < c_last) {  // invariant: accA holds chunk c0 (issued)
        frags(c0 + 32, av);
        chain(av, accB);
        epi(full, c0, accA);
        c0 += 32;
        if (c0 == c_last) {
          last_in_b = true;
          break;
        }
        frags(c0 + 32, av);
        chain(av, accA);
        epi(full, c0, accB);
        c0 += 32;
      }
      if (last_in_b)
        epi_last(accB);
      else
        epi_last(accA);
    }
    // ---- the two halves of the row: top-2 of the union
    const int o1 = xor32_i(k1), o2 = xor32_i(k2);
    k2 = min(max(k1, o1), min(k2, o2));
    k1 = min(k1, o1);
    const float b1 = __int_as_float(k1 & ~0x3ff);
    const float b2 = __int_as_float(k2 & ~0x3ff);
    const float tt = fmaf(thr_c, __builtin_amdgcn_sqrtf(nx2_s), thr_k) + 5e-5f * nx2_s +
                     2.5e-4f * fabsf(b2);
    // rows beyond fp16's comfortable range (alpha |x| >= 2^10) are always re-decided
    bool unsure = valid && (!(b2 - b1 > tt) || !(nx2_s < 1048576.f));
    // the refined test on the row's own residual (kmeans_frag.h refined_tt; wave-uniform: the
    // residual's exchange needs both halves)
    if (refine && __ballot(unsure) != 0ull) {
      const float em = static_cast<float>(X[KS - 1][3]);
      const float eo = xor32_f(em);
      const float rest = thr_k + 5e-5f * nx2_s + 2.5e-4f * fabsf(b2);
      const float tr = refined_tt(b1, b2, tt, rest, nx2_s, h ? em : eo, r2max);
      unsure = unsure && !(b1 >= 0.f && b2 - b1 > tr && nx2_s < 1048576.f);
    }
    // ---- defer unsure rows (wave-private sub-segment, in tile order)
    const unsigned long long um = __ballot(unsure && h == 0);
    buf_store_b32(rs_def, (n_def + lanes_below(um)) * 4u,
                  static_cast<int32_t>(row), unsure && h == 0);
    n_def += static_cast<unsigned>(__popcll(um));
    const bool done = valid && !unsure;
    int b = k1 & 0x3ff;
    b = (b < k) ? b : 0;  // only for degenerate (NaN / all-inf) inputs
    const bool moved = done && old >= 0 && old != b;
    {
      const unsigned long long mm = __ballot(moved && h == 0);
      if (mm) {
        if (moved && h == 0)
          mv_l[n_mv + lanes_below(mm)] =
              make_int2(static_cast<int>(row), b | (min(old, k - 1) << 16));
        n_mv += static_cast<unsigned>(__popcll(mm));
      }
    }
    // labels: only the rows that moved (the others already hold theirs)
    buf_store_b32(rs_lab, roff * 4, b, moved && h == 0);
    // bounds (when a following iteration may scan): the pick's alpha^2 distance is <= b1 + tt,
    // every other one >= b2 - tt
    float2 bnd = make_float2(0.f, 0.f);
    if (want_bounds) {
      const float mg = fmaf(mrel, nx2_s, mg_c);
      const float up = (b1 + tt + mg) * inv_a2, lo = (b2 - (tt + mg)) * inv_a2;
      bnd = make_float2(__builtin_amdgcn_sqrtf(fmaxf(up, 0.f)) * (1.f + 1e-6f) + 1e-30f,
                        __builtin_amdgcn_sqrtf(fmaxf(lo, 0.f)) * (1.f - 1e-6f));
    }
    buf_store_f2(rs_bnd, roff * 8, bnd, done && h == 0);
  };

  int64_t t = wave;
  unsigned n_pruned = 0;  // (row-scan passes; wave-uniform)
  auto trow = [&](int64_t q) OAP_AI -> int64_t { return tile_of(q) * 32 + r; };  // (dense)
  if constexpr (SCAN) {
    // The wave's dense tiles (t = wave + j stride) are scanned two at a time (h = 0 lanes the
    // first, h = 1 the second): the Hamerly test of kmeans_lean_scan_rows per row.  A pruned
    // row keeps its label and has its bounds advanced in place (rounded outward; no write once
    // no center moves); the others enter the ring in row order.  The ring holds [head, tail):
    // the current tile and the next one (whose operands are prefetched under the current one)
    // are complete before the current tile runs, except at the end of the wave's rows.
    int* ring = reinterpret_cast<int*>(smem + L.ring) + wave * kRing;
    const float dmax = ufl(a.drift[k]);
    const float cm2 = ufl(cmax * cmax);
    // (the tile norms of a pair are wave-uniform: scalar loads, held in SGPRs across the tiles
    // in between, so the prefetch costs the pipelined loop only its three vector registers)
    typedef const float __attribute__((address_space(4)))* xn_cptr;
    const xn_cptr xn_seg = (xn_cptr)(a.scan_xnorm + t0);
    unsigned head = 0, tail = 0;  // wave-uniform ring positions
    int64_t sq = wave;            // the next tile pair to scan (wave-uniform)
    // the scan of tile pair sq reads bounds, label and tile norm one step ahead: issued when the
    // previous pair is consumed, in flight under the tiles in between (an unpredicated issue:
    // offsets past the wave's rows read zeros)
    u32x2 pbw;
    int plab;
    float pxn0, pxn1;
    auto issue = [&]() OAP_AI {
      const int64_t q = sq + h * stride;
      const uint32_t roff = uint32_t(q * 32 + r);
      const bool in = q < dense_pos && int64_t(roff) < wrows;
      pbw = __builtin_bit_cast(
          u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_bnd, in ? roff * 8u : kBufOff, 0, 0));
      plab = buf_load_b32(rs_lab, roff * 4u, in);
      const int64_t q0 = sq < dense_pos ? sq : dense_pos - 1;
      const int64_t q1 = sq + stride < dense_pos ? sq + stride : dense_pos - 1;
      pxn0 = xn_seg[q0 < 0 ? 0 : q0];
      pxn1 = xn_seg[q1 < 0 ? 0 : q1];
    };
    auto refill = [&]() OAP_AI {
      while (tail - head < 64u && sq < dense_pos) {
        const int64_t q = sq + h * stride;
        const uint32_t roff = uint32_t(q * 32 + r);
        const bool in = q < dense_pos && int64_t(roff) < wrows;
        const float u = __uint_as_float(pbw[0]) + dr_l[min(max(plab, 0), k - 1)];
        const float lk = __uint_as_float(pbw[1]) - dmax;
        const float xn = h ? pxn1 : pxn0;
        const bool ok = in && lk > 0.f && (lk - u) * (lk + u) > mrel * (xn + cm2);
        buf_store_f2(rs_bnd, roff * 8u, make_float2(u * (1.f + 2.5e-7f), lk * (1.f - 2.5e-7f)),
                     ok && dmax > 0.f);
        const bool act = in && !ok;
        const unsigned long long m = __ballot(act);
        if (act) ring[(tail + lanes_below(m)) & (kRing - 1)] = static_cast<int>(roff);
        tail += static_cast<unsigned>(__popcll(m));
        n_pruned += static_cast<unsigned>(__popcll(__ballot(ok)));
        sq += 2 * stride;
        issue();
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    issue();
    // this lane's row of the tile starting at ring position i (-1 past the tail)
    auto ring_row = [&](unsigned i) OAP_AI -> int64_t {
      const int e = ring[(i + unsigned(r)) & (kRing - 1)];
      return i + unsigned(r) < tail ? row0 + e : int64_t(-1);
    };
    // (the rows of the current tile are re-read from the ring rather than carried across a
    // tile: after a refill the current tile is complete unless the scan is exhausted, so its
    // slots — whose operands were prefetched — are unchanged)
    const int64_t rfix = row0;
    f16x8 xa[KS], xb[KS];
    refill();
    {
      const int64_t r0v = ring_row(head);
      load_img_row(r0v >= 0 ? r0v : rfix, xa);
    }
    while (head < tail) {  // (wave-uniform)
      refill();
      {
        const int64_t nx = ring_row(head + 32u);
        body(std::true_type{}, 0, ring_row(head), nx >= 0 ? nx : rfix, xa, xb);
      }
      head = tail - head > 32u ? head + 32u : tail;
      if (head == tail) break;
      refill();
      {
        const int64_t nx = ring_row(head + 32u);
        body(std::true_type{}, 0, ring_row(head), nx >= 0 ? nx : rfix, xb, xa);
      }
      head = tail - head > 32u ? head + 32u : tail;
    }
  } else {
    f16x8 xa[KS], xb[KS];
    load_img_row(trow(t), xa);
    for (; t < npos; t += 2 * stride) {  // t is wave-uniform: every branch stays uniform
      body(std::true_type{}, t, trow(t), trow(t + stride), xa, xb);
      if (t + stride >= npos) break;
      body(std::true_type{}, t + stride, trow(t + stride), trow(t + 2 * stride), xb, xa);
    }
  }
  while (n_mv) {  // (at most 63 staged)
    flush(n_mv);
    n_mv = n_mv > 32 ? n_mv - 32 : 0;
  }
  if (lane == 0) {
    if (a.stat && blockIdx.x == 0 && wave == 0) atomicAdd(a.stat + 2, 1ull);  // (image passes)
    a.defer_row_count[blockIdx.x * kDeferSubs + wave] = n_def;
    if (a.stat && n_def) atomicAdd(a.stat, u64(n_def));
    if (a.stat && moved_total) atomicAdd(a.stat + 1, moved_total);
    if (SCAN && a.pruned && n_pruned) atomicAdd(a.pruned, u64(n_pruned));
  }
  __syncthreads();
  for (int i = tid; i < k * d; i += NT) {
    const int c = i / d, f = i - c * d;
    const double v = acc_l[c * rs + f];  // an exact integer, |v| < 2^53
    if (v != 0.0) atomicAdd(&a.sums[i], static_cast<u64>(static_cast<long long>(v)));
  }
  for (int i = tid; i < k; i += NT) {
    const int c = cnt_l[i];
    if (c) atomicAdd(&a.counts[i], static_cast<u64>(static_cast<long long>(c)));
  }
}

template <int KS, int WAVES, int CFG, int RM>
void launch_img_l(const ImgArgs& a, int grid, hipStream_t s) {
  const ImgSmem L = img_plan(16 * KS, a.kpad, a.k, WAVES, RM == 2);
  static bool attr_set = false;
  if (!attr_set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&oap_kmeans_lean_img<KS, WAVES, CFG, RM>),
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
    attr_set = true;
  }
  hipLaunchKernelGGL((oap_kmeans_lean_img<KS, WAVES, CFG, RM>), dim3(grid), dim3(WAVES * 64),
                     L.total, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

template <int KS, int WAVES, int CFG>
void launch_img(const ImgArgs& a, int grid, hipStream_t s) {
  if (a.scan_xnorm)
    launch_img_l<KS, WAVES, CFG, 2>(a, grid, s);
  else
    launch_img_l<KS, WAVES, CFG, 0>(a, grid, s);
}

constexpr int kImgDefaultCfg = 1;  // pipelined chunk loop, operands one tile ahead

// Production configurations: 0 (row-scan passes: the scan's prefetched bounds fit the
// non-pipelined loop's registers) and 1 (dense passes: the pipelined chunk loop).  The timing
// ablation builds of rounds 3-5 (no epilogue / MFMA / plane reads / loads / accumulation / stores,
// operands two tiles ahead) live in git history.
template <int KS, int WAVES>
void launch_img_cfg(const ImgArgs& a, int grid, int cfg, hipStream_t s) {
  OAP_CHECK(cfg == 0 || cfg == 1, "kmeans_lean_img: configuration " << cfg << " (0 or 1)");
  if (cfg == 0 && a.scan_xnorm)
    launch_img<KS, WAVES, 0>(a, grid, s);
  else if (cfg == 0)
    launch_img<KS, WAVES, 0>(a, grid, s);
  else
    launch_img<KS, WAVES, 1>(a, grid, s);
}

template <int WAVES>
void launch_img_w(const ImgArgs& a, int grid, int cfg, hipStream_t s) {
  switch ((a.d + 4 + 15) / 16) {
    case 1: launch_img_cfg<1, WAVES>(a, grid, cfg, s); break;
    case 2: launch_img_cfg<2, WAVES>(a, grid, cfg, s); break;
    case 3: launch_img_cfg<3, WAVES>(a, grid, cfg, s); break;
    case 4: launch_img_cfg<4, WAVES>(a, grid, cfg, s); break;
    case 5: launch_img_cfg<5, WAVES>(a, grid, cfg, s); break;
    case 6: launch_img_cfg<6, WAVES>(a, grid, cfg, s); break;
    case 7: launch_img_cfg<7, WAVES>(a, grid, cfg, s); break;
    case 8: launch_img_cfg<8, WAVES>(a, grid, cfg, s); break;
    default: OAP_THROW(ConfigError, "kmeans_lean_img: unsupported d=" << a.d);
  }
}

constexpr int kDecideBlocks = 64;
constexpr int kDecideThreads = 256;
constexpr int kDecidePerThread = 4;  // 65536 sampled rows, every load of a thread in flight

// scratch[0]: blocks done, scratch[1]: prunable samples (zero on entry; the last block resets)
__global__ __launch_bounds__(kDecideThreads) void oap_kmeans_scan_decide(
    int64_t n, int k, int d, const float2* __restrict__ bounds,
    const int32_t* __restrict__ labels, const float* __restrict__ xnorm,
    const float* __restrict__ drift, const float* __restrict__ cstat, float min_frac,
    int* __restrict__ gate, unsigned* __restrict__ scratch, const int* __restrict__ halt) {
  if (halt && *halt) return;
  __shared__ unsigned wsum[kDecideThreads / 64];
  __shared__ bool s_last;
  const int tid = threadIdx.x;
  const float dmax = drift[k];
  const float cmax = cstat[0];
  const float mrel = 4e-7f * float(d + 8);
  constexpr int64_t kS = int64_t(kDecideBlocks) * kDecideThreads * kDecidePerThread;
  const int64_t S = n < kS ? n : kS;
  float2 b[kDecidePerThread];
  int lab[kDecidePerThread];
  float xn[kDecidePerThread];
  bool in[kDecidePerThread];
#pragma unroll
  for (int j = 0; j < kDecidePerThread; ++j) {
    const int64_t i = (int64_t(j) * kDecideBlocks + blockIdx.x) * kDecideThreads + tid;
    in[j] = i < S;
    const int64_t row = in[j] ? static_cast<int64_t>((double(i) + 0.5) * double(n) / double(S))
                              : 0;
    b[j] = bounds[row];
    lab[j] = labels[row];
    xn[j] = xnorm[row >> 5];
  }
  unsigned ok_n = 0;
#pragma unroll
  for (int j = 0; j < kDecidePerThread; ++j) {
    const float u = b[j].x + drift[min(max(lab[j], 0), k - 1)];
    const float lk = b[j].y - dmax;
    ok_n += (in[j] && lk > 0.f && (lk - u) * (lk + u) > mrel * (xn[j] + cmax * cmax)) ? 1u : 0u;
  }
  for (int m = 32; m >= 1; m >>= 1) ok_n += __shfl_xor(ok_n, m, 64);
  if ((tid & 63) == 0) wsum[tid >> 6] = ok_n;
  __syncthreads();
  if (tid == 0) {
    unsigned t = 0;
    for (int w = 0; w < kDecideThreads / 64; ++w) t += wsum[w];
    if (t) atomicAdd(&scratch[1], t);
    __threadfence();
    s_last = atomicAdd(&scratch[0], 1u) == kDecideBlocks - 1;
  }
  __syncthreads();
  if (s_last && tid == 0) {
    __threadfence();
    const unsigned tot = atomicAdd(&scratch[1], 0u);
    gate[0] = double(tot) >= double(min_frac) * double(S) ? 1 : 0;
    scratch[0] = 0u;
    scratch[1] = 0u;
  }
}

}  // namespace

void kmeans_scan_decide(int64_t n, int k, int d, const float* bounds, const int32_t* labels,
                        const float* xnorm, const float* drift, const float* cstat,
                        float min_frac, int* gate, const int* halt, hipStream_t s) {
  OAP_CHECK(k >= 1 && gate && bounds && labels && xnorm && drift && cstat,
            "kmeans_scan_decide: bad arguments");
  if (n <= 0) return;
  // gate[0]: the choice; gate[2..3]: the kernel's block counter and sum (zeroed by the caller
  // once, reset by the kernel's last block)
  hipLaunchKernelGGL(oap_kmeans_scan_decide, dim3(kDecideBlocks), dim3(kDecideThreads), 0, s, n,
                     k, d, reinterpret_cast<const float2*>(bounds), labels, xnorm, drift, cstat,
                     min_frac, gate, reinterpret_cast<unsigned*>(gate + 2), halt);
  OAP_HIP_CHECK(hipGetLastError());
}

bool kmeans_refine_default() {  // (read per launch: tests switch it within a process)
  return knob_int("OAP_KMEANS_REFINE") != 0;
}

bool kmeans_lean_img_supported(int d, int k, int waves, bool scan) {
  if (d + 4 > 128 || k < 1 || (waves != 12 && waves != 16)) return false;
  const int dp = (d + 4 + 15) / 16 * 16;
  if (dp != kmeans_dp(d)) return false;
  const int kpad = (k + 31) / 32 * 32;
  if (kpad > 1024) return false;
  return img_plan(dp, kpad, k, waves, scan).total <= kLdsLimit;
}

void kmeans_lean_img(const KMeansAssignArgs& a, int grid, int waves, int cfg, hipStream_t s) {
  const bool scan = a.img_scan_xnorm != nullptr;
  OAP_CHECK(kmeans_lean_img_supported(a.d, a.k, waves, scan) && !a.xbf16 &&
                a.ximg && a.img_beta &&
                a.delta && a.labels && a.scale && a.sums && a.counts && a.accumulate &&
                a.sums_too && a.defer_rows && a.defer_row_count && a.cstat && !a.xnorm &&
                !a.cost_slab && !a.mindist && !a.centers_all && a.chunk_mode == 0 &&
                a.row_seg_cap == kmeans_lloyd_seg_cap(a.n, grid, waves) &&
                a.ld == kmeans_ld(a.d, false) && (!a.tile_list || a.tile_count) &&
                (!scan || (a.img_scan_drift && a.bounds && !a.tile_list)),
            "kmeans_lean_img: unsupported arguments");
  if (a.n == 0) return;
  ImgArgs l;
  l.img = static_cast<const f16x8*>(a.ximg);
  l.img_beta = a.img_beta;
  l.x = static_cast<const float*>(a.x);
  l.centers = a.centers;
  l.cnorm = a.cnorm;
  l.cstat = a.cstat;
  l.scale = a.scale;
  l.sums = a.sums;
  l.counts = a.counts;
  l.labels = a.labels;
  l.bounds = reinterpret_cast<float2*>(a.bounds);
  l.tile_list = a.tile_list;
  l.tile_count = a.tile_count;
  l.defer_rows = a.defer_rows;
  l.defer_row_count = a.defer_row_count;
  l.stat = a.deferred_rows;
  l.scan_xnorm = a.img_scan_xnorm;
  l.drift = a.img_scan_drift;
  l.pruned = a.img_scan_pruned;
  l.n = a.n;
  l.seg_cap = a.row_seg_cap;
  l.tiles_per_block = kmeans_lloyd_tiles_per_block(a.n, grid);
  l.ld = a.ld;
  l.d = a.d;
  l.k = a.k;
  l.kpad = a.kpad;
  l.refine = kmeans_refine_default() ? 1 : 0;
  l.halt = a.halt;
  l.gate = a.img_gate;
  l.gate_on = a.img_gate_on;
  if (waves == 12)
    launch_img_w<12>(l, grid, cfg < 0 ? kImgDefaultCfg : cfg, s);
  else
    launch_img_w<16>(l, grid, cfg < 0 ? kImgDefaultCfg : cfg, s);
}

}  // namespace kern
}  // namespace oap
