// PCA covariance statistics: fused shifted SYRK + column sums on MFMA.
//
// Replaces the reference's two passes — Spark StandardScaler centring (mllib-dal/src/main/scala/
// org/apache/spark/ml/feature/PCADALImpl.scala:101-106) followed by oneDAL's fp64 step1Local
// cross-product (native/PCADALImpl.cpp:63-69) — with ONE pass over the HBM-resident fp32 rows:
//
//   S = sum_rows (x - s)(x - s)^T      (upper 128x128 tiles only)
//   c = sum_rows (x - s)               (diagonal tiles)
//
// where s is a global shift close to the mean, so the later correction
// cov = (S - c c^T / n) / (n - 1) has no catastrophic cancellation.
//
// Products run on v_mfma_f32_32x32x16_bf16 with the 2-term bf16 split of (x - s):
// hi*hi + hi*lo + lo*hi (+ lo*lo with `four`), i.e. ~2^-17 relative per product, accumulated in
// fp32 for at most `flush_chunks` x 32 rows and then added into a per-workgroup fp64 slab that
// only this workgroup owns (deterministic); a second kernel sums the slabs in split order.
//
// Workgroup = 4 waves on one 128x128 output tile (each wave 64x64 = 2x2 MFMA blocks); rows are
// staged 32 at a time through LDS transposed to [feature][row] bf16 hi/lo planes (2 x 40 KB,
// double buffered: chunk c+1 is loaded and converted while chunk c feeds the MFMAs, one barrier
// per chunk), so A and B fragments are single 16-byte LDS reads.  Blocks are remapped so that
// all tiles of one row split land on one XCD and share its L2.
#include "kernels/device_utils.h"
#include "kernels/kernels.h"
#include "runtime/common.h"

namespace oap {
namespace kern {

namespace {

constexpr int kTile = 128;
constexpr int kChunk = 32;             // rows per LDS stage
constexpr int kPS = kChunk + 8;        // plane row stride in bf16 (80 B: conflict-free b128 reads)
constexpr int kPlane = kTile * kPS;    // bf16 elements per plane
constexpr int kSyrkThreads = 256;

struct SyrkArgs {
  const float* x;
  int64_t n, ld;
  int d;
  const float* shift;  // [nb*128], zero padded
  int nb, tiles, splits, flush_chunks;
  int64_t rows_per_split;
  double* part;   // [splits][tiles][128*128]
  double* cpart;  // [splits][nb][128]
};

__device__ inline void tile_coords(int tile, int nb, int& ti, int& tj) {
  int t = 0, rem = tile;
  while (rem >= nb - t) {
    rem -= nb - t;
    ++t;
  }
  ti = t;
  tj = t + rem;
}

template <bool FOUR>
__global__ __launch_bounds__(kSyrkThreads, 2) void oap_pca_syrk(SyrkArgs a) {
  // two stages x [side][plane hi/lo]: chunk c+1 is staged while chunk c feeds the MFMAs
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 4 * kPlane];
  const int G = a.splits * a.tiles;
  const int per = gridDim.x / 8;  // gridDim.x is a multiple of 8
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= G) return;
  const int split = L / a.tiles, tile = L - split * a.tiles;
  int ti, tj;
  tile_coords(tile, a.nb, ti, tj);
  const bool diag = ti == tj;
  const int64_t r_begin = int64_t(split) * a.rows_per_split;
  const int64_t r_end = min(a.n, r_begin + a.rows_per_split);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wi = wave >> 1, wj = wave & 1;
  // loader: rows 4*lg .. 4*lg+3 of the stage, features 4*lq .. 4*lq+3 of each side
  const int lg = tid & 7, lq = tid >> 3;
  const int fi = ti * kTile + 4 * lq, fj = tj * kTile + 4 * lq;
  const bool okI = fi < a.ld, okJ = fj < a.ld;
  const float4 shI = *reinterpret_cast<const float4*>(a.shift + fi);
  const float4 shJ = *reinterpret_cast<const float4*>(a.shift + fj);

  // two register stages: the rows of chunk c+2 are in flight while chunk c feeds the MFMAs and
  // chunk c+1 (loaded one chunk earlier) is converted into the other LDS buffer
  float4 vIa[4], vJa[4], vIb[4], vJb[4];
  double cs[4] = {0.0, 0.0, 0.0, 0.0};
  // Loads are unconditional (row clamped to r_end - 1, feature group clamped to 0): no
  // per-row branches; stage() zeroes what lies outside the matrix.
  const int fiL = okI ? fi : 0, fjL = okJ ? fj : 0;
  auto load = [&](int64_t r0, float4 (&vI)[4], float4 (&vJ)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = min(r0 + 4 * lg + i, r_end - 1);
      const float* p = a.x + row * a.ld;
      vI[i] = *reinterpret_cast<const float4*>(p + fiL);
      if (!diag) vJ[i] = *reinterpret_cast<const float4*>(p + fjL);
    }
  };
  // centre, split, transpose into the planes; rows past r_end contribute exact zeros
  auto stage = [&](__bf16* buf, int64_t r0, int side, const float4 (&v)[4], const float4 sh,
                   bool sums) {
    __bf16* hi = buf + (2 * side) * kPlane;
    __bf16* lo = hi + kPlane;
    const bool okF = side == 0 ? okI : okJ;
    float c[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = okF && r0 + 4 * lg + i < r_end;
      c[0][i] = ok ? v[i].x - sh.x : 0.f;
      c[1][i] = ok ? v[i].y - sh.y : 0.f;
      c[2][i] = ok ? v[i].z - sh.z : 0.f;
      c[3][i] = ok ? v[i].w - sh.w : 0.f;
    }
    if (sums) {  // column sums: 4 rows in fp32, then fp64 across chunks
#pragma unroll
      for (int f = 0; f < 4; ++f)
        cs[f] += static_cast<double>((c[f][0] + c[f][1]) + (c[f][2] + c[f][3]));
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 ph, pl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __bf16 a_, b_;
        bf16_split(c[f][i], a_, b_);
        ph[i] = a_;
        pl[i] = b_;
      }
      const int off = (4 * lq + f) * kPS + 4 * lg;
      *reinterpret_cast<bf16x4*>(hi + off) = ph;
      *reinterpret_cast<bf16x4*>(lo + off) = pl;
    }
  };

  f32x16 acc[2][2];
  auto zero = [&]() {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;
  };
  zero();
  double* slab = a.part + (size_t(split) * a.tiles + tile) * (kTile * kTile);
  bool first = true;
  auto flush = [&]() {
    // laundered per-lane base: keeps the 64 element addresses from being hoisted out of the row
    // loop as live registers
    double* base = slab + (64 * wi + 4 * h) * kTile + 64 * wj + r;
    asm volatile("" : "+v"(base));
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          double* p = base + (32 * x + (e & 3) + 8 * (e >> 2)) * kTile + 32 * y;
          const double v = static_cast<double>(acc[x][y][e]);
          *p = first ? v : *p + v;
          if ((e & 3) == 3) asm volatile("" ::: "memory");  // bound the loads in flight
        }
    first = false;
    zero();
  };

  const int aoff = (64 * wi + r) * kPS + 8 * h;
  const int boff = (diag ? 0 : 2 * kPlane) + (64 * wj + r) * kPS + 8 * h;
  int since = 0, cur = 0;
  if (r_begin < r_end) {
    load(r_begin, vIa, vJa);
    stage(lds, r_begin, 0, vIa, shI, diag);
    if (!diag) stage(lds, r_begin, 1, vJa, shJ, false);
    if (r_begin + kChunk < r_end) load(r_begin + kChunk, vIb, vJb);
    lds_barrier();
  }
  // one chunk: MFMAs on LDS buffer `cur`; rows of chunk r0 + 2 kChunk -> (nI, nJ) (the set that
  // held chunk r0, already staged); chunk r0 + kChunk from (sI, sJ) -> the other LDS buffer
  auto step = [&](int64_t r0, float4 (&sI)[4], float4 (&sJ)[4], float4 (&nI)[4],
                  float4 (&nJ)[4]) {
    const bool more = r0 + kChunk < r_end;
    if (r0 + 2 * kChunk < r_end) load(r0 + 2 * kChunk, nI, nJ);  // in flight for 2 chunks
    const __bf16* aH = lds + cur * (4 * kPlane) + aoff;
    const __bf16* bH = lds + cur * (4 * kPlane) + boff;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        ah[x] = *reinterpret_cast<const bf16x8*>(aH + 32 * x * kPS + 16 * ks);
        al[x] = *reinterpret_cast<const bf16x8*>(aH + kPlane + 32 * x * kPS + 16 * ks);
        bh[x] = *reinterpret_cast<const bf16x8*>(bH + 32 * x * kPS + 16 * ks);
        bl[x] = *reinterpret_cast<const bf16x8*>(bH + kPlane + 32 * x * kPS + 16 * ks);
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[x], bh[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[x], bl[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[x], bh[y], acc[x][y], 0, 0, 0);
          if (FOUR)
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[x], bl[y], acc[x][y], 0, 0, 0);
        }
    }
    if (more) {  // the other buffer was last read before the previous barrier
      __bf16* nb = lds + (cur ^ 1) * (4 * kPlane);
      stage(nb, r0 + kChunk, 0, sI, shI, diag);
      if (!diag) stage(nb, r0 + kChunk, 1, sJ, shJ, false);
    }
    lds_barrier();
    cur ^= 1;
    if (++since == a.flush_chunks) {
      flush();
      since = 0;
    }
  };
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 2 * kChunk) {
    step(r0, vIb, vJb, vIa, vJa);
    if (r0 + kChunk >= r_end) break;
    step(r0 + kChunk, vIa, vJa, vIb, vJb);
  }
  if (first || since > 0) flush();
  if (diag) {  // column sums: the 8 loader lanes of one feature group are adjacent
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      double v = cs[f];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (lg == 0) a.cpart[(size_t(split) * a.nb + ti) * kTile + 4 * lq + f] = v;
    }
  }
}

// 256 x 256 output tile per workgroup (d > 128): 8 waves in a 2 x 4 grid, each 128 x 64
// (4 x 2 MFMA blocks, 128 accumulator registers).  Per staged row the tile does twice the MFMA
// work of the 128-wide kernel, so the per-row staging VALU, the LDS writes, the barriers and the
// L2 / HBM traffic per flop all halve.  32-row chunks, two LDS stages (160 KB): chunk c+1 is
// converted into the other stage while chunk c feeds the MFMAs (one barrier per chunk), and the
// rows of chunk c+2 are in flight in registers.
constexpr int kTile2 = 256;
constexpr int kChunk2 = 32;
constexpr int kPS2 = kChunk2 + 8;        // 80 B per feature row: conflict-free b128 reads
constexpr int kRpt2 = kChunk2 / 8;      // rows per loader thread
constexpr int kPlane2 = kTile2 * kPS2;
constexpr int kSyrk2Threads = 512;

template <bool FOUR>
__global__ __launch_bounds__(kSyrk2Threads) void oap_pca_syrk_w256(SyrkArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 4 * kPlane2];  // [stage][side][hi|lo]
  const int G = a.splits * a.tiles;
  const int per = gridDim.x / 8;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= G) return;
  const int split = L / a.tiles, tile = L - split * a.tiles;
  int ti, tj;
  tile_coords(tile, a.nb, ti, tj);
  const bool diag = ti == tj;
  const int64_t r_begin = int64_t(split) * a.rows_per_split;
  const int64_t r_end = min(a.n, r_begin + a.rows_per_split);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wi = wave >> 2, wj = wave & 3;
  // loader: rows kRpt2*lg .. kRpt2*lg+kRpt2-1 of the chunk, features 4*lq .. 4*lq+3 of each side
  const int lg = tid & 7, lq = tid >> 3;
  const int fi = ti * kTile2 + 4 * lq, fj = tj * kTile2 + 4 * lq;
  const bool okI = fi < a.ld, okJ = fj < a.ld;
  const int fiL = okI ? fi : 0, fjL = okJ ? fj : 0;
  const float4 shI = *reinterpret_cast<const float4*>(a.shift + fi);
  const float4 shJ = *reinterpret_cast<const float4*>(a.shift + fj);

  float4 vI[kRpt2], vJ[kRpt2];
  double cs[4] = {0.0, 0.0, 0.0, 0.0};
  auto load = [&](int64_t r0) {
#pragma unroll
    for (int i = 0; i < kRpt2; ++i) {
      const int64_t row = min(r0 + kRpt2 * lg + i, r_end - 1);
      const float* p = a.x + row * a.ld;
      vI[i] = *reinterpret_cast<const float4*>(p + fiL);
      if (!diag) vJ[i] = *reinterpret_cast<const float4*>(p + fjL);
    }
  };
  auto stage = [&](__bf16* buf, int64_t r0, int side, const float4 (&v)[kRpt2], const float4 sh,
                   bool sums) {
    __bf16* hi = buf + (2 * side) * kPlane2;
    __bf16* lo = hi + kPlane2;
    const bool okF = side == 0 ? okI : okJ;
    float c[4][kRpt2];
#pragma unroll
    for (int i = 0; i < kRpt2; ++i) {
      const bool ok = okF && r0 + kRpt2 * lg + i < r_end;
      c[0][i] = ok ? v[i].x - sh.x : 0.f;
      c[1][i] = ok ? v[i].y - sh.y : 0.f;
      c[2][i] = ok ? v[i].z - sh.z : 0.f;
      c[3][i] = ok ? v[i].w - sh.w : 0.f;
    }
    if (sums) {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < kRpt2; ++i) t += c[f][i];
        cs[f] += static_cast<double>(t);
      }
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      typedef __bf16 bf16xr __attribute__((ext_vector_type(kRpt2)));
      bf16xr ph, pl;
#pragma unroll
      for (int i = 0; i < kRpt2; ++i) {
        __bf16 a_, b_;
        bf16_split(c[f][i], a_, b_);
        ph[i] = a_;
        pl[i] = b_;
      }
      const int off = (4 * lq + f) * kPS2 + kRpt2 * lg;
      *reinterpret_cast<bf16xr*>(hi + off) = ph;
      *reinterpret_cast<bf16xr*>(lo + off) = pl;
    }
  };

  f32x16 acc[4][2];
  auto zero = [&]() {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;
  };
  zero();
  double* slab = a.part + (size_t(split) * a.tiles + tile) * (size_t(kTile2) * kTile2);
  bool first = true;
  auto flush = [&]() {
    double* base = slab + (128 * wi + 4 * h) * kTile2 + 64 * wj + r;
    asm volatile("" : "+v"(base));
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          double* p = base + (32 * x + (e & 3) + 8 * (e >> 2)) * kTile2 + 32 * y;
          const double v = static_cast<double>(acc[x][y][e]);
          *p = first ? v : *p + v;
          if ((e & 3) == 3) asm volatile("" ::: "memory");
        }
    first = false;
    zero();
  };

  const int aoff = (128 * wi + r) * kPS2 + 8 * h;
  const int boff = (diag ? 0 : 2 * kPlane2) + (64 * wj + r) * kPS2 + 8 * h;
  const int flush_every = a.flush_chunks * (kChunk / kChunk2);  // same rows per flush
  int since = 0, cur = 0;
  if (r_begin < r_end) {
    load(r_begin);
    stage(lds, r_begin, 0, vI, shI, diag);
    if (!diag) stage(lds, r_begin, 1, vJ, shJ, false);
    if (r_begin + kChunk2 < r_end) load(r_begin + kChunk2);
    lds_barrier();
  }
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kChunk2) {
    const __bf16* buf = lds + cur * (4 * kPlane2);
#pragma unroll
    for (int ks = 0; ks < kChunk2 / 16; ++ks) {
      bf16x8 ah[4], al[4], bh[2], bl[2];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        ah[x] = *reinterpret_cast<const bf16x8*>(buf + aoff + 32 * x * kPS2 + 16 * ks);
        al[x] = *reinterpret_cast<const bf16x8*>(buf + kPlane2 + aoff + 32 * x * kPS2 + 16 * ks);
      }
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        bh[y] = *reinterpret_cast<const bf16x8*>(buf + boff + 32 * y * kPS2 + 16 * ks);
        bl[y] = *reinterpret_cast<const bf16x8*>(buf + kPlane2 + boff + 32 * y * kPS2 + 16 * ks);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[x], bh[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[x], bl[y], acc[x][y], 0, 0, 0);
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[x], bh[y], acc[x][y], 0, 0, 0);
          if (FOUR)
            acc[x][y] =
                __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[x], bl[y], acc[x][y], 0, 0, 0);
        }
    }
    if (r0 + kChunk2 < r_end) {  // the other stage was last read before the previous barrier
      __bf16* nb = lds + (cur ^ 1) * (4 * kPlane2);
      stage(nb, r0 + kChunk2, 0, vI, shI, diag);
      if (!diag) stage(nb, r0 + kChunk2, 1, vJ, shJ, false);
      if (r0 + 2 * kChunk2 < r_end) load(r0 + 2 * kChunk2);
    }
    lds_barrier();
    cur ^= 1;
    if (++since == flush_every) {
      flush();
      since = 0;
    }
  }
  if (first || since > 0) flush();
  if (diag) {  // column sums: the 8 loader lanes of one feature group are adjacent
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      double v = cs[f];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (lg == 0) a.cpart[(size_t(split) * a.nb + ti) * kTile2 + 4 * lq + f] = v;
    }
  }
}

// ---- exact mode: fp64 products, fp64 accumulation (v_mfma_f64_16x16x4_f64) -------------------
// The reference's precision (oneDAL fp64 step1Local, PCADALImpl.cpp:31,63-69): every product
// (x_i - s_i)(x_j - s_j) is formed and summed in fp64 — fp32 rows are widened exactly, fp64 rows
// are used as they are.  128 x 128 output tile per 256-thread workgroup; each wave owns a 64 x 64
// quarter = 4 x 4 blocks of 16 x 16 (16 independent accumulators of 4 doubles).  Rows are staged
// 16 at a time through LDS as fp64 [feature][row] planes (double buffered, one barrier per
// chunk); an A or B fragment is ONE ds_read_b64 per lane.  The accumulators are fp64 for the
// whole split: no intermediate flush, the slab is written once.
// 8 waves (2 x 4) of 64 x 32 each: 8 accumulators (64 VGPRs) per wave — with 16 per wave the
// f64 MFMA chain ran at under half its rate (measured: tools/mfma_f64_probe.hip, 71-78 TFLOP/s
// with 8 independent accumulators per wave, 30-37 with 16).
constexpr int kXTile = 128;
constexpr int kXRows = 32;              // rows per LDS stage (8 k-steps of the 16x16x4 MFMA)
constexpr int kXS = kXRows + 2;         // plane stride in doubles (68 dwords: conflict-free)
constexpr int kXPlane = kXTile * kXS;   // doubles per side plane
constexpr int kXThreads = 512;

typedef double f64x4 __attribute__((ext_vector_type(4)));

struct SyrkF64Args {
  const void* x;
  int64_t n, ld;
  int d;
  const double* shift;  // [nb*128], zero padded
  int nb, tiles, splits;
  int64_t rows_per_split;
  double* part;         // [splits][tiles][128*128]
  double* cpart;        // [splits][nb][128]
};

// 4 features f0 .. f0+3 of one row, loaded unconditionally (a group past the row end reads the
// row's first group instead; stage() zeroes every feature >= d): a conditional load ends in a
// divergent region whose join waits for it (s_waitcnt vmcnt(0) right behind each load), which
// serialised the row prefetch.  VEC: 16-byte aligned rows and ld % 4 == 0.
template <typename T, bool VEC>
__device__ inline void load4(const T* __restrict__ p, int f0, int ld, T (&v)[4]) {
  if constexpr (VEC) {
    const int fl = f0 < ld ? f0 : 0;
    if constexpr (sizeof(T) == 4) {
      const float4 a = *reinterpret_cast<const float4*>(p + fl);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else {
      const double2 a = *reinterpret_cast<const double2*>(p + fl);
      const double2 b = *reinterpret_cast<const double2*>(p + fl + 2);
      v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = p[min(f0 + q, ld - 1)];
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kXThreads, 1) void oap_pca_syrk_f64(SyrkF64Args a) {
  __shared__ double lds[2 * 2 * kXPlane];  // [stage][side][feature][row]
  const int G = a.splits * a.tiles;
  const int per = gridDim.x / 8;  // XCD-aware: the tiles of one split share an XCD (its L2)
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= G) return;
  const int split = L / a.tiles, tile = L - split * a.tiles;
  int ti, tj;
  tile_coords(tile, a.nb, ti, tj);
  const bool diag = ti == tj;
  const int64_t r_begin = int64_t(split) * a.rows_per_split;
  const int64_t r_end = min(a.n, r_begin + a.rows_per_split);
  const T* __restrict__ X = static_cast<const T*>(a.x);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 2, wj = wave & 3;  // 2 x 4 waves, 64 x 32 each
  // loader: rows lr + 16 j (j < kXRows / 16) of the stage, features 4*lq .. 4*lq+3 of each side
  constexpr int kRpt = kXRows / 16;
  const int lr = tid >> 5, lq = tid & 31;
  const int fI = ti * kXTile + 4 * lq, fJ = tj * kXTile + 4 * lq;
  double shI[4], shJ[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    shI[q] = a.shift[fI + q];
    shJ[q] = a.shift[fJ + q];
  }
  // the rows stay in their storage type until stage() widens them: a conversion right behind
  // the load would wait for it (the prefetch must stay in flight under a chunk of MFMAs)
  T vI[kRpt][4], vJ[kRpt][4];
#pragma unroll
  for (int j = 0; j < kRpt; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) vI[j][q] = vJ[j][q] = T(0);
  double cs[4] = {0, 0, 0, 0};
  const int ld = int(a.ld);  // (< 2^31: checked on the host)
  // unconditional loads (row clamped to the split's last row): stage() masks what lies outside
  auto load = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < kRpt; ++j) {
      const T* p = X + min(r0 + lr + 16 * j, r_end - 1) * a.ld;
      load4<T, VEC>(p, fI, ld, vI[j]);
      load4<T, VEC>(p, fJ, ld, vJ[j]);  // (diagonal tiles re-read their own block: no branch)
    }
  };
  // centre (fp64, exact for fp32 rows) and transpose into the planes; rows past r_end and
  // features past d contribute exact zeros — through 0/1 factors, not branches (the loaded
  // values are finite data either way: rows clamped, groups clamped)
  double mI[4], mJ[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    mI[q] = fI + q < a.d ? 1.0 : 0.0;
    mJ[q] = fJ + q < a.d ? 1.0 : 0.0;
  }
  auto stage = [&](double* buf, int64_t r0) {
#pragma unroll
    for (int j = 0; j < kRpt; ++j) {
      const double mr = r0 + lr + 16 * j < r_end ? 1.0 : 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double c = (double(vI[j][q]) - shI[q]) * (mr * mI[q]);
        cs[q] += c;  // (only the diagonal tiles store their column sums)
        buf[(4 * lq + q) * kXS + lr + 16 * j] = c;
      }
      if (!diag) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          buf[kXPlane + (4 * lq + q) * kXS + lr + 16 * j] =
              (double(vJ[j][q]) - shJ[q]) * (mr * mJ[q]);
      }
    }
  };

  f64x4 acc[4][2];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
  // fragments: lane l holds A[i = l & 15][k = l >> 4] = plane[feature][row k]
  const int fa = 64 * wi + (lane & 15), fb = 32 * wj + (lane & 15), kr = lane >> 4;
  const int boff = diag ? 0 : kXPlane;
  int cur = 0;
  if (r_begin < r_end) {
    load(r_begin);
    stage(lds, r_begin);
    if (r_begin + kXRows < r_end) load(r_begin + kXRows);
    lds_barrier();
  }
  // one staged element of the next chunk (el = 8 j + 2 q + side): the staging is spread over
  // the k-steps, between MFMA groups, instead of running as its own phase before the barrier
  // (same elements, same order per column sum: bitwise the phase form)
  auto stage_el = [&](double* nb, int64_t rn, int el) {
    const int side = el & 1, q = (el >> 1) & 3, j = el >> 3;
    const double mr = rn + lr + 16 * j < r_end ? 1.0 : 0.0;
    if (side == 0) {
      const double c = (double(vI[j][q]) - shI[q]) * (mr * mI[q]);
      cs[q] += c;
      nb[(4 * lq + q) * kXS + lr + 16 * j] = c;
    } else if (!diag) {
      nb[kXPlane + (4 * lq + q) * kXS + lr + 16 * j] = (double(vJ[j][q]) - shJ[q]) * (mr * mJ[q]);
    }
  };
  constexpr int kEl = kRpt * 8, kPerStep = kEl / (kXRows / 4);
  static_assert(kEl % (kXRows / 4) == 0, "staging elements per k-step");
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kXRows) {
    const double* buf = lds + cur * (2 * kXPlane);
    double* nbuf = lds + (cur ^ 1) * (2 * kXPlane);  // last read before the previous barrier
    const bool more = r0 + kXRows < r_end;
    // fragments one k-step ahead (two register sets): k-step ks + 1's LDS reads are in flight
    // under k-step ks's MFMAs instead of waited for between them (the staging writes between
    // the steps target the other stage, but the compiler cannot tell, so it never hoisted them)
    double av[2][4], bv[2][2];
    auto frag = [&](int ks, double (&a4)[4], double (&b2)[2]) {
#pragma unroll
      for (int x = 0; x < 4; ++x) a4[x] = buf[(fa + 16 * x) * kXS + 4 * ks + kr];
#pragma unroll
      for (int y = 0; y < 2; ++y) b2[y] = buf[boff + (fb + 16 * y) * kXS + 4 * ks + kr];
    };
    frag(0, av[0], bv[0]);
#pragma unroll
    for (int ks = 0; ks < kXRows / 4; ++ks) {
      const int cs = ks & 1;
      if (ks + 1 < kXRows / 4) frag(ks + 1, av[cs ^ 1], bv[cs ^ 1]);
      __builtin_amdgcn_sched_barrier(0);  // (the reads stay ahead of this step's MFMAs)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] =
              __builtin_amdgcn_mfma_f64_16x16x4f64(av[cs][x], bv[cs][y], acc[x][y], 0, 0, 0);
      if (more) {
#pragma unroll
        for (int e = 0; e < kPerStep; ++e) stage_el(nbuf, r0 + kXRows, ks * kPerStep + e);
      }
    }
    if (more && r0 + 2 * kXRows < r_end) load(r0 + 2 * kXRows);
    lds_barrier();
    cur ^= 1;
  }
  // the split's fp64 sums, written once: C/D map col = lane & 15, row = (lane >> 4) + 4 reg
  double* slab = a.part + (size_t(split) * a.tiles + tile) * (kXTile * kXTile);
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 64 * wi + 16 * x + (lane >> 4) + 4 * e;
        const int col = 32 * wj + 16 * y + (lane & 15);
        slab[row * kXTile + col] = acc[x][y][e];
      }
  if (diag) {  // column sums over the 16 loader rows: through LDS (the stages are free now)
#pragma unroll
    for (int q = 0; q < 4; ++q) lds[lr * kXTile + 4 * lq + q] = cs[q];
    __syncthreads();
    if (tid < kXTile) {
      double v = 0.0;
      for (int q = 0; q < 16; ++q) v += lds[q * kXTile + tid];
      a.cpart[(size_t(split) * a.nb + ti) * kXTile + tid] = v;
    }
  }
}

// cov = (S - c c^T / n) / (n - 1) on the device (the host formula, operation for operation)
__global__ void oap_pca_cov(const double* __restrict__ stats, int d, double n,
                            double* __restrict__ cov) {
  const double* S = stats;
  const double* c = stats + size_t(d) * d;
  const int64_t total = int64_t(d) * d;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int i = static_cast<int>(idx / d), j = static_cast<int>(idx - int64_t(i) * d);
    const double q = c[i] * c[j];
    cov[idx] = (S[idx] - q / n) / (n - 1.0);
  }
}

__global__ void oap_pca_reduce(const double* __restrict__ part, const double* __restrict__ cpart,
                               int splits, int tiles, int nb, int d, int tw,
                               double* __restrict__ out, double* __restrict__ colsum) {
  const int kTile = tw;  // 128 or 256
  const int64_t total = int64_t(tiles) * kTile * kTile;
  for (int64_t idx = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int tile = static_cast<int>(idx / (kTile * kTile));
    const int e = static_cast<int>(idx - int64_t(tile) * kTile * kTile);
    int ti, tj;
    tile_coords(tile, nb, ti, tj);
    const int ii = e / kTile, jj = e - ii * kTile;
    const int i = ti * kTile + ii, j = tj * kTile + jj;
    if (i >= d || j >= d || (ti == tj && ii > jj)) continue;
    double s = 0.0;
    for (int sp = 0; sp < splits; ++sp) s += part[(size_t(sp) * tiles + tile) * kTile * kTile + e];
    out[size_t(i) * d + j] = s;
    out[size_t(j) * d + i] = s;
  }
  for (int64_t f = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; f < d;
       f += int64_t(gridDim.x) * blockDim.x) {
    double s = 0.0;
    for (int sp = 0; sp < splits; ++sp)
      s += cpart[(size_t(sp) * nb + f / kTile) * kTile + f % kTile];
    colsum[f] = s;
  }
}

}  // namespace

PcaPlan pca_syrk_plan(int64_t n, int d, int num_cus) {
  PcaPlan p;
  // 256-wide tiles (one 512-thread workgroup per CU) once there are at least two 128-wide column
  // blocks; 128-wide tiles (two 256-thread workgroups per CU) for d <= 128
  p.tw = d > kTile ? kTile2 : kTile;
  p.nb = (d + p.tw - 1) / p.tw;
  p.tiles = p.nb * (p.nb + 1) / 2;
  const int per_cu = p.tw == kTile2 ? 3 : 6;  // resident workgroups per CU x ~3 waves of them
  const int64_t want = int64_t(std::max(num_cus, 64)) * per_cu;
  int64_t s = (want + p.tiles - 1) / p.tiles;
  const int64_t max_s = std::max<int64_t>(1, (n + 4 * kChunk - 1) / (4 * kChunk));
  s = std::max<int64_t>(1, std::min(s, max_s));
  // bound the fp64 slab (splits x tiles x tw^2 doubles) to 1 GiB unless one split exceeds it
  const int64_t slab_tile = int64_t(p.tw) * p.tw * 8;
  while (s > 1 && s * p.tiles * slab_tile > (int64_t(1) << 30)) --s;
  p.splits = static_cast<int>(s);
  p.rows_per_split = round_up((n + s - 1) / s, kChunk);  // a multiple of both chunk sizes
  if (p.rows_per_split == 0) p.rows_per_split = kChunk;
  p.part_elems = size_t(p.splits) * p.tiles * p.tw * p.tw;
  p.cpart_elems = size_t(p.splits) * p.nb * p.tw;
  p.shift_elems = size_t(p.nb) * p.tw;
  const int64_t g = int64_t(p.splits) * p.tiles;
  p.grid = static_cast<int>(round_up(g, 8));
  return p;
}

void pca_syrk(const float* x, int64_t n, int64_t ld, int d, const float* shift, const PcaPlan& p,
              double* part, double* cpart, bool four, int flush_rows, hipStream_t s) {
  OAP_CHECK(ld % 4 == 0 && ld >= d, "pca_syrk: ld must be a multiple of 4 and >= d");
  OAP_CHECK(reinterpret_cast<uintptr_t>(x) % 16 == 0, "pca_syrk: rows must be 16-byte aligned");
  SyrkArgs a;
  a.x = x;
  a.n = n;
  a.ld = ld;
  a.d = d;
  a.shift = shift;
  a.nb = p.nb;
  a.tiles = p.tiles;
  a.splits = p.splits;
  a.flush_chunks = std::max(1, flush_rows / kChunk);
  a.rows_per_split = p.rows_per_split;
  a.part = part;
  a.cpart = cpart;
  if (p.tw == kTile2) {
    if (four)
      hipLaunchKernelGGL(oap_pca_syrk_w256<true>, dim3(p.grid), dim3(kSyrk2Threads), 0, s, a);
    else
      hipLaunchKernelGGL(oap_pca_syrk_w256<false>, dim3(p.grid), dim3(kSyrk2Threads), 0, s, a);
  } else if (four) {
    hipLaunchKernelGGL(oap_pca_syrk<true>, dim3(p.grid), dim3(kSyrkThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL(oap_pca_syrk<false>, dim3(p.grid), dim3(kSyrkThreads), 0, s, a);
  }
  OAP_HIP_CHECK(hipGetLastError());
}

PcaPlan pca_syrk_plan_f64(int64_t n, int d, int num_cus) {
  PcaPlan p;
  p.tw = kXTile;
  p.nb = (d + p.tw - 1) / p.tw;
  p.tiles = p.nb * (p.nb + 1) / 2;
  // one 512-thread workgroup per CU: pick the split count whose (splits x tiles) workgroups
  // fill whole rounds of the CUs (t = 36 tiles at d = 1000 -> 64 splits = 9 full rounds of 256),
  // at least two rounds when the rows allow it
  const int64_t R = std::max(num_cus, 64);
  const int64_t max_s = std::max<int64_t>(1, (n + 8 * kXRows - 1) / (8 * kXRows));
  const int64_t s_lo = std::max<int64_t>(1, (2 * R + p.tiles - 1) / p.tiles);
  int64_t s = s_lo;
  double best = 1e30;
  for (int64_t c = s_lo; c <= 4 * s_lo; ++c) {
    const int64_t g = c * p.tiles;
    const double waste = double((g + R - 1) / R * R) / double(g);
    if (waste < best - 1e-9) {
      best = waste;
      s = c;
    }
  }
  s = std::max<int64_t>(1, std::min(s, max_s));
  const int64_t slab_tile = int64_t(p.tw) * p.tw * 8;
  while (s > 1 && s * p.tiles * slab_tile > (int64_t(1) << 30)) --s;
  p.splits = static_cast<int>(s);
  p.rows_per_split = round_up((n + s - 1) / s, kXRows);
  if (p.rows_per_split == 0) p.rows_per_split = kXRows;
  p.part_elems = size_t(p.splits) * p.tiles * p.tw * p.tw;
  p.cpart_elems = size_t(p.splits) * p.nb * p.tw;
  p.shift_elems = size_t(p.nb) * p.tw;
  p.grid = static_cast<int>(round_up(int64_t(p.splits) * p.tiles, 8));
  return p;
}

void pca_syrk_f64(const void* x, bool x_f64, int64_t n, int64_t ld, int d, const double* shift,
                  const PcaPlan& p, double* part, double* cpart, hipStream_t s) {
  OAP_CHECK(p.tw == kXTile, "pca_syrk_f64 needs a pca_syrk_plan_f64 plan");
  OAP_CHECK(ld >= d && ld < INT32_MAX, "pca_syrk_f64: bad ld");
  SyrkF64Args a;
  a.x = x;
  a.n = n;
  a.ld = ld;
  a.d = d;
  a.shift = shift;
  a.nb = p.nb;
  a.tiles = p.tiles;
  a.splits = p.splits;
  a.rows_per_split = p.rows_per_split;
  const size_t es = x_f64 ? 8 : 4;
  const bool vec = (reinterpret_cast<uintptr_t>(x) % 16 == 0) && ld % 4 == 0 &&
                   (size_t(ld) * es) % 16 == 0;
  a.part = part;
  a.cpart = cpart;
  const dim3 g(p.grid), b(kXThreads);
  if (x_f64 && vec)
    hipLaunchKernelGGL((oap_pca_syrk_f64<double, true>), g, b, 0, s, a);
  else if (x_f64)
    hipLaunchKernelGGL((oap_pca_syrk_f64<double, false>), g, b, 0, s, a);
  else if (vec)
    hipLaunchKernelGGL((oap_pca_syrk_f64<float, true>), g, b, 0, s, a);
  else
    hipLaunchKernelGGL((oap_pca_syrk_f64<float, false>), g, b, 0, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

void pca_cov(const double* stats, int d, int64_t n, double* cov, hipStream_t s) {
  const int64_t total = int64_t(d) * d;
  const int grid = static_cast<int>(std::min<int64_t>((total + 255) / 256, 4096));
  hipLaunchKernelGGL(oap_pca_cov, dim3(grid), dim3(256), 0, s, stats, d, double(n), cov);
  OAP_HIP_CHECK(hipGetLastError());
}

void pca_reduce(const PcaPlan& p, const double* part, const double* cpart, int d, double* out,
                double* colsum, hipStream_t s) {
  const int64_t total = int64_t(p.tiles) * p.tw * p.tw;
  hipLaunchKernelGGL(oap_pca_reduce, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s, part,
                     cpart, p.splits, p.tiles, p.nb, d, p.tw, out, colsum);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
