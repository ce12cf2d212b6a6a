// PCA exact-mode statistics on the int8 matrix cores (integer-sliced, Ozaki-style SYRK).
//
// The reference forms every product (x_i - s_i)(x_j - s_j) and its sum in fp64 (oneDAL
// step1Local, mllib-dal/src/main/native/PCADALImpl.cpp:31,63-69).  The fp64 MFMA path
// (pca.hip, oap_pca_syrk_f64) does the same at ~78 TFLOP/s peak.  Here the centred rows are
// written as 7 signed base-128 digits per element, relative to a per-column power of two, and the
// products of digits run on v_mfma_i32_32x32x32_i8 (int8 in, int32 accumulate: exact), 64x the
// fp64 MFMA rate per instruction; 28 digit products (p + q <= 6) replace one fp64 product.
//
//   v = x - s (fp64),  M_j = max_i |v_ij| < 2^E_j,
//   v = 2^(E-6) (t_0 + t_1 2^-7 + ... + t_6 2^-42 + rho),   t_p in [-64, 64],  |rho| <= 2^-43
//   S_jk = sum_i v_ij v_ik ~= 2^(E_j + E_k - 12) sum_{L=0..6} 2^(-7L) sum_{p+q=L} sum_i t_p t_q
//
// Error per row (the bound pca.cpp reports, docs/ARCHITECTURE.md "PCA exact"):
//   |v_j v_k - approx| <= 2^(E_j+E_k-49) (2 [representation] + 6.04 [dropped p+q >= 7])
// i.e. <= 8.05 * 2^-49 * 4 M_j M_k, plus the fp64 rounding of v and of the slab sums that the fp64
// path has too.  The level sums are exact integers: |t_p t_q| <= 2^12, at most 7 products per
// level and row, so 2048 row blocks (65536 rows) stay below 2^31 before an fp64 flush.
//
// Kernels (one fit = one minmax pass over all rows, then per row chunk: slice + SYRK):
//   oap_oz_minmax   column min / max of x per row group (fp32, exact), over every row or an
//                   even sample of 65536 rows (then one bit of margin, and the digitising pass
//                   flags any digit past [-64, 64]: the caller redoes the pass with exact scales)
//   oap_oz_exponent E_j and the scale 2^(6 - E_j) from max(xmax - s, s - xmin) (fp64)
//   oap_oz_slice    the 7 digit planes [p][row block][feature][32 rows] int8 + fp64 column sums
//   oap_oz_syrk     128 x 64 output tile per 4-wave workgroup (each wave 32 x 64: 7 levels x 2
//                   blocks of 32 x 32 int32 accumulators = 224 registers); the digit fragments of
//                   a 32-row block (each a contiguous 1 KB of a plane) stage through LDS by
//                   global_load_lds, three blocks deep, the B fragments shared by the 4 waves
//   oap_oz_reduce   sum of the split slabs (fixed order), times 2^(E_i + E_j - 12), both halves
#include <algorithm>
#include <cmath>

#include "kernels/device_utils.h"
#include "kernels/kernels.h"
#include "runtime/common.h"

namespace oap {
namespace kern {

namespace {

constexpr int kOzDigits = 7;
constexpr int kOzRB = 32;          // rows per row block (the MFMA's k)
constexpr int kOzTile = 64;        // output tile (64 x 64 per workgroup)
constexpr int kOzThreads = 256;
constexpr int kOzFlush = 2048;     // row blocks per int32 flush (7 * 2^12 * 32 * 2048 < 2^31)
constexpr int kOzRowGroup = 2048;  // rows per minmax partial
constexpr int kOzSample = 65536;   // rows of the sampled column ranges
constexpr int kOzSliceRB = 16;     // row blocks per slice-kernel block (one column-sum partial)
constexpr int kOzFeat = 256;       // features per minmax block
constexpr int kOzSliceFeat = 128;  // features per slice block (two threads each)

constexpr int kOzStage = 4 * kOzDigits * 1024;  // 28 KB: A 2 x 7, B 2 x 7 fragments

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// rows idx * rstride for idx in [g * per, (g + 1) * per) of the n_s sampled rows (rstride 1: all)
__global__ __launch_bounds__(kOzFeat) void oap_oz_minmax(const float* __restrict__ x, int64_t n_s,
                                                          int64_t rstride, int per, int64_t ld,
                                                          int d, int dp,
                                                          float2* __restrict__ mm) {
  const int f = blockIdx.y * kOzFeat + threadIdx.x;
  const int64_t r0 = int64_t(blockIdx.x) * per;
  const int64_t r1 = min(n_s, r0 + per);
  float lo = INFINITY, hi = -INFINITY;
  if (f < d) {
    const float* p = x + f;
    const int64_t st = rstride * ld;
    int64_t r = r0;
    for (; r + 8 <= r1; r += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(r + u) * st];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        lo = fminf(lo, v[u]);
        hi = fmaxf(hi, v[u]);
      }
    }
    for (; r < r1; ++r) {
      const float v = p[r * st];
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
  }
  if (f < dp) mm[size_t(blockIdx.x) * dp + f] = make_float2(lo, hi);
}

__global__ __launch_bounds__(256) void oap_oz_exponent(const float2* __restrict__ mm, int groups,
                                                        int d, int dp, int margin,
                                                        const double* __restrict__ shift,
                                                        int* __restrict__ E,
                                                        double* __restrict__ sc) {
  __shared__ float slo[256], shi[256];
  const int f = blockIdx.x;
  float lo = INFINITY, hi = -INFINITY;
  if (f < d)
    for (int g = threadIdx.x; g < groups; g += 256) {
      const float2 v = mm[size_t(g) * dp + f];
      lo = fminf(lo, v.x);
      hi = fmaxf(hi, v.y);
    }
  slo[threadIdx.x] = lo;
  shi[threadIdx.x] = hi;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      slo[threadIdx.x] = fminf(slo[threadIdx.x], slo[threadIdx.x + w]);
      shi[threadIdx.x] = fmaxf(shi[threadIdx.x], shi[threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int e = 0;
    if (f < d && groups > 0) {
      // the slice kernel's v = (double)x - s is monotone in x: its extreme values are these
      const double s = shift[f];
      const double m = fmax(double(shi[0]) - s, s - double(slo[0]));
      if (m > 0.0 && m <= 1.7e308) e = min(max(ilogb(m) + 1 + margin, -900), 1000);  // m < 2^e
    }
    E[f] = e;
    sc[f] = ldexp(1.0, 6 - e);
  }
}

// digits of 16 rows of one feature per thread, two threads (adjacent lanes) per feature: lane l
// covers feature f0 + l / 2, rows 16 (l & 1) .. + 15 of each row block, so one wave's store of a
// digit plane is a contiguous 1 KB (32 features x 32 bytes)
__global__ __launch_bounds__(256) void oap_oz_slice(
    const float* __restrict__ x, int64_t n, int64_t ld, int d, int dp, int64_t row0,
    int64_t nrb, const double* __restrict__ shift, const double* __restrict__ sc,
    int8_t* __restrict__ planes, double* __restrict__ cpart, int64_t group0,
    int* __restrict__ ovf) {
  const int f = blockIdx.y * kOzSliceFeat + (threadIdx.x >> 1);
  const int half = threadIdx.x & 1;
  const int64_t rb0 = int64_t(blockIdx.x) * kOzSliceRB;
  const int64_t rb1 = min(nrb, rb0 + kOzSliceRB);
  const bool okf = f < d;
  const double s = okf ? shift[f] : 0.0, scale = okf ? sc[f] : 0.0;
  const size_t plane = size_t(nrb) * dp * kOzRB;
  double csum = 0.0;
  bool over = false;  // a digit past [-64, 64]: the sampled scales were too small
  // rows of block rb + 1 in flight while block rb is digitised (unconditional loads: rows
  // clamped to n - 1, features to 0; masked below)
  const int fl = okf ? f : 0;
  auto load = [&](int64_t rb, float (&v)[16]) {
    const int64_t r = row0 + min(rb, rb1 - 1) * kOzRB + 16 * half;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = x[min(r + i, n - 1) * ld + fl];
  };
  auto digitise = [&](int64_t rb, const float (&xv)[16]) {
    const int64_t r = row0 + rb * kOzRB + 16 * half;
    unsigned pk[kOzDigits][4];
#pragma unroll
    for (int p = 0; p < kOzDigits; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) pk[p][q] = 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const bool ok = okf && r + i < n;
      const double v = ok ? double(xv[i]) - s : 0.0;
      csum += v;
      double w = v * scale;  // exact (power of two), |w| < 64 (checked)
      over |= !(fabs(w) < 64.0);
      double t = __builtin_rint(w);
      pk[0][i >> 2] |= (unsigned(int(t)) & 0xffu) << (8 * (i & 3));
      w -= t;  // exact: |w| <= 1/2
#pragma unroll
      for (int p = 1; p < kOzDigits; ++p) {
        w *= 128.0;
        t = __builtin_rint(w);
        pk[p][i >> 2] |= (unsigned(int(t)) & 0xffu) << (8 * (i & 3));
        w -= t;
      }
    }
#pragma unroll
    for (int p = 0; p < kOzDigits; ++p)
      *reinterpret_cast<v4i*>(planes + p * plane + (size_t(rb) * dp + f) * kOzRB + 16 * half) =
          v4i{int(pk[p][0]), int(pk[p][1]), int(pk[p][2]), int(pk[p][3])};
  };
  float xa[16], xb[16];
  load(rb0, xa);
  for (int64_t rb = rb0; rb < rb1; rb += 2) {
    load(rb + 1, xb);
    digitise(rb, xa);
    if (rb + 1 >= rb1) break;
    load(rb + 2, xa);
    digitise(rb + 1, xb);
  }
  if (over) atomicOr(ovf, 1);
  csum += __shfl_xor(csum, 1, 64);  // (the two halves of the feature, fixed order)
  if (half == 0) cpart[size_t(group0 + blockIdx.x) * dp + f] = csum;
}

struct OzArgs {
  const int8_t* planes;  // [7][nrb][dp][32]
  int64_t nrb;
  int dp, nb, tiles;
  int64_t rb_per_split;
  double* slab;  // [splits][tiles][64][64], accumulated (+=)
};

// upper-triangular 64 x 64 tile t of nb blocks -> (bi, bj), bj >= bi
__device__ inline void oz_tile(int tile, int nb, int& bi, int& bj) {
  int t = tile, b = 0;
  while (t >= nb - b) {
    t -= nb - b;
    ++b;
  }
  bi = b;
  bj = b + t;
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* glb_ptr_t;

// 64 x 64 output tile per 4-wave workgroup, each wave one 32 x 32 block (wave (wi, wj)) with its
// 7 level accumulators (112 AGPRs): ~200 registers, so two workgroups share a CU (two waves per
// SIMD) and one's LDS reads and barrier waits hide under the other's MFMAs.
__global__ __launch_bounds__(kOzThreads, 2) void oap_oz_syrk(OzArgs a) {
  __shared__ __attribute__((aligned(1024))) int oz_lds[2 * kOzStage / 4];  // the only LDS object
  const int G = gridDim.x;
  const int per = G / 8;  // XCD-aware: the tiles of one split share an XCD (its L2)
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const int split = L / a.tiles, tile = L - split * a.tiles;
  const int64_t rb0 = int64_t(split) * a.rb_per_split;
  const int64_t rb1 = min(a.nrb, rb0 + a.rb_per_split);
  if (rb0 >= rb1) return;
  int bi, bj;
  oz_tile(tile, a.nb, bi, bj);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  const size_t plane = size_t(a.nrb) * a.dp * kOzRB;
  const size_t rbs = size_t(a.dp) * kOzRB;

  v16i acc[kOzDigits];
#pragma unroll
  for (int l = 0; l < kOzDigits; ++l)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[l][e] = 0;

  double* slab = a.slab + (size_t(split) * a.tiles + tile) * (kOzTile * kOzTile);
  auto flush = [&]() {
    // laundered per-lane base: keeps the 16 element addresses from being hoisted out of the row
    // loop as live registers; 4 read-modify-writes in flight at a time
    double* base = slab + (32 * wi + 4 * (lane >> 5)) * kOzTile + 32 * wj + (lane & 31);
    asm volatile("" : "+v"(base));
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      double v = double(acc[kOzDigits - 1][e]);
#pragma unroll
      for (int l = kOzDigits - 2; l >= 0; --l) v = fma(v, 0x1p-7, double(acc[l][e]));
      double* q = base + ((e & 3) + 8 * (e >> 2)) * kOzTile;
      *q += v;
      if ((e & 3) == 3) asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int l = 0; l < kOzDigits; ++l)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[l][e] = 0;
  };

  // Digit fragments stage through LDS by global_load_lds, two row blocks deep (block rb + 1 is
  // in flight while rb feeds the MFMAs).  A stage holds the tile's two A blocks (slots 7 i + p)
  // and two B blocks (slots 14 + 7 j + p), 1 KB each; wave w loads the 7 slots 7 w .. 7 w + 6
  // (exactly 7 per wave and stage).  Lane l fetches byte g(l) = (l & 31) * 32 + 16 (l >> 5)
  // of a fragment into LDS byte 16 l, so the MFMA lane l reads its operand at 16 l.  Only raw
  // s_barriers in the loop (a __syncthreads would also drain the in-flight stage).
  char* st0 = reinterpret_cast<char*>(oz_lds);
  const size_t gl = size_t(lane & 31) * kOzRB + 16 * (lane >> 5);
  const int blk = wave < 2 ? bi : bj;  // the 64-feature block wave w's slots come from
  const int8_t* pw = a.planes + (size_t(blk) * kOzTile + 32 * (wave & 1)) * kOzRB;
  auto issue = [&](int64_t rb, int stg) {
    const size_t o = size_t(min(rb, rb1 - 1)) * rbs + gl;
    char* sb = st0 + stg * kOzStage + wave * kOzDigits * 1024;
#pragma unroll
    for (int p = 0; p < kOzDigits; ++p)
      __builtin_amdgcn_global_load_lds((glb_ptr_t)(pw + p * plane + o),
                                       (lds_ptr_t)(sb + p * 1024), 16, 0, 0);
  };
  auto compute = [&](int stg) {
    const char* sb = st0 + stg * kOzStage + 16 * lane;
    v4i A[kOzDigits], B[kOzDigits];
#pragma unroll
    for (int p = 0; p < kOzDigits; ++p) {
      A[p] = *reinterpret_cast<const v4i*>(sb + (wi * kOzDigits + p) * 1024);
      B[p] = *reinterpret_cast<const v4i*>(sb + ((2 + wj) * kOzDigits + p) * 1024);
    }
#pragma unroll
    for (int l = 0; l < kOzDigits; ++l)
#pragma unroll
      for (int p = 0; p <= l; ++p)
        acc[l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[p], B[l - p], acc[l], 0, 0, 0);
  };
  issue(rb0, 0);
  int stg = 0, since = 0;
  for (int64_t rb = rb0; rb < rb1; ++rb) {
    // this wave's loads of block rb have landed, then everyone's; the barrier also frees the
    // stage block rb - 1 was read from (every wave's reads of it retired before its MFMAs)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_s_barrier();
    issue(rb + 1, stg ^ 1);
    compute(stg);
    stg ^= 1;
    if (++since == kOzFlush) {
      flush();
      since = 0;
    }
  }
  if (since > 0) flush();
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): nothing in flight at exit
}

__global__ __launch_bounds__(256) void oap_oz_reduce(const double* __restrict__ slab, int splits,
                                                      int group, int tiles, int nb, int d,
                                                      const int* __restrict__ E,
                                                      double* __restrict__ out) {
  const int64_t total = int64_t(d) * d;
  for (int64_t idx = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int i = static_cast<int>(idx / d), j = static_cast<int>(idx - int64_t(i) * d);
    if (i > j) continue;
    const int bi = i / kOzTile, bj = j / kOzTile;
    const int tile = bi * nb - bi * (bi - 1) / 2 + (bj - bi);
    const size_t e = size_t(i - bi * kOzTile) * kOzTile + (j - bj * kOzTile);
    // two-level sum over the splits (groups of ceil(sqrt(splits)), fixed order): an fp64
    // rounding chain of ~2 sqrt(splits) additions instead of splits
    const double* sl = slab + size_t(tile) * (kOzTile * kOzTile) + e;
    const size_t sstride = size_t(tiles) * (kOzTile * kOzTile);
    double s = 0.0;
    for (int g0 = 0; g0 < splits; g0 += group) {
      double gs = 0.0;
      for (int sp = g0; sp < min(splits, g0 + group); ++sp) gs += sl[sp * sstride];
      s += gs;
    }
    const double v = ldexp(s, E[i] + E[j] - 12);
    out[size_t(i) * d + j] = v;
    out[size_t(j) * d + i] = v;
  }
}

__global__ __launch_bounds__(256) void oap_oz_colsum(const double* __restrict__ cpart,
                                                      int64_t groups, int dp,
                                                      double* __restrict__ colsum) {
  __shared__ double sh[256];
  const int f = blockIdx.x;
  double s = 0.0;
  for (int64_t g = threadIdx.x; g < groups; g += 256) s += cpart[size_t(g) * dp + f];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) colsum[f] = sh[0];
}

// *bound = rows * 2^(2 max_j E_j) * coef: the per-entry bound on |S - S_exact| (pca.cpp)
__global__ __launch_bounds__(256) void oap_oz_bound(const int* __restrict__ E, int d, double rows,
                                                     double coef, const int* __restrict__ ovf,
                                                     double* __restrict__ bound) {
  __shared__ int sh[256];
  int m = INT_MIN;
  for (int f = threadIdx.x; f < d; f += 256) m = max(m, E[f]);
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) sh[threadIdx.x] = max(sh[threadIdx.x], sh[threadIdx.x + w]);
    __syncthreads();
  }
  // an overflowed digit (sampled scales too small) poisons the bound: the caller redoes the pass
  // with exact scales (-1e300 keeps the allreduced sum negative)
  if (threadIdx.x == 0)
    bound[0] = ovf[0] ? -1e300 : rows > 0 ? ldexp(rows * coef, 2 * sh[0]) : 0.0;
}

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

}  // namespace

PcaOzakiPlan pca_ozaki_plan(int64_t n, int d, int num_cus, size_t max_plane_bytes) {
  PcaOzakiPlan p;
  p.n = n;
  p.d = d;
  p.dp = int(round_up(size_t(std::max(d, 1)), kOzSliceFeat));
  p.nb = p.dp / kOzTile;
  p.tiles = p.nb * (p.nb + 1) / 2;
  p.nrb = (n + kOzRB - 1) / kOzRB;
  p.groups = (n + kOzRowGroup - 1) / kOzRowGroup;
  // row blocks per chunk: the digit planes of one chunk within max_plane_bytes, whole slice
  // groups (so the column-sum partials of all chunks tile one array)
  const size_t per_rb = size_t(kOzDigits) * p.dp * kOzRB;
  int64_t crb = int64_t(std::max<size_t>(1, max_plane_bytes / per_rb));
  crb = std::max<int64_t>(kOzSliceRB, crb / kOzSliceRB * kOzSliceRB);
  p.chunk_rb = std::min<int64_t>(round_up(size_t(std::max<int64_t>(p.nrb, 1)), kOzSliceRB), crb);
  p.chunks = std::max<int64_t>(1, (p.nrb + p.chunk_rb - 1) / p.chunk_rb);
  p.cgroups = (p.nrb + kOzSliceRB - 1) / kOzSliceRB;
  // two 256-thread workgroups per CU (~200 registers per lane, 56 KB of LDS each): splits x
  // tiles in whole rounds of the resident slots, at least two rounds when the rows allow
  const int64_t R = 2 * int64_t(std::max(num_cus, 64));
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
  s = std::max<int64_t>(1, std::min<int64_t>(s, std::max<int64_t>(1, p.chunk_rb / 8)));
  p.splits = int(s);
  // longest chain of fp64 additions into one output: the slab flushes of a split over all
  // chunks, the sum over splits, the final scaling
  const int64_t rps = (p.chunk_rb + s - 1) / s;
  p.split_group = std::max(1, int(std::ceil(std::sqrt(double(s)))));
  p.fp64_adds = int(p.chunks * ((rps + kOzFlush - 1) / kOzFlush) + p.split_group +
                    (s + p.split_group - 1) / p.split_group + 2);
  p.slab_elems = size_t(p.splits) * p.tiles * kOzTile * kOzTile;
  // workspace: planes | slab | minmax partials | E | scale | shift | column-sum partials
  p.off_slab = align256(size_t(p.chunk_rb) * per_rb);
  p.off_mm = p.off_slab + align256(p.slab_elems * sizeof(double));
  // minmax partials: every row's groups or the sample's (kOzSample / 256), whichever is more
  const int64_t mm_groups = std::max<int64_t>({p.groups, int64_t(kOzSample / 256), 1});
  p.off_e = p.off_mm + align256(size_t(mm_groups) * p.dp * sizeof(float2));
  p.off_sc = p.off_e + align256(size_t(p.dp + 1) * sizeof(int));  // E | overflow flag
  p.off_shift = p.off_sc + align256(size_t(p.dp) * sizeof(double));
  p.off_cpart = p.off_shift + align256(size_t(p.dp) * sizeof(double));
  p.ws_bytes =
      p.off_cpart + align256(size_t(std::max<int64_t>(p.cgroups, 1)) * p.dp * sizeof(double));
  return p;
}

void pca_syrk_ozaki(const float* x, int64_t ld, const double* shift_host, const PcaOzakiPlan& p,
                    void* ws, double* out, double* colsum, double* bound, bool exact_scales,
                    hipStream_t s) {
  OAP_CHECK(ld >= p.d, "pca_syrk_ozaki: bad ld");
  char* w = static_cast<char*>(ws);
  int8_t* planes = reinterpret_cast<int8_t*>(w);
  double* slab = reinterpret_cast<double*>(w + p.off_slab);
  float2* mm = reinterpret_cast<float2*>(w + p.off_mm);
  int* E = reinterpret_cast<int*>(w + p.off_e);
  double* sc = reinterpret_cast<double*>(w + p.off_sc);
  double* shift = reinterpret_cast<double*>(w + p.off_shift);
  double* cpart = reinterpret_cast<double*>(w + p.off_cpart);
  OAP_HIP_CHECK(hipMemcpyAsync(shift, shift_host, size_t(p.d) * sizeof(double),
                               hipMemcpyHostToDevice, s));
  OAP_HIP_CHECK(hipMemsetAsync(slab, 0, p.slab_elems * sizeof(double), s));
  int* ovf = E + p.dp;
  OAP_HIP_CHECK(hipMemsetAsync(ovf, 0, sizeof(int), s));
  const int fblocks = p.dp / kOzFeat + (p.dp % kOzFeat ? 1 : 0);
  // column exponents: from every row (exact_scales, or few rows), else from an even sample of
  // kOzSample rows with one bit of margin — a digit past [-64, 64] then flags the pass (the
  // caller redoes it with exact scales); the margin costs one bit of the bound
  const bool sampled = !exact_scales && p.n > int64_t(kOzSample);
  const int64_t n_s = sampled ? kOzSample : p.n;
  const int64_t rstride = sampled ? p.n / kOzSample : 1;
  const int per = sampled ? 256 : kOzRowGroup;
  const int64_t groups = (n_s + per - 1) / per;  // (the plan sizes the partials for both)
  if (groups > 0)
    hipLaunchKernelGGL(oap_oz_minmax, dim3(unsigned(groups), fblocks), dim3(kOzFeat), 0, s, x,
                       n_s, rstride, per, ld, p.d, p.dp, mm);
  hipLaunchKernelGGL(oap_oz_exponent, dim3(p.dp), dim3(256), 0, s, mm, int(groups), p.d, p.dp,
                     sampled ? 1 : 0, shift, E, sc);
  OAP_HIP_CHECK(hipGetLastError());
  const int64_t G = round_up(size_t(p.splits) * p.tiles, 8);
  for (int64_t c = 0; c < p.chunks; ++c) {
    const int64_t rb0 = c * p.chunk_rb;
    const int64_t nrb = std::min<int64_t>(p.chunk_rb, p.nrb - rb0);
    if (nrb <= 0) break;
    const int64_t sg = (nrb + kOzSliceRB - 1) / kOzSliceRB;
    hipLaunchKernelGGL(oap_oz_slice, dim3(unsigned(sg), p.dp / kOzSliceFeat), dim3(256), 0, s, x,
                       p.n, ld, p.d, p.dp, rb0 * kOzRB, nrb, shift, sc, planes, cpart,
                       rb0 / kOzSliceRB, ovf);
    OzArgs a;
    a.planes = planes;
    a.nrb = nrb;
    a.dp = p.dp;
    a.nb = p.nb;
    a.tiles = p.tiles;
    a.rb_per_split = (nrb + p.splits - 1) / p.splits;
    a.slab = slab;
    hipLaunchKernelGGL(oap_oz_syrk, dim3(unsigned(G)), dim3(kOzThreads), 0, s, a);
    OAP_HIP_CHECK(hipGetLastError());
  }
  const int64_t total = int64_t(p.d) * p.d;
  hipLaunchKernelGGL(oap_oz_reduce, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s, slab,
                     p.splits, p.split_group, p.tiles, p.nb, p.d, E, out);
  hipLaunchKernelGGL(oap_oz_colsum, dim3(p.d), dim3(256), 0, s, cpart, p.cgroups, p.dp, colsum);
  // per row: 2^(E_j+E_k-49) (2 representation + 6.04 dropped digit products + 2^-4 rounding of
  // v) + 2^(E_j+E_k-53) per fp64 addition of the longest chain
  const double coef = 0x1p-49 * (8.04 + 0.0625) + 0x1p-53 * p.fp64_adds;
  hipLaunchKernelGGL(oap_oz_bound, dim3(1), dim3(256), 0, s, E, p.d, double(p.n), coef, ovf,
                     bound);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
