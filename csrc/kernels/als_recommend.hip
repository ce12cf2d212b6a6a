// oap_rec_topk — fused score + top-k for ALSModel.recommendForAll* / *Subset (gfx950, CDNA4).
//
// Spark scores blocks of users x items with a GEMM and keeps a bounded priority queue per user
// (spark-3.1.1/mllib/src/main/scala/org/apache/spark/ml/recommendation/ALS.scala:365-505); the
// previous implementation here materialised 4096 x n_items score blocks through rocBLAS and
// torch.topk.  This kernel never stores a score:
// * every workgroup (8 waves, 2 per SIMD) holds 32 UG source rows per wave in registers as the
//   MFMA B operand (split fp16: hi and lo planes, KS k-steps of 16 features each);
// * destination rows stream through two 32 KiB LDS buffers (64 rows up to rank 128, 32 above)
//   filled by global_load_lds (1 KiB lane-linear pieces, XOR-swizzled on the source address so
//   the A-fragment reads are conflict-free), one block ahead of the MFMAs, one barrier a block;
// * a 32 x 32 score tile is hi.hi + hi.lo + lo.hi on v_mfma_f32_32x32x16_f16 (fp32
//   accumulation; ~2^-21 relative to sum |s_k d_k|, an fp32-class score; every source row at
//   its own power-of-two scale, the destinations at one);
// * each lane owns one source row and 16 of the tile's destinations; its sorted top-num list
//   lives in LDS and only the list's minimum in a register: a tile costs 16 compares unless
//   some lane's score beats its minimum (after the first blocks rare), then the lanes pop
//   their largest candidate and insert it, round by round;
// * at the end the two half-wave lists of a row merge (ties: lower index first).
// Work per launch: all destinations x (grid * 256 UG) source rows; all resident workgroups read
// the destination blocks in the same order, so the stream is shared through L2 / MALL.
#include "kernels/als_recommend.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "runtime/common.h"

namespace oap {
namespace kern {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* glb_ptr_t;

constexpr int kRecWaves = 8;    // waves per workgroup (2 per SIMD)
constexpr size_t kRecLds = 160 * 1024;

__host__ __device__ constexpr int slots_of(int ks) { return ks <= 8 ? 32 : 64; }

// 2^e scale of a matrix whose max |x| has these float bits: max |x| 2^e in [128, 256)
__device__ inline int scale_exp(unsigned amax_bits) {
  const float a = __uint_as_float(amax_bits);
  if (!(a > 0.f) || !(a < INFINITY)) return 0;
  int e;
  frexpf(a, &e);  // a = f 2^e, f in [0.5, 1)
  return 8 - e;
}

__global__ void oap_rec_absmax(const float* __restrict__ x, int64_t n, int rank, int64_t ld,
                               unsigned* amax) {
  // one wave per row (grid-stride), lanes over the columns
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t ws = (int64_t(gridDim.x) * blockDim.x) >> 6;
  float m = 0.f;
  for (int64_t row = w0; row < n; row += ws)
    for (int c = lane; c < rank; c += 64) m = fmaxf(m, fabsf(x[row * ld + c]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0 && m > 0.f) atomicMax(amax, __float_as_uint(m));
}

// per-row 2^e scales (source rows: each row's own max |x| in [128, 256)), one wave per row
__global__ void oap_rec_row_exp(const float* __restrict__ x, int64_t n, int rank, int64_t ld,
                                int32_t* __restrict__ row_exp) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t ws = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t row = w0; row < n; row += ws) {
    float m = 0.f;
    for (int c = lane; c < rank; c += 64) m = fmaxf(m, fabsf(x[row * ld + c]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) row_exp[row] = scale_exp(__float_as_uint(m));
  }
}

// amax: the matrix's scale (destinations), or row_exp: each row's (sources)
__global__ void oap_rec_pack(const float* __restrict__ x, int64_t n, int rank, int64_t ld,
                             const unsigned* __restrict__ amax,
                             const int32_t* __restrict__ row_exp, f16x8* __restrict__ img,
                             int64_t rows_pad, int ks) {
  const int rs = slots_of(ks);
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= rows_pad * rs) return;
  const int64_t row = t / rs;
  const int q = int(t - row * rs);
  f16x8 out = {};
  if (row < n && q < 4 * ks) {
    const float sc = ldexpf(1.f, row_exp ? row_exp[row] : scale_exp(amax[0]));
    const int plane = q / (2 * ks), rem = q - plane * 2 * ks;
    const int f0 = 16 * (rem >> 1) + 8 * (rem & 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = f0 + j < rank ? x[row * ld + f0 + j] * sc : 0.f;
      const _Float16 hi = static_cast<_Float16>(v);
      out[j] = plane == 0 ? hi : static_cast<_Float16>(v - static_cast<float>(hi));
    }
  }
  img[t] = out;
}

struct RecArgs {
  const f16x8* src;  // [rows][RS] slots
  const f16x8* dst;
  const int32_t* src_exp;  // per source row
  const unsigned* dst_amax;
  int32_t* out_idx;
  float* out_val;
  int64_t n_src, n_dst;
  int num;
};

// destination rows per LDS block (one 32 KiB buffer), and the lists' share of LDS
__host__ __device__ constexpr int blk_of(int ks) { return ks <= 8 ? 64 : 32; }
constexpr size_t kRecBufs = 2 * 32 * 1024;
__host__ __device__ constexpr size_t lists_bytes(int ug, int num) {
  return size_t(kRecWaves) * 64 * ug * num * 8;
}

template <int KS, int UG>
__global__ __launch_bounds__(kRecWaves * 64, 1) void oap_rec_topk(RecArgs a) {
  constexpr int RS = slots_of(KS), ROWB = RS * 16, BLK = blk_of(KS), BUFB = BLK * ROWB;
  constexpr int CH = BUFB / 1024 / kRecWaves;  // 1-KiB glds pieces per wave per block
  static_assert(2 * BUFB == kRecBufs, "two 32 KiB destination buffers");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int num = a.num;
  const int64_t ubase = (int64_t(blockIdx.x) * kRecWaves + wave) * (32 * UG);

  // ---- this wave's source rows: B operands (row r of group g; k half h)
  f16x8 uh[UG][KS], ul[UG][KS];
#pragma unroll
  for (int g = 0; g < UG; ++g) {
    const f16x8* up = a.src + (ubase + 32 * g + r) * RS;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uh[g][s] = up[2 * s + h];
      ul[g][s] = up[2 * KS + 2 * s + h];
    }
  }
  // ---- per lane and group: a sorted list of num (score, index) in LDS, its minimum in a
  // register (the filter every score meets first)
  float* lv_all = reinterpret_cast<float*>(smem + kRecBufs);
  int* li_all = reinterpret_cast<int*>(smem + kRecBufs + lists_bytes(UG, num) / 2);
  auto lst = [&](int g, int ln) { return ((wave * UG + g) * 64 + ln) * num; };
  float thr[UG];
#pragma unroll
  for (int g = 0; g < UG; ++g) {
    thr[g] = -INFINITY;
    for (int j = 0; j < num; ++j) {
      lv_all[lst(g, lane) + j] = -INFINITY;
      li_all[lst(g, lane) + j] = 0x7fffffff;
    }
  }

  // ---- destination blocks: lane-linear LDS pieces, logical slot q of row i at q ^ (i & 7)
  const int64_t nblk = (a.n_dst + BLK - 1) / BLK;
  auto stage = [&](int64_t blk, int buf) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = wave * CH + j;
      const int byte = c * 1024 + lane * 16;
      const int row = byte / ROWB, p = (byte % ROWB) / 16;
      const f16x8* src = a.dst + (blk * BLK + row) * RS + (p ^ (row & 7));
      __builtin_amdgcn_global_load_lds((glb_ptr_t)(src), (lds_ptr_t)(smem + buf * BUFB + c * 1024),
                                       16, 0, 0);
    }
  };
  auto frag = [&](int buf, int row, int q) -> f16x8 {
    return *reinterpret_cast<const f16x8*>(smem + buf * BUFB + row * ROWB +
                                           ((q ^ (row & 7)) << 4));
  };
  // the candidates of one 32 x 32 tile: pop the lane's largest remaining score while some
  // lane's beats its list minimum (a wave runs as many rounds as its busiest lane has
  // candidates: after the first blocks almost always none) and insert it into the LDS list
  // (strictly greater only, the lowest tile slot first among equal scores: destinations reach
  // a lane in increasing index, so ties keep the lower index first)
  auto update = [&](f32x16 acc, int ibase, int g) {
    float* L = lv_all + lst(g, lane);
    int* I = li_all + lst(g, lane);
    while (true) {
      float mx = -INFINITY;
      int me = 0;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const bool gt = acc[e] > mx;
        mx = gt ? acc[e] : mx;
        me = gt ? e : me;
      }
      const bool ins = mx > thr[g];
      if (!__ballot(ins)) break;  // (wave-uniform)
      if (ins) {
        int j = num - 1;
        while (j > 0) {
          const float pv = L[j - 1];
          if (!(mx > pv)) break;
          L[j] = pv;
          I[j] = I[j - 1];
          --j;
        }
        L[j] = mx;
        I[j] = ibase + 8 * (me >> 2) + (me & 3);
        thr[g] = L[num - 1];
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = e == me ? -INFINITY : acc[e];
    }
  };

  stage(0, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's pieces landed
  __syncthreads();
  for (int64_t blk = 0; blk < nblk; ++blk) {
    const int buf = int(blk & 1);
    if (blk + 1 < nblk) stage(blk + 1, buf ^ 1);  // (its buffer was released by the barrier)
#pragma unroll
    for (int sub = 0; sub < BLK / 32; ++sub) {
      const int row = sub * 32 + r;
      f32x16 acc[UG];
#pragma unroll
      for (int g = 0; g < UG; ++g) acc[g] = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const f16x8 ih = frag(buf, row, 2 * s + h);
        const f16x8 il = frag(buf, row, 2 * KS + 2 * s + h);
#pragma unroll
        for (int g = 0; g < UG; ++g) {
          acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ih, uh[g][s], acc[g], 0, 0, 0);
          acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ih, ul[g][s], acc[g], 0, 0, 0);
          acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(il, uh[g][s], acc[g], 0, 0, 0);
        }
      }
      const int ibase = int(blk * BLK) + sub * 32 + 4 * h;
      if (blk == nblk - 1) {  // (padded destinations never enter a list)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const bool pad = ibase + 8 * (e >> 2) + (e & 3) >= a.n_dst;
#pragma unroll
          for (int g = 0; g < UG; ++g) acc[g][e] = pad ? -INFINITY : acc[g][e];
        }
      }
#pragma unroll
      for (int g = 0; g < UG; ++g) update(acc[g], ibase, g);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // the next block's pieces (this wave's) landed
    __syncthreads();
  }

  // ---- merge the two half-wave lists of each row, write the top num
  const int dexp = scale_exp(a.dst_amax[0]);
#pragma unroll
  for (int g = 0; g < UG; ++g) {
    const int64_t u = ubase + 32 * g + r;
    if (h == 0 && u < a.n_src) {
      const float inv = ldexpf(1.f, -(a.src_exp[u] + dexp));
      const float* va = lv_all + lst(g, r);
      const float* vb = lv_all + lst(g, r + 32);
      const int* ia = li_all + lst(g, r);
      const int* ib = li_all + lst(g, r + 32);
      int pa = 0, pb = 0;
      for (int t = 0; t < num; ++t) {
        const float x = pa < num ? va[pa] : -INFINITY, y = pb < num ? vb[pb] : -INFINITY;
        const int xi = pa < num ? ia[pa] : 0x7fffffff, yi = pb < num ? ib[pb] : 0x7fffffff;
        const bool takea = x > y || (x == y && xi < yi);
        const float v = takea ? x : y;
        const int i = takea ? xi : yi;
        pa += takea ? 1 : 0;
        pb += takea ? 0 : 1;
        const bool real = v > -INFINITY;
        a.out_idx[u * num + t] = real ? i : -1;
        a.out_val[u * num + t] = real ? v * inv : -INFINITY;
      }
    }
  }
}

template <int KS, int UG>
void launch_topk(const RecArgs& a, hipStream_t s) {
  const size_t lds = kRecBufs + lists_bytes(UG, a.num);
  OAP_CHECK(lds <= kRecLds, "oap_rec_topk: LDS plan");
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_rec_topk<KS, UG>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(kRecLds)));
    attr = true;
  }
  const int64_t per = int64_t(kRecWaves) * 32 * UG;
  const int64_t grid = (a.n_src + per - 1) / per;
  OAP_CHECK(grid < (int64_t(1) << 31), "rec_topk: too many source rows for one launch");
  hipLaunchKernelGGL((oap_rec_topk<KS, UG>), dim3(unsigned(grid)), dim3(kRecWaves * 64), lds, s,
                     a);
  OAP_HIP_CHECK(hipGetLastError());
}

// two 32-row source groups per wave where the lists' LDS allows (num <= 12) and the source
// operands leave room (rank <= 160: no spills), else one
int ug_of(int ks, int num) { return ks <= 10 && kRecBufs + lists_bytes(2, num) <= kRecLds ? 2 : 1; }

template <int KS>
void launch_ks(const RecArgs& a, hipStream_t s) {
  if (ug_of(KS, a.num) == 2)
    launch_topk<KS, 2>(a, s);
  else
    launch_topk<KS, 1>(a, s);
}

// ---- num beyond the LDS lists: candidate buffers in HBM, wave-cooperative compaction --------
// Each lane (a source row's half of the destinations, as above) appends every score that can
// still reach its top-num (above its threshold) to its own HBM buffer of `cap` entries (cap = the
// power of two >= 2 num + 16).  When a lane's buffer could overflow with the next tile, the wave
// compacts it to exactly its num best under the key (score desc, index asc) — a total order, so
// nothing depends on arrival order — and the num-th score becomes the lane's threshold: later
// arrivals need a strictly larger score (an equal one has a larger index, so it ranks behind).
// Spark's bounded priority queue per source row (ALS.scala:451-505) for num up to 4088.
//  * num <= 1016 (cap <= 2048): 4 waves per workgroup; the compaction is a radix select with
//    the lane's entries in the wave's registers (32 per lane: bisection of the ordered score
//    bits by wave-summed counts, then of the index bits among ties), no sort and no LDS; at the
//    end each row's two half lists are sorted once (bitonic) in the freed destination buffers.
//  * num > 1016: one wave, the compaction a bitonic sort in a 64 KiB LDS buffer beside the
//    destination stream.
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr int kBigMaxCap = 8192;
constexpr int kSelQ = 32;  // entries per lane in a register compaction (cap <= 64 * kSelQ)
__host__ __device__ constexpr int big_waves(int cap) { return cap <= 64 * kSelQ ? 4 : 1; }

__host__ __device__ constexpr int big_cap(int num) {
  int c = 64;
  while (c < 2 * num + 16) c <<= 1;
  return c;
}

__device__ inline bool rec_before(int2 x, int2 y) {  // x ranks ahead of y
  const float a = __int_as_float(x.x), b = __int_as_float(y.x);
  return a > b || (a == b && x.y < y.y);
}
__device__ inline unsigned ord_key(int bits) {  // float bits -> unsigned of the same order
  return bits < 0 ? ~unsigned(bits) : unsigned(bits) | 0x80000000u;
}
__device__ inline int ord_bits(unsigned k) {
  return k & 0x80000000u ? int(k & 0x7fffffffu) : int(~k);
}
__device__ inline int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// wave-cooperative bitonic sort of p[0..sz) (sz a power of two >= 64) best-first
__device__ inline void wave_bitonic(int2* p, int sz, int lane) {
  for (int kk = 2; kk <= sz; kk <<= 1)
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < sz; i += 64) {
        const int q = i ^ j;
        if (q > i) {
          const int2 x = p[i], y = p[q];
          const bool fwd = (i & kk) == 0;  // this pair's run is sorted best-first
          if (fwd ? rec_before(y, x) : rec_before(x, y)) {
            p[i] = y;
            p[q] = x;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// lane buffer b[0..n) (n > num, n <= 64 kSelQ) -> exactly its num best (score desc, index asc)
// in b[0..num), unsorted; returns the num-th score.
__device__ __attribute__((always_inline)) inline float rec_select(int2* b, int n, int num,
                                                                  int lane) {
  // reads stay below n (<= cap, the lane buffer's length): entry lane + 64 q only for q < qn
  unsigned kh[kSelQ];  // ordered score bits; the indices stay in the buffer
  const int2* bl = b + lane;
  const int qn = (n + 63) >> 6;  // (wave-uniform)
#pragma unroll
  for (int q = 0; q < kSelQ; ++q) {
    const bool in = q < qn && lane + 64 * q < n;
    kh[q] = in ? ord_key(bl[64 * q].x) : 0u;  // (every real key is above 0x007fffff)
  }
  unsigned t = 0;  // the num-th largest key: max t with #{key >= t} >= num
  for (int bit = 31; bit >= 0; --bit) {
    const unsigned c = t | (1u << bit);
    int m = 0;
#pragma unroll
    for (int q = 0; q < kSelQ; ++q) m += kh[q] >= c ? 1 : 0;
    if (wave_sum(m) >= num) t = c;
  }
  int gt = 0, eq = 0;
#pragma unroll
  for (int q = 0; q < kSelQ; ++q) {
    gt += kh[q] > t ? 1 : 0;
    eq += kh[q] == t ? 1 : 0;
  }
  gt = wave_sum(gt);
  eq = wave_sum(eq);
  const int need = num - gt;
  int li = 0x7fffffff;  // ties at t (rare): the `need` smallest indices stay
  if (eq > need) {
    int y = 0;  // max y with #{tie, index < y} < need: the need-th smallest tie index
    for (int bit = 30; bit >= 0; --bit) {
      const int c = y | (1 << bit);
      int m = 0;
#pragma unroll
      for (int q = 0; q < kSelQ; ++q)
        if (q < qn && kh[q] == t) m += bl[64 * q].y < c ? 1 : 0;  // (kh == t: a real entry)
      if (wave_sum(m) < need) y = c;
    }
    li = y;
  }
  int ix[kSelQ];
#pragma unroll
  for (int q = 0; q < kSelQ; ++q) ix[q] = kh[q] >= t ? bl[64 * q].y : 0;  // (real entries)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // every lane's reads done first
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int base = 0;  // kept entries move down: a write never passes a later read position
#pragma unroll
  for (int q = 0; q < kSelQ; ++q) {
    const bool k = kh[q] > t || (kh[q] == t && ix[q] <= li);
    const unsigned long long mk = __ballot(k);
    const int pos = base + int(__builtin_amdgcn_mbcnt_hi(
                               unsigned(mk >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(mk), 0)));
    if (k) b[pos] = make_int2(ord_bits(kh[q]), ix[q]);
    base += __popcll(mk);
  }
  return __int_as_float(ord_bits(t));
}

template <int KS, int kBigWaves>
__global__ __launch_bounds__(kBigWaves * 64, kBigWaves == 4 ? 2 : 1) void oap_rec_topk_big(
    RecArgs a, int2* cand, int64_t wg_base, int cap) {
  constexpr int RS = slots_of(KS), ROWB = RS * 16, BLK = blk_of(KS), BUFB = BLK * ROWB;
  constexpr int CH = BUFB / 1024 / kBigWaves;  // 1-KiB glds pieces per wave per block
  constexpr bool kSel = kBigWaves == 4;         // register select (else LDS bitonic)
  static_assert(2 * BUFB == kRecBufs, "two 32 KiB destination buffers");
  static_assert(!kSel || kBigWaves * 64 * kSelQ * 8 <= kRecBufs, "final sorts fit the buffers");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int num = a.num;
  const int64_t ubase = ((wg_base + blockIdx.x) * kBigWaves + wave) * 32;
  const int2 pad = make_int2(__float_as_int(-INFINITY), 0x7fffffff);
  f16x8 uh[KS], ul[KS];
  {
    const f16x8* up = a.src + (ubase + r) * RS;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uh[s] = up[2 * s + h];
      ul[s] = up[2 * KS + 2 * s + h];
    }
  }
  auto buf_of = [&](int ln) {
    return cand + ((int64_t(blockIdx.x) * kBigWaves + wave) * 64 + ln) * cap;
  };
  int2* const wbuf = buf_of(0);  // the wave's 64 lane buffers, cap entries each
  int2* const mine = wbuf + int64_t(lane) * cap;
  int cnt = 0;
  float thr = -INFINITY;
  auto fence = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // lane L's buffer -> exactly its num best (n > num), threshold = the num-th score
  auto compact = [&](int L) {
    const int n = __shfl(cnt, L, 64);
    int2* b = buf_of(L);
    float t_out;
    if constexpr (kSel) {
      t_out = rec_select(b, n, num, lane);
    } else {
      int2* sb = reinterpret_cast<int2*>(smem + kRecBufs);  // (one wave)
      for (int i = lane; i < cap; i += 64) {
        const int2 e = b[i];  // (i < cap: inside the lane buffer; past n masked)
        sb[i] = i < n ? e : pad;
      }
      fence();
      wave_bitonic(sb, cap, lane);
      for (int i = lane; i < num; i += 64) b[i] = sb[i];
      t_out = __int_as_float(sb[num - 1].x);
    }
    if (lane == L) {
      cnt = num;
      thr = t_out;
    }
    fence();
  };
  const int64_t nblk = (a.n_dst + BLK - 1) / BLK;
  auto stage = [&](int64_t blk, int buf) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = wave * CH + j;
      const int byte = c * 1024 + lane * 16;
      const int row = byte / ROWB, p = (byte % ROWB) / 16;
      const f16x8* src = a.dst + (blk * BLK + row) * RS + (p ^ (row & 7));
      __builtin_amdgcn_global_load_lds((glb_ptr_t)(src), (lds_ptr_t)(smem + buf * BUFB + c * 1024),
                                       16, 0, 0);
    }
  };
  auto frag = [&](int buf, int row, int q) -> f16x8 {
    return *reinterpret_cast<const f16x8*>(smem + buf * BUFB + row * ROWB +
                                           ((q ^ (row & 7)) << 4));
  };
  stage(0, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  for (int64_t blk = 0; blk < nblk; ++blk) {
    const int buf = int(blk & 1);
    if (blk + 1 < nblk) stage(blk + 1, buf ^ 1);
#pragma unroll
    for (int sub = 0; sub < BLK / 32; ++sub) {
      const int row = sub * 32 + r;
      f32x16 acc = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const f16x8 ih = frag(buf, row, 2 * s + h);
        const f16x8 il = frag(buf, row, 2 * KS + 2 * s + h);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ih, uh[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ih, ul[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(il, uh[s], acc, 0, 0, 0);
      }
      const int ibase = int(blk * BLK) + sub * 32 + 4 * h;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int di = ibase + 8 * (e >> 2) + (e & 3);
        const float v = acc[e];
        if (di < a.n_dst && v > thr) mine[cnt++] = make_int2(__float_as_int(v), di);
      }
      while (true) {  // room for the next tile's 16 in every lane
        const unsigned long long full = __ballot(cnt > cap - 16);
        if (!full) break;
        compact(__builtin_ctzll(full));
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
  }
  for (int L = 0; L < 64; ++L)  // every list at most num long
    if (__shfl(cnt, L, 64) > num) compact(L);
  // ---- per row: its two half lists sorted together (ties: lower index first), top num out
  const int dexp = scale_exp(a.dst_amax[0]);
  int2* sw = reinterpret_cast<int2*>(smem + (kSel ? wave * 64 * kSelQ * 8 : kRecBufs));
  for (int rr = 0; rr < 32; ++rr) {
    const int ca = __shfl(cnt, rr, 64), cb = __shfl(cnt, rr + 32, 64), tot = ca + cb;
    int sz = 64;
    while (sz < tot) sz <<= 1;
    for (int i = lane; i < sz; i += 64) {  // (offsets selected, never pointers)
      const int off = i < ca ? rr * cap + i : i < tot ? (rr + 32) * cap + (i - ca) : 0;
      const int2 e = wbuf[off];
      sw[i] = i < tot ? e : pad;
    }
    fence();
    wave_bitonic(sw, sz, lane);
    const int64_t u = ubase + rr;
    if (u < a.n_src) {
      const float inv = ldexpf(1.f, -(a.src_exp[u] + dexp));
      for (int t = lane; t < num; t += 64) {
        const bool real = t < tot;
        const int2 z = sw[real ? t : 0];
        a.out_idx[u * num + t] = real ? z.y : -1;
        a.out_val[u * num + t] = real ? __int_as_float(z.x) * inv : -INFINITY;
      }
    }
    fence();
  }
}

template <int KS, int kBigWaves>
void launch_big_w(const RecArgs& a, void* scratch, size_t scratch_bytes, hipStream_t s) {
  const int cap = big_cap(a.num);
  const size_t lds = kRecBufs + (kBigWaves == 4 ? 0 : size_t(cap) * 8);
  OAP_CHECK(cap <= kBigMaxCap && lds <= kRecLds, "oap_rec_topk_big: LDS plan");
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(
        hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_rec_topk_big<KS, kBigWaves>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(kRecLds)));
    attr = true;
  }
  const int64_t per = int64_t(kBigWaves) * 32;
  const int64_t grid = (a.n_src + per - 1) / per;
  const size_t per_wg = size_t(kBigWaves) * 64 * cap * sizeof(int2);
  const int64_t chunk = int64_t(scratch_bytes / per_wg);
  OAP_CHECK(chunk >= 1, "rec_topk: candidate scratch below one workgroup's " << per_wg << " B");
  for (int64_t g0 = 0; g0 < grid; g0 += chunk) {  // (chunks reuse the scratch in stream order)
    const int64_t g = std::min(chunk, grid - g0);
    hipLaunchKernelGGL((oap_rec_topk_big<KS, kBigWaves>), dim3(unsigned(g)),
                       dim3(kBigWaves * 64), lds, s, a, static_cast<int2*>(scratch), g0, cap);
    OAP_HIP_CHECK(hipGetLastError());
  }
}

template <int KS>
void launch_big(const RecArgs& a, void* scratch, size_t scratch_bytes, hipStream_t s) {
  if (big_waves(big_cap(a.num)) == 4)
    launch_big_w<KS, 4>(a, scratch, scratch_bytes, s);
  else
    launch_big_w<KS, 1>(a, scratch, scratch_bytes, s);
}

}  // namespace

int rec_ks(int rank) { return (rank + 15) / 16; }
int rec_row_slots(int rank) { return slots_of(rec_ks(rank)); }
int rec_max_num(int rank) {
  const int ks = rec_ks(rank);
  return ks < 1 || ks > 16 ? 0 : int((kRecLds - kRecBufs) / lists_bytes(1, 1));
}
int rec_big_max_num(int rank) {
  const int ks = rec_ks(rank);
  return ks < 1 || ks > 16 ? 0 : (kBigMaxCap - 16) / 2;
}
size_t rec_big_scratch_per_wg(int num) {
  return size_t(big_waves(big_cap(num))) * 64 * big_cap(num) * sizeof(int2);
}
size_t rec_src_granule(int rank, int num) {
  if (num > rec_max_num(rank)) return size_t(big_waves(big_cap(num))) * 32;
  return size_t(kRecWaves) * 32 * ug_of(rec_ks(rank), num);
}

void rec_row_exp(const float* x, int64_t n, int rank, int64_t ld, int32_t* row_exp,
                 hipStream_t s) {
  if (n <= 0) return;
  const int64_t waves = n < 65536 ? n : 65536;
  hipLaunchKernelGGL(oap_rec_row_exp, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, s, x, n,
                     rank, ld, row_exp);
  OAP_HIP_CHECK(hipGetLastError());
}

void rec_absmax(const float* x, int64_t n, int rank, int64_t ld, unsigned* amax, hipStream_t s) {
  if (n <= 0) return;
  const int64_t waves = n < 8192 ? n : 8192;
  hipLaunchKernelGGL(oap_rec_absmax, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, s, x, n,
                     rank, ld, amax);
  OAP_HIP_CHECK(hipGetLastError());
}

void rec_pack(const float* x, int64_t n, int rank, int64_t ld, const unsigned* amax,
              const int32_t* row_exp, void* img, int64_t rows_pad, hipStream_t s) {
  const int ks = rec_ks(rank);
  OAP_CHECK(ks >= 1 && ks <= 16 && rows_pad >= n, "rec_pack: rank 1..256");
  const int64_t t = rows_pad * slots_of(ks);
  if (t == 0) return;
  hipLaunchKernelGGL(oap_rec_pack, dim3(unsigned((t + 255) / 256)), dim3(256), 0, s, x, n, rank,
                     ld, amax, row_exp, static_cast<f16x8*>(img), rows_pad, ks);
  OAP_HIP_CHECK(hipGetLastError());
}

void rec_topk_big(const void* src_img, const int32_t* src_exp, int64_t n_src,
                  const void* dst_img, const unsigned* dst_amax, int64_t n_dst, int rank, int num,
                  int32_t* out_idx, float* out_val, void* scratch, size_t scratch_bytes,
                  hipStream_t s) {
  OAP_CHECK(num >= 1 && num <= rec_big_max_num(rank) && n_dst >= 1,
            "rec_topk_big: num 1.." << rec_big_max_num(rank) << " at rank " << rank);
  if (n_src <= 0) return;
  RecArgs a;
  a.src = static_cast<const f16x8*>(src_img);
  a.dst = static_cast<const f16x8*>(dst_img);
  a.src_exp = src_exp;
  a.dst_amax = dst_amax;
  a.out_idx = out_idx;
  a.out_val = out_val;
  a.n_src = n_src;
  a.n_dst = n_dst;
  a.num = num;
  switch (rec_ks(rank)) {
    case 1: launch_big<1>(a, scratch, scratch_bytes, s); break;
    case 2: launch_big<2>(a, scratch, scratch_bytes, s); break;
    case 3: launch_big<3>(a, scratch, scratch_bytes, s); break;
    case 4: launch_big<4>(a, scratch, scratch_bytes, s); break;
    case 5: launch_big<5>(a, scratch, scratch_bytes, s); break;
    case 6: launch_big<6>(a, scratch, scratch_bytes, s); break;
    case 7: launch_big<7>(a, scratch, scratch_bytes, s); break;
    case 8: launch_big<8>(a, scratch, scratch_bytes, s); break;
    case 9: launch_big<9>(a, scratch, scratch_bytes, s); break;
    case 10: launch_big<10>(a, scratch, scratch_bytes, s); break;
    case 11: launch_big<11>(a, scratch, scratch_bytes, s); break;
    case 12: launch_big<12>(a, scratch, scratch_bytes, s); break;
    case 13: launch_big<13>(a, scratch, scratch_bytes, s); break;
    case 14: launch_big<14>(a, scratch, scratch_bytes, s); break;
    case 15: launch_big<15>(a, scratch, scratch_bytes, s); break;
    case 16: launch_big<16>(a, scratch, scratch_bytes, s); break;
    default: OAP_THROW(ConfigError, "rec_topk_big: rank " << rank << " beyond 256");
  }
}

void rec_topk(const void* src_img, const int32_t* src_exp, int64_t n_src, const void* dst_img,
              const unsigned* dst_amax, int64_t n_dst, int rank, int num, int32_t* out_idx,
              float* out_val, hipStream_t s) {
  OAP_CHECK(num >= 1 && num <= rec_max_num(rank) && n_dst >= 1,
            "rec_topk: num 1.." << rec_max_num(rank) << " at rank " << rank);
  if (n_src <= 0) return;
  RecArgs a;
  a.src = static_cast<const f16x8*>(src_img);
  a.dst = static_cast<const f16x8*>(dst_img);
  a.src_exp = src_exp;
  a.dst_amax = dst_amax;
  a.out_idx = out_idx;
  a.out_val = out_val;
  a.n_src = n_src;
  a.n_dst = n_dst;
  a.num = num;
  switch (rec_ks(rank)) {
    case 1: launch_ks<1>(a, s); break;
    case 2: launch_ks<2>(a, s); break;
    case 3: launch_ks<3>(a, s); break;
    case 4: launch_ks<4>(a, s); break;
    case 5: launch_ks<5>(a, s); break;
    case 6: launch_ks<6>(a, s); break;
    case 7: launch_ks<7>(a, s); break;
    case 8: launch_ks<8>(a, s); break;
    case 9: launch_ks<9>(a, s); break;
    case 10: launch_ks<10>(a, s); break;
    case 11: launch_ks<11>(a, s); break;
    case 12: launch_ks<12>(a, s); break;
    case 13: launch_ks<13>(a, s); break;
    case 14: launch_ks<14>(a, s); break;
    case 15: launch_ks<15>(a, s); break;
    case 16: launch_ks<16>(a, s); break;
    default: OAP_THROW(ConfigError, "rec_topk: rank " << rank << " beyond 256");
  }
}

}  // namespace kern
}  // namespace oap
