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

}  // namespace

int rec_ks(int rank) { return (rank + 15) / 16; }
int rec_row_slots(int rank) { return slots_of(rec_ks(rank)); }
int rec_max_num(int rank) {
  const int ks = rec_ks(rank);
  return ks < 1 || ks > 16 ? 0 : int((kRecLds - kRecBufs) / lists_bytes(1, 1));
}
size_t rec_src_granule(int rank, int num) {
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
