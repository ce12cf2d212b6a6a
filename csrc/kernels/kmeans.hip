// K-Means support kernels (MI355X / gfx950) and the assign dispatcher.
//
// * kmeans_assign: picks the fused MFMA kernel (kmeans_assign.hip) when d <= 128 and the
//   centroids fit one LDS plan, else the generic VALU kernel below.
// * oap_kmeans_finalize — K2+K3 fused: new centroids from the allreduced
//   fixed-point sums (Spark rule: empty clusters keep their center,
//   spark-3.1.1/mllib/clustering/KMeans.scala:306-330) and the tolerance test Σ(Δc)² <= tol²,
//   evaluated redundantly on every rank — the reference needs a root merge plus a `converged`
//   broadcast for this (KMeansDALImpl.cpp:101-130, :207-214).
// * oap_kmeans_accumulate_owned — label-driven fixed-point accumulation for the chunked large-k
//   path (cluster ranges owned by workgroup groups, sums in LDS).
#include <hip/hip_runtime.h>

#include <hip/hip_bf16.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "kernels/device_utils.h"
#include "kernels/kmeans_internal.h"

namespace oap {
namespace kern {

namespace {

// Generic fallback (d > 128): one thread per row, VALU distances, global integer atomics.
template <typename T>
__global__ __launch_bounds__(256) void oap_kmeans_assign_generic(KMeansAssignArgs a, int dp) {
  const T* x = static_cast<const T*>(a.x);
  __shared__ double wsum[4];
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  double my_cost = 0.0;
  for (int64_t row = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; row < a.n; row += stride) {
    const T* xr = x + row * a.ld;
    float best = INFINITY;
    int bidx = 0;
    for (int c = 0; c < a.k; ++c) {
      const float* cr = a.centers + size_t(c) * dp;
      float acc = 0.f;
      for (int f = 0; f < a.d; ++f) {
        const float df = static_cast<float>(xr[f]) - cr[f];
        acc = fmaf(df, df, acc);
      }
      if (acc < best) {
        best = acc;
        bidx = c;
      }
    }
    if (a.merge) {
      if (best < a.mindist[row]) {
        a.mindist[row] = best;
        a.labels[row] = a.base + bidx;
      }
    } else {
      if (a.labels) a.labels[row] = a.base + bidx;
      if (a.mindist) a.mindist[row] = best;
    }
    my_cost += double(best);
    if (a.accumulate && !a.merge) {
      atomicAdd(&a.counts[bidx], 1ull);
      for (int f = 0; a.sums_too && f < a.d; ++f) {
        const long long q = static_cast<long long>(rintf(static_cast<float>(xr[f]) * a.scale[f]));
        atomicAdd(&a.sums[size_t(bidx) * a.d + f], static_cast<u64>(q));
      }
    }
  }
  const double v = wave_sum_f64(my_cost);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0 && a.cost_slab) {
    double t = 0.0;
    for (int w = 0; w < int(blockDim.x / 64); ++w) t += wsum[w];
    a.cost_slab[blockIdx.x] = t;
  }
}

// Label-driven accumulation, global-atomic fallback (rows wider than 64 x 16 bytes).
template <typename T>
__global__ void oap_kmeans_accumulate_global(const T* x, int64_t n, int ld, int d,
                                             const int32_t* labels, int k, const float* scale,
                                             u64* sums, u64* counts) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n * d; i += stride) {
    const int64_t row = i / d;
    const int f = static_cast<int>(i - row * d);
    const int b = labels[row];
    if (b < 0 || b >= k) continue;
    if (f == 0) atomicAdd(&counts[b], 1ull);
    if (!sums) continue;
    const long long q =
        static_cast<long long>(rintf(static_cast<float>(x[row * ld + f]) * scale[f]));
    atomicAdd(&sums[size_t(b) * d + f], static_cast<u64>(q));
  }
}

// Label-driven accumulation for the chunked (large-k) path, deterministic and LDS-resident.
// The k clusters are split into G ranges of kg; block i serves range i % G over row slice i / G
// (256 slices, so per-block partial sums obey the fixed-point bound of
// kmeans_rows_per_block_bound).  A wave reads 64 labels, compacts the rows of its range into a
// wave-private LDS list (ballot + popcount), then gathers those rows 16 bytes per lane — SEG
// lanes cover one padded row, 64 / SEG rows per load instruction, U load groups in flight — and
// adds rint(x * 2^e) into the range's fp64 LDS table (exact integers, so the atomic order cannot
// change a bit).  Table layout: cluster stride `rs` (odd), segment stride EPS + 1 doubles, so
// the SEG lanes of one row hit distinct banks.  One global int64 atomic per (cluster, feature)
// per block at the end.  Replaces a global atomic per row element.
constexpr int kAccThreads = 512;  // (1024: 60 -> 63 ms at 1B rows, k = 1000)
constexpr int kAccU = 4;
template <typename T>
__global__ __launch_bounds__(kAccThreads) void oap_kmeans_accumulate_owned(
    const T* x, int64_t n, int ld, int d, const int32_t* labels, int k, int kg, int G, int rs,
    const float* scale, u64* sums, u64* counts) {
  constexpr int EPS = 16 / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int g = blockIdx.x % G, b = blockIdx.x / G, B = gridDim.x / G;
  const int c0 = g * kg, nk = min(k, c0 + kg) - c0;
  double* acc = reinterpret_cast<double*>(smem);
  const size_t acc_bytes = (size_t(kg) * rs * 8 + 15) / 16 * 16;
  unsigned* cnt = reinterpret_cast<unsigned*>(smem + acc_bytes);
  int* lists = reinterpret_cast<int*>(smem + acc_bytes + (size_t(kg) * 4 + 15) / 16 * 16);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < nk * rs; i += kAccThreads) acc[i] = 0.0;
  for (int i = tid; i < nk; i += kAccThreads) cnt[i] = 0u;
  __syncthreads();
  const int SEG = ld * int(sizeof(T)) / 16, rpi = 64 / SEG;
  const int slot = lane / SEG, seg = lane - slot * SEG;
  const bool lane_ok = slot < rpi;
  float sc[EPS];
#pragma unroll
  for (int j = 0; j < EPS; ++j) {
    const int f = seg * EPS + j;
    sc[j] = (sums && lane_ok && f < d) ? scale[f] : 0.f;
  }
  int* rows_l = lists + wave * 128;
  int* cls_l = rows_l + 64;
  const int64_t r0 = n * b / B, r1 = n * (b + 1) / B;
  for (int64_t base = r0 + int64_t(wave) * 64; base < r1; base += int64_t(kAccThreads)) {
    const int64_t row = base + lane;
    int cl = -1;
    if (row < r1) {
      const int lab = labels[row];
      if (static_cast<unsigned>(lab - c0) < static_cast<unsigned>(nk)) cl = lab - c0;
    }
    const u64 mask = __ballot(cl >= 0);
    if (mask == 0) continue;
    if (cl >= 0) {
      const int pos = __popcll(mask & ((1ull << lane) - 1ull));
      rows_l[pos] = lane;
      cls_l[pos] = cl;
      atomicAdd(&cnt[cl], 1u);
    }
    if (!sums) continue;
    __builtin_amdgcn_wave_barrier();  // the list is written and read by this wave only
    const int m = __popcll(mask);
    for (int q0 = 0; q0 < m; q0 += rpi * kAccU) {
      T v[kAccU][EPS];
      int clq[kAccU];
      bool ok[kAccU];
#pragma unroll
      for (int u = 0; u < kAccU; ++u) {
        const int qi = q0 + u * rpi + slot;
        ok[u] = lane_ok && qi < m;
        clq[u] = 0;
        if (ok[u]) {
          clq[u] = cls_l[qi];
          const T* p = x + (base + rows_l[qi]) * ld + seg * EPS;
          const uint4 raw = *reinterpret_cast<const uint4*>(p);
          __builtin_memcpy(&v[u][0], &raw, 16);
        }
      }
#pragma unroll
      for (int u = 0; u < kAccU; ++u) {
        if (!ok[u]) continue;
        double* ap = acc + clq[u] * rs + seg * (EPS + 1);
#pragma unroll
        for (int j = 0; j < EPS; ++j)
          if (seg * EPS + j < d)
            atomicAdd(ap + j, static_cast<double>(rintf(static_cast<float>(v[u][j]) * sc[j])));
      }
    }
    __builtin_amdgcn_wave_barrier();  // list reads done before the next batch overwrites it
  }
  __syncthreads();
  if (sums)
    for (int i = tid; i < nk * d; i += kAccThreads) {
      const int c = i / d, f = i - c * d;
      const double v = acc[c * rs + (f / EPS) * (EPS + 1) + f % EPS];  // exact, |v| < 2^53
      if (v != 0.0)
        atomicAdd(&sums[size_t(c0 + c) * d + f], static_cast<u64>(static_cast<long long>(v)));
    }
  for (int i = tid; i < nk; i += kAccThreads)
    if (cnt[i]) atomicAdd(&counts[c0 + i], static_cast<u64>(cnt[i]));
}

// ---- counts only (k-means|| candidate weights): a label histogram, the rows are never read.
// Per-block LDS histogram of all k clusters, one global atomic per non-empty (block, cluster).
constexpr int kCntThreads = 256;
__global__ __launch_bounds__(kCntThreads) void oap_kmeans_count_labels(const int32_t* labels,
                                                                        int64_t n, int k,
                                                                        u64* counts) {
  extern __shared__ unsigned hist[];
  for (int i = threadIdx.x; i < k; i += kCntThreads) hist[i] = 0u;
  __syncthreads();
  const int64_t n4 = n / 4;
  const int4* l4 = reinterpret_cast<const int4*>(labels);
  for (int64_t q = int64_t(blockIdx.x) * kCntThreads + threadIdx.x; q < n4;
       q += int64_t(gridDim.x) * kCntThreads) {
    const int4 v = l4[q];
    if (unsigned(v.x) < unsigned(k)) atomicAdd(&hist[v.x], 1u);
    if (unsigned(v.y) < unsigned(k)) atomicAdd(&hist[v.y], 1u);
    if (unsigned(v.z) < unsigned(k)) atomicAdd(&hist[v.z], 1u);
    if (unsigned(v.w) < unsigned(k)) atomicAdd(&hist[v.w], 1u);
  }
  if (blockIdx.x == 0)
    for (int64_t r = n4 * 4 + threadIdx.x; r < n; r += kCntThreads) {
      const int v = labels[r];
      if (unsigned(v) < unsigned(k)) atomicAdd(&hist[v], 1u);
    }
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += kCntThreads)
    if (hist[i]) atomicAdd(&counts[i], static_cast<u64>(hist[i]));
}

// ---- binned accumulation: rows grouped by cluster range first (two cheap passes over the
// labels), so every lane of the accumulation kernel works on a row of its range — the scan
// variant above reads every label in every range and keeps a dependent load chain per 64 rows.
constexpr int kBinThreads = 256;
constexpr int kBinRows = 4096;  // rows per bin block chunk
__global__ __launch_bounds__(kBinThreads) void oap_kmeans_bin_count(const int32_t* labels,
                                                                     int64_t n, int kg, int G,
                                                                     unsigned* gcount) {
  extern __shared__ unsigned hist[];
  for (int i = threadIdx.x; i < G; i += kBinThreads) hist[i] = 0u;
  __syncthreads();
  for (int64_t r = int64_t(blockIdx.x) * kBinThreads + threadIdx.x; r < n;
       r += int64_t(gridDim.x) * kBinThreads) {
    const int g = labels[r] / kg;
    atomicAdd(&hist[min(max(g, 0), G - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBinThreads)
    if (hist[i]) atomicAdd(&gcount[i], hist[i]);
}

// gcount [G] -> goff [G+1] exclusive offsets; gfill [G] = goff (scatter cursors)
__global__ void oap_kmeans_bin_offsets(const unsigned* gcount, int G, unsigned* goff,
                                       unsigned* gfill) {
  if (threadIdx.x != 0) return;
  unsigned acc = 0;
  for (int g = 0; g < G; ++g) {
    goff[g] = acc;
    gfill[g] = acc;
    acc += gcount[g];
  }
  goff[G] = acc;
}

// One chunk of kBinRows rows per block iteration: LDS ranks per range, one global reservation
// per (chunk, range), then the (row, label) entries land in their range's region.
__global__ __launch_bounds__(kBinThreads) void oap_kmeans_bin_scatter(const int32_t* labels,
                                                                       int64_t n, int kg, int G,
                                                                       unsigned* gfill,
                                                                       int2* bins) {
  extern __shared__ unsigned sm[];
  unsigned* cnt = sm;       // [G]
  unsigned* base = sm + G;  // [G]
  constexpr int kPer = kBinRows / kBinThreads;
  for (int64_t c0 = int64_t(blockIdx.x) * kBinRows; c0 < n; c0 += int64_t(gridDim.x) * kBinRows) {
    for (int i = threadIdx.x; i < G; i += kBinThreads) cnt[i] = 0u;
    __syncthreads();
    int lab[kPer];
    unsigned pos[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t r = c0 + j * kBinThreads + threadIdx.x;
      lab[j] = r < n ? labels[r] : -1;
      pos[j] = 0u;
      if (r < n) pos[j] = atomicAdd(&cnt[min(max(lab[j] / kg, 0), G - 1)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G; i += kBinThreads)
      base[i] = cnt[i] ? atomicAdd(&gfill[i], cnt[i]) : 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t r = c0 + j * kBinThreads + threadIdx.x;
      if (r < n) {
        const int g = min(max(lab[j] / kg, 0), G - 1);
        bins[base[g] + pos[j]] = make_int2(static_cast<int>(r), lab[j]);
      }
    }
    __syncthreads();
  }
}

// Accumulation over the binned entries of range g = blockIdx % G: block slice b of the range's
// entries (256 slices: the fixed-point per-block bound holds as in the scan variant).  Entries
// are fetched two batches ahead and rows one batch ahead of the LDS atomics, so the dependent
// entry -> row load chain overlaps the previous batch's atomics.
template <typename T>
__global__ __launch_bounds__(kAccThreads) void oap_kmeans_accumulate_binned(
    const T* x, int ld, int d, const int2* bins, const unsigned* goff, int k, int kg, int G,
    int rs, const float* scale, u64* sums, u64* counts) {
  constexpr int EPS = 16 / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int g = blockIdx.x % G, b = blockIdx.x / G, B = gridDim.x / G;
  const int c0 = g * kg, nk = min(k, c0 + kg) - c0;
  double* acc = reinterpret_cast<double*>(smem);
  const size_t acc_bytes = (size_t(kg) * rs * 8 + 15) / 16 * 16;
  unsigned* cnt = reinterpret_cast<unsigned*>(smem + acc_bytes);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < nk * rs; i += kAccThreads) acc[i] = 0.0;
  for (int i = tid; i < nk; i += kAccThreads) cnt[i] = 0u;
  __syncthreads();
  const int SEG = ld * int(sizeof(T)) / 16, rpi = 64 / SEG;
  const int slot = lane / SEG, seg = lane - slot * SEG;
  const bool lane_ok = slot < rpi;
  float sc[EPS];
#pragma unroll
  for (int j = 0; j < EPS; ++j) {
    const int f = seg * EPS + j;
    sc[j] = (sums && lane_ok && f < d) ? scale[f] : 0.f;
  }
  const int64_t tot = int64_t(goff[g + 1]) - goff[g];
  const int64_t e0 = goff[g] + tot * b / B, e1 = goff[g] + tot * (b + 1) / B;
  const int per = rpi * kAccU;                       // entries per wave batch
  const int64_t step = int64_t(kAccThreads / 64) * per;  // entries per block batch
  struct Batch {
    int2 en[kAccU];
    T v[kAccU][EPS];
  };
  // entry (row, cluster): row >= 0 adds the row, row <= -2 subtracts row -row - 2 (delta
  // accumulation of moved rows), -1 is empty
  auto load_entries = [&](int64_t q0, Batch& bt) {
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      const int64_t qi = q0 + u * rpi + slot;
      bt.en[u] = (lane_ok && qi < e1) ? bins[qi] : make_int2(-1, -1);
    }
  };
  auto load_rows = [&](Batch& bt) {
#pragma unroll
    for (int u = 0; u < kAccU; ++u)
      if (bt.en[u].x != -1) {
        const int64_t row = bt.en[u].x >= 0 ? int64_t(bt.en[u].x) : -int64_t(bt.en[u].x) - 2;
        const T* p = x + row * ld + seg * EPS;
        const uint4 raw = *reinterpret_cast<const uint4*>(p);
        __builtin_memcpy(&bt.v[u][0], &raw, 16);
      }
  };
  auto consume = [&](const Batch& bt) {
#pragma unroll
    for (int u = 0; u < kAccU; ++u) {
      if (bt.en[u].x == -1) continue;
      const bool neg = bt.en[u].x < -1;
      const int cl = bt.en[u].y - c0;
      if (seg == 0) atomicAdd(&cnt[cl], neg ? 0xffffffffu : 1u);
      if (!sums) continue;
      double* ap = acc + cl * rs + seg * (EPS + 1);
      const float sg = neg ? -1.f : 1.f;
#pragma unroll
      for (int j = 0; j < EPS; ++j)
        if (seg * EPS + j < d)
          atomicAdd(ap + j,
                    static_cast<double>(sg * rintf(static_cast<float>(bt.v[u][j]) * sc[j])));
    }
  };
  // three rotating batches: at the top of each step X0 holds batch q (rows in flight) and X1
  // the entries of batch q + step
  int64_t q = e0 + int64_t(wave) * per;
  Batch X0, X1, X2;
  load_entries(q, X0);
  load_rows(X0);
  load_entries(q + step, X1);
  for (; q < e1; q += 3 * step) {
    load_rows(X1);
    load_entries(q + 2 * step, X2);
    consume(X0);
    if (q + step >= e1) break;
    load_rows(X2);
    load_entries(q + 3 * step, X0);
    consume(X1);
    if (q + 2 * step >= e1) break;
    load_rows(X0);
    load_entries(q + 4 * step, X1);
    consume(X2);
  }
  __syncthreads();
  if (sums)
    for (int i = tid; i < nk * d; i += kAccThreads) {
      const int c = i / d, f = i - c * d;
      const double v = acc[c * rs + (f / EPS) * (EPS + 1) + f % EPS];  // exact, |v| < 2^53
      if (v != 0.0)
        atomicAdd(&sums[size_t(c0 + c) * d + f], static_cast<u64>(static_cast<long long>(v)));
    }
  for (int i = tid; i < nk; i += kAccThreads)  // (signed: delta entries may subtract)
    if (cnt[i])
      atomicAdd(&counts[c0 + i],
                static_cast<u64>(static_cast<long long>(static_cast<int>(cnt[i]))));
}

// ---- delta accumulation (moved rows only): rows whose label changed become two entries,
// (row, new) and (-row - 2, old).  Two passes so that a fallback costs no writes and no
// contended counter: oap_kmeans_moved_count (one atomic per block), then oap_kmeans_moved_write
// over chunks of kMovedRows rows per block step (a block-wide exclusive scan of the per-thread
// counts, ONE reservation per chunk).  The entry order is irrelevant (integer sums).
constexpr int kMovedPer = 16, kMovedRows = 256 * kMovedPer;
__device__ inline bool row_moved(const int32_t* oldl, const int32_t* newl, int64_t r, int64_t n,
                                 int k, int& o, int& nw) {
  if (r >= n) return false;
  o = oldl[r];
  nw = newl[r];
  return o != nw && unsigned(o) < unsigned(k) && unsigned(nw) < unsigned(k);
}

__global__ __launch_bounds__(256) void oap_kmeans_moved_count(const int32_t* __restrict__ oldl,
                                                              const int32_t* __restrict__ newl,
                                                              int64_t n, int k, unsigned* count) {
  __shared__ unsigned ws[4];
  unsigned c = 0;
  for (int64_t r = int64_t(blockIdx.x) * 256 + threadIdx.x; r < n; r += int64_t(gridDim.x) * 256) {
    int o, nw;
    c += row_moved(oldl, newl, r, n, k, o, nw) ? 1u : 0u;
  }
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = ws[0] + ws[1] + ws[2] + ws[3];
    if (t) atomicAdd(count, t);
  }
}

__global__ __launch_bounds__(256) void oap_kmeans_moved_write(const int32_t* __restrict__ oldl,
                                                              const int32_t* __restrict__ newl,
                                                              int64_t n, int k, int2* ent,
                                                              unsigned* fill) {
  __shared__ unsigned scan[256];
  __shared__ unsigned base;
  const int t = threadIdx.x;
  for (int64_t c0 = int64_t(blockIdx.x) * kMovedRows; c0 < n;
       c0 += int64_t(gridDim.x) * kMovedRows) {
    unsigned mine = 0;
#pragma unroll
    for (int j = 0; j < kMovedPer; ++j) {
      int o, nw;
      mine += row_moved(oldl, newl, c0 + int64_t(t) * kMovedPer + j, n, k, o, nw) ? 1u : 0u;
    }
    scan[t] = mine;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {  // inclusive Hillis-Steele scan
      const unsigned v = t >= off ? scan[t - off] : 0u;
      __syncthreads();
      scan[t] += v;
      __syncthreads();
    }
    if (t == 255) base = scan[255] ? atomicAdd(fill, 2u * scan[255]) : 0u;
    __syncthreads();
    unsigned at = base + 2u * (scan[t] - mine);
#pragma unroll
    for (int j = 0; j < kMovedPer; ++j) {
      const int64_t r = c0 + int64_t(t) * kMovedPer + j;
      int o, nw;
      if (row_moved(oldl, newl, r, n, k, o, nw)) {
        ent[at] = make_int2(static_cast<int>(r), nw);
        ent[at + 1] = make_int2(-static_cast<int>(r) - 2, o);
        at += 2;
      }
    }
    __syncthreads();
  }
}

// bin_count / bin_scatter over an entry list whose length is on the device
__global__ __launch_bounds__(kBinThreads) void oap_kmeans_bin_count_e(const int2* ent,
                                                                       const unsigned* count,
                                                                       unsigned cap, int kg, int G,
                                                                       unsigned* gcount) {
  extern __shared__ unsigned hist[];
  const int64_t n = min(*count, cap);
  for (int i = threadIdx.x; i < G; i += kBinThreads) hist[i] = 0u;
  __syncthreads();
  for (int64_t r = int64_t(blockIdx.x) * kBinThreads + threadIdx.x; r < n;
       r += int64_t(gridDim.x) * kBinThreads)
    atomicAdd(&hist[min(max(ent[r].y / kg, 0), G - 1)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBinThreads)
    if (hist[i]) atomicAdd(&gcount[i], hist[i]);
}

__global__ __launch_bounds__(kBinThreads) void oap_kmeans_bin_scatter_e(const int2* ent,
                                                                         const unsigned* count,
                                                                         unsigned cap, int kg,
                                                                         int G, unsigned* gfill,
                                                                         int2* bins) {
  extern __shared__ unsigned sm[];
  unsigned* cnt = sm;       // [G]
  unsigned* base = sm + G;  // [G]
  constexpr int kPer = kBinRows / kBinThreads;
  const int64_t n = min(*count, cap);
  for (int64_t c0 = int64_t(blockIdx.x) * kBinRows; c0 < n; c0 += int64_t(gridDim.x) * kBinRows) {
    for (int i = threadIdx.x; i < G; i += kBinThreads) cnt[i] = 0u;
    __syncthreads();
    int2 e[kPer];
    unsigned pos[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t r = c0 + j * kBinThreads + threadIdx.x;
      e[j] = r < n ? ent[r] : make_int2(-1, -1);
      pos[j] = 0u;
      if (r < n) pos[j] = atomicAdd(&cnt[min(max(e[j].y / kg, 0), G - 1)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G; i += kBinThreads)
      base[i] = cnt[i] ? atomicAdd(&gfill[i], cnt[i]) : 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t r = c0 + j * kBinThreads + threadIdx.x;
      if (r < n) bins[base[min(max(e[j].y / kg, 0), G - 1)] + pos[j]] = e[j];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void oap_kmeans_finalize(KMeansFinalizeArgs a) {
  if (a.halt && *a.halt) return;
  __shared__ int s_conv, s_nonempty;
  __shared__ double s_shift[4];
  __shared__ float s_norm[4], s_drift[4];
  if (threadIdx.x == 0) {
    s_conv = 1;
    s_nonempty = 0;
  }
  __syncthreads();
  double my_max = 0.0;
  float my_nmax = 0.f, my_drift = 0.f;
  for (int c = threadIdx.x; c < a.k; c += blockDim.x) {
    const long long cntv = static_cast<long long>(a.counts[c]);
    double* c64 = a.centers64 + size_t(c) * a.d;
    double shift2 = 0.0, nrm = 0.0, dr2 = 0.0;
    if (cntv > 0) {
      atomicAdd(&s_nonempty, 1);
      for (int f = 0; f < a.d; ++f) {
        const long long sv = static_cast<long long>(a.sums[size_t(c) * a.d + f]);
        const double nv = double(sv) * a.inv_scale[f] / double(cntv);  // == CPU engine formula
        const double df = nv - c64[f];
        const double dv = double(static_cast<float>(nv) - static_cast<float>(c64[f]));
        shift2 += df * df;
        dr2 += dv * dv;
        c64[f] = nv;
      }
      if (shift2 > a.tol * a.tol) atomicAnd(&s_conv, 0);
      if (shift2 > my_max) my_max = shift2;
    }
    if (a.drift) {
      const float dr = static_cast<float>(sqrt(dr2) * (1.0 + 1e-6));  // rounded up
      a.drift[c] = dr;
      my_drift = fmaxf(my_drift, dr);
    }
    for (int f = 0; f < a.d; ++f) {
      const float v = static_cast<float>(c64[f]);
      a.centers32[size_t(c) * a.dp + f] = v;
      nrm += double(v) * double(v);
    }
    a.cnorm[c] = static_cast<float>(nrm);
    my_nmax = fmaxf(my_nmax, sqrtf(static_cast<float>(nrm)));
  }
  // wave maxima by shuffles, then the block's 4 waves (a serial loop over 256 LDS slots was
  // most of the finalize's ~16 us)
  for (int m = 32; m >= 1; m >>= 1) {
    my_max = fmax(my_max, __shfl_xor(my_max, m, 64));
    my_nmax = fmaxf(my_nmax, __shfl_xor(my_nmax, m, 64));
    my_drift = fmaxf(my_drift, __shfl_xor(my_drift, m, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    s_shift[threadIdx.x >> 6] = my_max;
    s_norm[threadIdx.x >> 6] = my_nmax;
    s_drift[threadIdx.x >> 6] = my_drift;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double mx = 0.0;
    float nm = 0.f, dm = 0.f;
    for (int i = 0; i < int(blockDim.x) / 64; ++i) {
      mx = fmax(mx, s_shift[i]);
      nm = fmaxf(nm, s_norm[i]);
      dm = fmaxf(dm, s_drift[i]);
    }
    KMeansFlags* fl = static_cast<KMeansFlags*>(a.flags);
    fl->converged = s_conv;
    fl->nonempty = s_nonempty;
    fl->cost = a.cost_in ? a.cost_in[0] : 0.0;
    fl->max_shift2 = mx;
    if (a.cost_reset) a.cost_reset[0] = 0.0;
    if (a.cstat) a.cstat[0] = nm * 1.0000001f;
    if (a.drift) a.drift[a.k] = dm;
    if (a.halt && s_conv && a.tol >= 0.0) a.halt[0] = 1;
  }
}

// The flags of a multi-block finalize from the per-cluster scratch (one block of 256 threads).
__device__ void finalize_flags_block(const KMeansFinalizeArgs& a) {
  __shared__ double s_shift[4];
  __shared__ float s_norm[4], s_drift[4];
  __shared__ int s_conv, s_nonempty;
  if (threadIdx.x == 0) {
    s_conv = 1;
    s_nonempty = 0;
  }
  __syncthreads();
  double my_max = 0.0;
  float my_nmax = 0.f, my_drift = 0.f;
  for (int c = threadIdx.x; c < a.k; c += blockDim.x) {
    const double sh = a.scratch[c];
    if (sh >= 0.0) {
      atomicAdd(&s_nonempty, 1);
      if (sh > a.tol * a.tol) atomicAnd(&s_conv, 0);
      my_max = fmax(my_max, sh);
    }
    my_nmax = fmaxf(my_nmax, static_cast<float>(a.scratch[a.k + c]));
    if (a.drift) my_drift = fmaxf(my_drift, a.drift[c]);
  }
  // wave maxima by shuffles, then the block's 4 waves (a serial loop over 256 LDS slots was
  // most of the finalize's ~16 us)
  for (int m = 32; m >= 1; m >>= 1) {
    my_max = fmax(my_max, __shfl_xor(my_max, m, 64));
    my_nmax = fmaxf(my_nmax, __shfl_xor(my_nmax, m, 64));
    my_drift = fmaxf(my_drift, __shfl_xor(my_drift, m, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    s_shift[threadIdx.x >> 6] = my_max;
    s_norm[threadIdx.x >> 6] = my_nmax;
    s_drift[threadIdx.x >> 6] = my_drift;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double mx = 0.0;
    float nm = 0.f, dm = 0.f;
    for (int i = 0; i < int(blockDim.x) / 64; ++i) {
      mx = fmax(mx, s_shift[i]);
      nm = fmaxf(nm, s_norm[i]);
      dm = fmaxf(dm, s_drift[i]);
    }
    if (a.drift) a.drift[a.k] = dm;
    KMeansFlags* fl = static_cast<KMeansFlags*>(a.flags);
    fl->converged = s_conv;
    fl->nonempty = s_nonempty;
    fl->cost = a.cost_in ? a.cost_in[0] : 0.0;
    fl->max_shift2 = mx;
    if (a.cost_reset) a.cost_reset[0] = 0.0;
    if (a.cstat) a.cstat[0] = nm * 1.0000001f;
    if (a.halt && s_conv && a.tol >= 0.0) a.halt[0] = 1;
  }
}

// Multi-block finalize (one wave per cluster): new centers + per-cluster shift / norm into
// scratch; the flags from them (the last block to finish when a.done is set, else
// oap_kmeans_finalize_flags).  The fp64 sums keep the single-block kernel's sequential feature
// order (lane 0), so results are bitwise unchanged.
__global__ __launch_bounds__(256) void oap_kmeans_finalize_clusters(KMeansFinalizeArgs a) {
  if (a.halt && *a.halt) return;  // (every block: the done counter stays untouched)
  __shared__ double s_df[4][256];
  __shared__ float s_dv[4][256], s_v[4][256];
  __shared__ bool s_last;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + w;
  if (c < a.k) {
    const long long cntv = static_cast<long long>(a.counts[c]);
    double* c64 = a.centers64 + size_t(c) * a.d;
    // lane 0: the shift, the squared movement of the fp32 center and |c|^2 (fp32 values), each
    // summed in feature order from this wave's LDS rows (no serial global reads)
    double sh = 0.0, dr2 = 0.0, nrm = 0.0;
    for (int f0 = 0; f0 < a.d; f0 += 256) {
      const int nf = min(256, a.d - f0);
      for (int f = lane; f < nf; f += 64) {
        double df = 0.0;
        float dv = 0.f;
        if (cntv > 0) {
          const long long sv = static_cast<long long>(a.sums[size_t(c) * a.d + f0 + f]);
          const double nv = double(sv) * a.inv_scale[f0 + f] / double(cntv);  // == CPU formula
          df = nv - c64[f0 + f];
          dv = static_cast<float>(nv) - static_cast<float>(c64[f0 + f]);
          c64[f0 + f] = nv;
        }
        const float v = static_cast<float>(c64[f0 + f]);
        a.centers32[size_t(c) * a.dp + f0 + f] = v;
        s_df[w][f] = df;
        s_dv[w][f] = dv;
        s_v[w][f] = v;
      }
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
#pragma unroll 8
        for (int f = 0; f < nf; ++f) {
          sh += s_df[w][f] * s_df[w][f];
          dr2 += double(s_dv[w][f]) * double(s_dv[w][f]);
          nrm += double(s_v[w][f]) * double(s_v[w][f]);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) {
      if (a.drift) a.drift[c] = static_cast<float>(sqrt(dr2) * (1.0 + 1e-6));
      a.cnorm[c] = static_cast<float>(nrm);
      a.scratch[a.k + c] = double(sqrtf(static_cast<float>(nrm)));
      a.scratch[c] = cntv <= 0 ? -1.0 : sh;  // empty: keeps its center, not part of the test
    }
  }
  if (!a.done) return;
  // last block: every other block's scratch / drift writes are visible (release before the
  // count, acquire after it)
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(a.done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  finalize_flags_block(a);
  if (threadIdx.x == 0) a.done[0] = 0u;
}

__global__ __launch_bounds__(256) void oap_kmeans_finalize_flags(KMeansFinalizeArgs a) {
  if (a.halt && *a.halt) return;
  finalize_flags_block(a);
}

__global__ __launch_bounds__(256) void oap_copy_guarded(uint4* __restrict__ dst,
                                                        const uint4* __restrict__ src, int64_t n16,
                                                        unsigned* __restrict__ dst4,
                                                        const unsigned* __restrict__ src4, int n4,
                                                        const int* __restrict__ halt) {
  if (halt && *halt) return;
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i < n16) dst[i] = src[i];
  if (blockIdx.x == 0 && threadIdx.x < n4) dst4[threadIdx.x] = src4[threadIdx.x];
}

// (one thread: a handful of counters per batch)
__global__ void oap_kmeans_ctl(KMeansCtlArgs a) {
  if (threadIdx.x != 0) return;
  const unsigned long long t2 = a.refine ? a.refine[1] : 0ull;
  const unsigned long long df = a.ldstat ? a.ldstat[0] : 0ull;
  const unsigned long long mv = a.ldstat ? a.ldstat[1] : 0ull;
  const unsigned long long pr = a.pruned ? a.pruned[0] : 0ull;
  const double tiles = double((a.rows + 31) / 32);
  double share = 0.0, frac = 1.0, mvf = 0.0;
  if (a.rows > 0) {
    share = double(t2 - a.snap[0]) / (0.02 * tiles * a.nb_it);
    if (a.ldstat) share = fmax(share, double(df - a.snap[1]) / (0.25 * double(a.rows) * a.nb_it));
    if (a.scan_iters > 0 && a.scan_local)
      frac = double(pr - a.snap[2]) / (tiles * a.scan_iters + 1e-9);
    mvf = double(mv) / double(a.rows);
  }
  a.snap[0] = t2;
  a.snap[1] = df;
  a.snap[2] = pr;
  a.out[0] = share;
  a.out[1] = -frac;
  a.out[2] = mvf;
  double fl = 0.0, ncap = 0.0;
  if (a.bound_flag) {
    fl = double(a.bound_flag[0]);
    ncap = sqrt(double(__uint_as_float(a.bound_flag[1])) * (1.0 + 1e-5));
  }
  a.out[3] = fl;
  a.out[4] = ncap;
}

__global__ void oap_kmeans_prepare_centers(const double* c64, int k, int d, int dp, float* c32,
                                           float* cnorm, float* cstat, int kpad) {
  __shared__ float s_norm[256];
  float nmax = 0.f;
  for (int c = threadIdx.x; c < kpad; c += blockDim.x) {
    if (c >= k) {
      cnorm[c] = INFINITY;
      for (int f = 0; f < dp; ++f) c32[size_t(c) * dp + f] = 0.f;
      continue;
    }
    double nrm = 0.0;
    for (int f = 0; f < dp; ++f) {
      const float v = f < d ? static_cast<float>(c64[size_t(c) * d + f]) : 0.f;
      c32[size_t(c) * dp + f] = v;
      nrm += double(v) * double(v);
    }
    cnorm[c] = static_cast<float>(nrm);
    nmax = fmaxf(nmax, sqrtf(static_cast<float>(nrm)));
  }
  s_norm[threadIdx.x] = nmax;
  __syncthreads();
  if (threadIdx.x == 0 && cstat) {
    float m = 0.f;
    for (int i = 0; i < int(blockDim.x); ++i) m = fmaxf(m, s_norm[i]);
    cstat[0] = m * 1.0000001f;
  }
}

}  // namespace

// --------------------------------------------------------------------------- host wrappers
int kmeans_ld(int d, bool bf16) { return bf16 ? (d + 7) / 8 * 8 : (d + 3) / 4 * 4; }
int kmeans_dp(int d) { return d <= 128 ? (d + 15) / 16 * 16 : d; }
int kmeans_cost_slab_size(int num_cus) { return num_cus > 8192 ? num_cus : 8192; }
int kmeans_lds_kmax(int d, bool precise) { return kmeans_mfma_kmax(d, precise); }

int64_t kmeans_rows_per_block_bound(int64_t n) {
  const int64_t tiles = (n + 31) / 32;
  const int64_t per_wave = (tiles + 2047) / 2048;  // grid >= 256 blocks x 8 waves once busy
  return 256 * (per_wave < 1 ? 1 : per_wave);
}

int kmeans_assign(const KMeansAssignArgs& a, int num_cus, hipStream_t s) {
  OAP_CHECK(a.kpad % 32 == 0 && a.kpad >= a.k, "kpad must be a multiple of 32 >= k");
  OAP_CHECK(a.ld == kmeans_ld(a.d, a.xbf16),
            "row stride " << a.ld << " != kmeans_ld(" << a.d << ", " << a.xbf16 << ")");
  OAP_CHECK(!a.merge || (a.labels && a.mindist), "merge mode needs labels and mindist");
  if (a.n == 0) return 0;
  const int dp = kmeans_dp(a.d);
  const bool generic = a.d > 128 || a.kpad > kmeans_mfma_kmax(a.d, a.precise);
  if (generic) {
    const int grid = grid_for(a.n, 256, 4096);
    if (a.xbf16)
      hipLaunchKernelGGL(oap_kmeans_assign_generic<__bf16>, dim3(grid), dim3(256), 0, s, a, dp);
    else
      hipLaunchKernelGGL(oap_kmeans_assign_generic<float>, dim3(grid), dim3(256), 0, s, a, dp);
    OAP_HIP_CHECK(hipGetLastError());
    return grid;
  }
  const int grid = kmeans_mfma_grid(a.n, num_cus);
  launch_kmeans_assign_mfma(a, grid, s);
  return grid;
}

void kmeans_assign_rows(const KMeansAssignArgs& a, int grid, hipStream_t s) {
  OAP_CHECK(a.row_list && a.row_count && a.row_seg_cap > 0 && !a.merge && !a.precise &&
                a.d <= 128 && a.kpad <= kmeans_mfma_kmax(a.d, false) && !a.tile_list,
            "kmeans_assign_rows: unsupported arguments");
  if (a.n == 0) return;
  launch_kmeans_assign_mfma(a, grid, s);
}

void kmeans_seed_mindist(const KMeansAssignArgs& a, hipStream_t s) {
  launch_kmeans_seed_mindist(a, s);
}

int kmeans_label_cost(const KMeansAssignArgs& a, double* slab, int max_blocks, hipStream_t s) {
  return launch_kmeans_label_cost(a, slab, max_blocks, s);
}

__global__ void oap_kmeans_count_pruned(const unsigned* listed, int64_t ntiles, int passes,
                                        unsigned long long* pruned) {
  if (threadIdx.x == 0)
    *pruned += static_cast<unsigned long long>(ntiles - int64_t(*listed)) * passes;
}

void kmeans_count_pruned(const unsigned* listed, int64_t ntiles, int passes,
                         unsigned long long* pruned, hipStream_t s) {
  hipLaunchKernelGGL(oap_kmeans_count_pruned, dim3(1), dim3(64), 0, s, listed, ntiles, passes,
                     pruned);
  OAP_HIP_CHECK(hipGetLastError());
}

// Delta-mode pruning scan: one thread per row, a wave = two 32-row tiles.  The test is the assign
// kernel's own single-launch pruning test (kmeans_assign.hip, `prune_single`) with the tile's
// largest |x|^2 (stored per tile by the assign kernel) in the margin — never looser per row.
__global__ __launch_bounds__(256) void oap_kmeans_prune_scan(
    int64_t n, int k, int d, float2* __restrict__ bounds, const int32_t* __restrict__ labels,
    const float* __restrict__ xnorm, const float* __restrict__ drift,
    const float* __restrict__ drift_max, const float* __restrict__ cstat,
    int32_t* __restrict__ tile_list, unsigned* __restrict__ tile_count,
    unsigned long long* __restrict__ pruned) {
  __shared__ unsigned wcnt[4], wbase[4];
  __shared__ unsigned long long bpruned;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const float dmax = drift_max[0];
  const float cmax = cstat[0];
  const float mrel = 4e-7f * float(d + 8);
  const int64_t ntiles = (n + 31) / 32;
  const int64_t nchunks = (n + 255) / 256;  // a chunk = 256 rows = 8 tiles, one per block step
  if (threadIdx.x == 0) bpruned = 0;
  unsigned long long n_pruned = 0;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {  // block-uniform trip count
    const int64_t w = c * 4 + wave;  // this wave's tile pair
    const int64_t row = w * 64 + lane;
    const bool valid = row < n;
    bool ok = true;
    float2 bnew = make_float2(0.f, 0.f);
    if (valid) {
      const float2 b = bounds[row];
      const int lab = min(max(labels[row], 0), k - 1);
      const float u = b.x + drift[lab];
      const float lk = b.y - dmax;
      ok = lk > 0.f && (lk - u) * (lk + u) > mrel * (xnorm[row >> 5] + cmax * cmax);
      // outward rounding: the advanced bounds stay bounds whatever fp32 did to the sums
      bnew = make_float2(u * (1.f + 2.5e-7f), lk * (1.f - 2.5e-7f));
    }
    const unsigned long long all_ok = __ballot(ok);
    const bool pr0 = static_cast<unsigned>(all_ok) == 0xffffffffu;
    const bool pr1 = static_cast<unsigned>(all_ok >> 32) == 0xffffffffu;
    // no center moved (dmax == 0, every drift is 0): the stored bounds already hold, no write
    if (dmax > 0.f && valid && (h ? pr1 : pr0)) bounds[row] = bnew;
    const bool has0 = 2 * w < ntiles, has1 = 2 * w + 1 < ntiles;
    const bool act0 = has0 && !pr0, act1 = has1 && !pr1;
    if (lane == 0) {
      wcnt[wave] = unsigned(act0) + unsigned(act1);
      n_pruned += unsigned(has0 && pr0) + unsigned(has1 && pr1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
      unsigned pos = tot ? atomicAdd(tile_count, tot) : 0u;
      for (int i = 0; i < 4; ++i) {
        wbase[i] = pos;
        pos += wcnt[i];
      }
    }
    __syncthreads();
    if (lane == 0) {
      unsigned pos = wbase[wave];
      if (act0) tile_list[pos++] = static_cast<int32_t>(2 * w);
      if (act1) tile_list[pos] = static_cast<int32_t>(2 * w + 1);
    }
  }
  if (lane == 0 && n_pruned) atomicAdd(&bpruned, n_pruned);
  __syncthreads();
  if (threadIdx.x == 0 && bpruned && pruned) atomicAdd(pruned, bpruned);
}

void kmeans_prune_scan(int64_t n, int k, int d, float* bounds, const int32_t* labels,
                       const float* xnorm, const float* drift, const float* drift_max,
                       const float* cstat, int32_t* tile_list, unsigned* tile_count,
                       unsigned long long* pruned, hipStream_t s) {
  if (n <= 0) return;
  const int grid = static_cast<int>(std::min<int64_t>((n + 255) / 256, 8192));
  hipLaunchKernelGGL(oap_kmeans_prune_scan, dim3(grid), dim3(256), 0, s, n, k, d,
                     reinterpret_cast<float2*>(bounds), labels, xnorm, drift, drift_max, cstat,
                     tile_list, tile_count, pruned);
  OAP_HIP_CHECK(hipGetLastError());
}

namespace {
// counts without sums: label histogram (labels must be 16-byte aligned, as device buffers are)
bool count_labels(const int32_t* labels, int64_t n, int k, unsigned long long* counts,
                  hipStream_t s) {
  if (size_t(k) * 4 > kLdsLimit - 64 || (reinterpret_cast<uintptr_t>(labels) & 15)) return false;
  const int grid = static_cast<int>(std::max<int64_t>(
      1, std::min<int64_t>((n / 4 + kCntThreads - 1) / kCntThreads, 2048)));
  static bool set = false;
  if (!set) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_kmeans_count_labels),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(kLdsLimit)));
    set = true;
  }
  hipLaunchKernelGGL(oap_kmeans_count_labels, dim3(grid), dim3(kCntThreads), size_t(k) * 4, s,
                     labels, n, k, counts);
  OAP_HIP_CHECK(hipGetLastError());
  return true;
}
}  // namespace

void kmeans_accumulate(const void* x, bool xbf16, int64_t n, int ld, int d,
                       const int32_t* labels, int k, const float* scale,
                       unsigned long long* sums, unsigned long long* counts, hipStream_t s) {
  if (n == 0) return;
  if (!sums && count_labels(labels, n, k, counts, s)) return;
  const int es = xbf16 ? 2 : 4, eps = 16 / es;
  const int seg = ld * es / 16;
  OAP_CHECK(ld * es % 16 == 0, "kmeans_accumulate: rows must be 16-byte multiples");
  // LDS plan: [kg x rs] fp64 sums | [kg] counts | 8 waves x 128 ints of compaction lists
  const size_t fixed = size_t(kAccThreads / 64) * 128 * 4 + 32;
  int rs = 0, kg = k;
  if (sums) {
    rs = (seg * (eps + 1)) | 1;
    kg = static_cast<int>((kLdsLimit - fixed) / (size_t(rs) * 8 + 4));
  } else {
    kg = static_cast<int>(std::min<size_t>(size_t(k), (kLdsLimit - fixed) / 4));
  }
  if (seg > 64 || kg < 1) {  // very wide rows: global atomics
    const dim3 grid(grid_for(n * d, 256));
    if (xbf16)
      hipLaunchKernelGGL(oap_kmeans_accumulate_global<__bf16>, grid, dim3(256), 0, s,
                         static_cast<const __bf16*>(x), n, ld, d, labels, k, scale, sums, counts);
    else
      hipLaunchKernelGGL(oap_kmeans_accumulate_global<float>, grid, dim3(256), 0, s,
                         static_cast<const float*>(x), n, ld, d, labels, k, scale, sums, counts);
    OAP_HIP_CHECK(hipGetLastError());
    return;
  }
  const int G = (k + kg - 1) / kg;
  kg = (k + G - 1) / G;
  const size_t lds = (size_t(kg) * rs * 8 + 15) / 16 * 16 + (size_t(kg) * 4 + 15) / 16 * 16 +
                     size_t(kAccThreads / 64) * 128 * 4;
  OAP_CHECK(lds <= kLdsLimit, "kmeans_accumulate: LDS plan " << lds);
  const dim3 grid(256 * G);  // 256 row slices per cluster range (fixed-point bound)
  if (xbf16) {
    static bool set = false;
    if (!set) {
      OAP_HIP_CHECK(hipFuncSetAttribute(
          reinterpret_cast<const void*>(&oap_kmeans_accumulate_owned<__bf16>),
          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
      set = true;
    }
    hipLaunchKernelGGL(oap_kmeans_accumulate_owned<__bf16>, grid, dim3(kAccThreads), lds, s,
                       static_cast<const __bf16*>(x), n, ld, d, labels, k, kg, G, rs, scale, sums,
                       counts);
  } else {
    static bool set = false;
    if (!set) {
      OAP_HIP_CHECK(hipFuncSetAttribute(
          reinterpret_cast<const void*>(&oap_kmeans_accumulate_owned<float>),
          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
      set = true;
    }
    hipLaunchKernelGGL(oap_kmeans_accumulate_owned<float>, grid, dim3(kAccThreads), lds, s,
                       static_cast<const float*>(x), n, ld, d, labels, k, kg, G, rs, scale, sums,
                       counts);
  }
  OAP_HIP_CHECK(hipGetLastError());
}

bool kmeans_accumulate_moved(const void* x, bool xbf16, int64_t n, int ld, int d,
                             const int32_t* old_labels, const int32_t* new_labels, int k,
                             const float* scale, unsigned long long* sums,
                             unsigned long long* counts, void* scratch, size_t scratch_bytes,
                             int64_t* entries, hipStream_t s) {
  *entries = 0;
  if (n == 0) return true;
  const int es = xbf16 ? 2 : 4, eps = 16 / es;
  const int seg = ld * es / 16;
  OAP_CHECK(sums && ld * es % 16 == 0 && seg <= 64 && n < (int64_t(1) << 30),
            "kmeans_accumulate_moved: unsupported layout");
  const int rs = (seg * (eps + 1)) | 1;
  int kg = static_cast<int>((kLdsLimit - 64) / (size_t(rs) * 8 + 4));
  OAP_CHECK(kg >= 1, "kmeans_accumulate_moved: rows too wide");
  const int G = (k + kg - 1) / kg;
  kg = (k + G - 1) / G;
  const size_t lds = (size_t(kg) * rs * 8 + 15) / 16 * 16 + (size_t(kg) * 4 + 15) / 16 * 16;
  // scratch: [count | G gcount | G + 1 goff | G gfill] then two entry arrays of cap each
  unsigned* hdr = static_cast<unsigned*>(scratch);
  const size_t hdr_words = (3 * size_t(G) + 2 + 3) / 4 * 4;
  const size_t cap = (scratch_bytes - hdr_words * 4) / (2 * sizeof(int2));
  int2* ent = reinterpret_cast<int2*>(hdr + hdr_words);
  int2* bins = ent + cap;
  unsigned* count = hdr;
  unsigned* gcount = hdr + 1;
  unsigned* goff = gcount + G;
  unsigned* gfill = goff + G + 1;
  OAP_HIP_CHECK(hipMemsetAsync(hdr, 0, sizeof(unsigned) * (1 + G), s));
  const int mgrid = static_cast<int>(std::min<int64_t>((n + 255) / 256, 4096));
  hipLaunchKernelGGL(oap_kmeans_moved_count, dim3(mgrid), dim3(256), 0, s, old_labels,
                     new_labels, n, k, count);
  OAP_HIP_CHECK(hipGetLastError());
  unsigned moved = 0;
  OAP_HIP_CHECK(hipMemcpyAsync(&moved, count, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  const unsigned h = 2u * moved;
  *entries = int64_t(h);
  // nothing accumulated (the caller recounts): over the capacity, or so many moved rows that
  // the scattered double reads cost more than the full binned pass (measured at 1B rows,
  // k = 1000: 14% moved rows 489 vs 381 ms/iteration; break-even near 5%)
  if (size_t(h) > cap || int64_t(h) > n / 10) return false;
  if (h == 0) return true;
  OAP_HIP_CHECK(hipMemsetAsync(count, 0, sizeof(unsigned), s));  // reused as the fill cursor
  const int wgrid = static_cast<int>(std::min<int64_t>((n + kMovedRows - 1) / kMovedRows, 4096));
  hipLaunchKernelGGL(oap_kmeans_moved_write, dim3(wgrid), dim3(256), 0, s, old_labels, new_labels,
                     n, k, ent, count);
  OAP_HIP_CHECK(hipGetLastError());
  const int bgrid = static_cast<int>(std::min<int64_t>((int64_t(h) + kBinRows - 1) / kBinRows,
                                                       4096));
  hipLaunchKernelGGL(oap_kmeans_bin_count_e, dim3(bgrid), dim3(kBinThreads),
                     sizeof(unsigned) * G, s, ent, count, h, kg, G, gcount);
  hipLaunchKernelGGL(oap_kmeans_bin_offsets, dim3(1), dim3(64), 0, s, gcount, G, goff, gfill);
  hipLaunchKernelGGL(oap_kmeans_bin_scatter_e, dim3(bgrid), dim3(kBinThreads),
                     sizeof(unsigned) * 2 * G, s, ent, count, h, kg, G, gfill, bins);
  OAP_HIP_CHECK(hipGetLastError());
  const dim3 grid(256 * G);
  if (xbf16) {
    static bool set = false;
    if (!set) {
      OAP_HIP_CHECK(hipFuncSetAttribute(
          reinterpret_cast<const void*>(&oap_kmeans_accumulate_binned<__bf16>),
          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
      set = true;
    }
    hipLaunchKernelGGL(oap_kmeans_accumulate_binned<__bf16>, grid, dim3(kAccThreads), lds, s,
                       static_cast<const __bf16*>(x), ld, d, bins, goff, k, kg, G, rs, scale, sums,
                       counts);
  } else {
    static bool set = false;
    if (!set) {
      OAP_HIP_CHECK(hipFuncSetAttribute(
          reinterpret_cast<const void*>(&oap_kmeans_accumulate_binned<float>),
          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
      set = true;
    }
    hipLaunchKernelGGL(oap_kmeans_accumulate_binned<float>, grid, dim3(kAccThreads), lds, s,
                       static_cast<const float*>(x), ld, d, bins, goff, k, kg, G, rs, scale, sums,
                       counts);
  }
  OAP_HIP_CHECK(hipGetLastError());
  return true;
}

size_t kmeans_bin_scratch_bytes(int64_t n, int k) {
  return sizeof(int2) * size_t(std::max<int64_t>(n, 1)) + sizeof(unsigned) * (3 * size_t(k) + 8);
}

bool kmeans_accumulate_binned(const void* x, bool xbf16, int64_t n, int ld, int d,
                              const int32_t* labels, int k, const float* scale,
                              unsigned long long* sums, unsigned long long* counts, void* scratch,
                              hipStream_t s) {
  if (n == 0) return true;
  if (!sums) return count_labels(labels, n, k, counts, s);
  const int es = xbf16 ? 2 : 4, eps = 16 / es;
  const int seg = ld * es / 16;
  if (ld * es % 16 != 0 || seg > 64 || n >= (int64_t(1) << 31)) return false;
  int rs = 0, kg = k;
  if (sums) {
    rs = (seg * (eps + 1)) | 1;
    kg = static_cast<int>((kLdsLimit - 64) / (size_t(rs) * 8 + 4));
  } else {
    kg = static_cast<int>(std::min<size_t>(size_t(k), (kLdsLimit - 64) / 4));
  }
  if (kg < 1) return false;
  const int G = (k + kg - 1) / kg;
  kg = (k + G - 1) / G;
  const size_t lds = (size_t(kg) * rs * 8 + 15) / 16 * 16 + (size_t(kg) * 4 + 15) / 16 * 16;
  if (lds > kLdsLimit) return false;
  int2* bins = static_cast<int2*>(scratch);
  unsigned* gcount = reinterpret_cast<unsigned*>(bins + n);
  unsigned* goff = gcount + G;  // [G + 1]
  unsigned* gfill = goff + G + 1;
  OAP_HIP_CHECK(hipMemsetAsync(gcount, 0, sizeof(unsigned) * G, s));
  const int bgrid = static_cast<int>(std::min<int64_t>((n + kBinRows - 1) / kBinRows, 4096));
  hipLaunchKernelGGL(oap_kmeans_bin_count, dim3(bgrid), dim3(kBinThreads), sizeof(unsigned) * G,
                     s, labels, n, kg, G, gcount);
  hipLaunchKernelGGL(oap_kmeans_bin_offsets, dim3(1), dim3(64), 0, s, gcount, G, goff, gfill);
  hipLaunchKernelGGL(oap_kmeans_bin_scatter, dim3(bgrid), dim3(kBinThreads),
                     sizeof(unsigned) * 2 * G, s, labels, n, kg, G, gfill, bins);
  OAP_HIP_CHECK(hipGetLastError());
  const dim3 grid(256 * G);  // 256 slices per cluster range (fixed-point bound)
  if (xbf16) {
    static bool set = false;
    if (!set) {
      OAP_HIP_CHECK(hipFuncSetAttribute(
          reinterpret_cast<const void*>(&oap_kmeans_accumulate_binned<__bf16>),
          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
      set = true;
    }
    hipLaunchKernelGGL(oap_kmeans_accumulate_binned<__bf16>, grid, dim3(kAccThreads), lds, s,
                       static_cast<const __bf16*>(x), ld, d, bins, goff, k, kg, G, rs, scale, sums,
                       counts);
  } else {
    static bool set = false;
    if (!set) {
      OAP_HIP_CHECK(hipFuncSetAttribute(
          reinterpret_cast<const void*>(&oap_kmeans_accumulate_binned<float>),
          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsLimit)));
      set = true;
    }
    hipLaunchKernelGGL(oap_kmeans_accumulate_binned<float>, grid, dim3(kAccThreads), lds, s,
                       static_cast<const float*>(x), ld, d, bins, goff, k, kg, G, rs, scale, sums,
                       counts);
  }
  OAP_HIP_CHECK(hipGetLastError());
  return true;
}

void kmeans_finalize(const KMeansFinalizeArgs& a, hipStream_t s) {
  if (a.scratch) {
    hipLaunchKernelGGL(oap_kmeans_finalize_clusters, dim3((a.k + 3) / 4), dim3(256), 0, s, a);
    OAP_HIP_CHECK(hipGetLastError());
    if (!a.done) hipLaunchKernelGGL(oap_kmeans_finalize_flags, dim3(1), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(oap_kmeans_finalize, dim3(1), dim3(256), 0, s, a);
  }
  OAP_HIP_CHECK(hipGetLastError());
}

void copy_guarded(void* dst, const void* src, size_t bytes, const int* halt, hipStream_t s) {
  OAP_CHECK(bytes % 4 == 0 && reinterpret_cast<uintptr_t>(dst) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(src) % 16 == 0,
            "copy_guarded: 16-byte aligned buffers of whole dwords");
  if (bytes == 0) return;
  const int64_t n16 = int64_t(bytes / 16);
  const int n4 = int((bytes % 16) / 4);
  const int grid = int(n16 > 0 ? (n16 + 255) / 256 : 1);
  hipLaunchKernelGGL(oap_copy_guarded, dim3(grid), dim3(256), 0, s, static_cast<uint4*>(dst),
                     static_cast<const uint4*>(src), n16,
                     reinterpret_cast<unsigned*>(static_cast<char*>(dst) + n16 * 16),
                     reinterpret_cast<const unsigned*>(static_cast<const char*>(src) + n16 * 16),
                     n4, halt);
  OAP_HIP_CHECK(hipGetLastError());
}

void kmeans_ctl(const KMeansCtlArgs& a, hipStream_t s) {
  OAP_CHECK(a.snap && a.out && a.nb_it >= 1, "kmeans_ctl: bad arguments");
  hipLaunchKernelGGL(oap_kmeans_ctl, dim3(1), dim3(64), 0, s, a);
  OAP_HIP_CHECK(hipGetLastError());
}

void kmeans_prepare_centers(const double* centers64, int k, int d, int dp, float* centers32,
                            float* cnorm, float* cstat, int kpad, hipStream_t s) {
  hipLaunchKernelGGL(oap_kmeans_prepare_centers, dim3(1), dim3(256), 0, s, centers64, k, d, dp,
                     centers32, cnorm, cstat, kpad);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
