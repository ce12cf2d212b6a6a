// Device-side ALS setup: dense id re-indexing and both CSR matrices on the GPU (see
// kernels/als_setup.h).  Ids are re-indexed through a presence bitmap over [min, max] and an
// exclusive scan (rank = index among the distinct ids, ascending); each rating becomes one
// packed 64-bit key (row << cbits | col) per CSR and a stable LSD radix sort (rocPRIM) orders
// the ratings by (row, col) — row pointers come from a per-row count and a scan.  Every pass is
// a streaming pass over HBM: ~50 ms of device time per CSR at 1B ratings.
//
// The multi-rank variant (als_device_setup_dist) does the reference's ratings shuffle
// (ALSShuffle.cpp:62-127: alltoall of lengths, alltoallv of 20-byte records, std::sort) and CSR
// build (ALSDALImpl.scala:184-230, ALSDALImpl.cpp:153-214) as three owner partitions of SoA
// device buffers: a stable radix sort by owner rank, a gather, and an alltoallv of the three
// columns (RCCL grouped send/recv; host comms stage through pinned memory).
#include "kernels/als_setup.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdint>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "runtime/common.h"

namespace oap {
namespace kern {

namespace {

constexpr int kThreads = 256;

int grid_of(int64_t n) {
  const int64_t g = (n + kThreads - 1) / kThreads;
  return int(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

#define OAP_GRID_LOOP(k, n)                                                                    \
  for (int64_t k = blockIdx.x * int64_t(kThreads) + threadIdx.x; k < (n);                      \
       k += int64_t(gridDim.x) * kThreads)

__global__ void oap_als_minmax(const int32_t* __restrict__ u, const int32_t* __restrict__ it,
                               int64_t n, int* mm) {
  int umin = INT_MAX, umax = INT_MIN, imin = INT_MAX, imax = INT_MIN;
  OAP_GRID_LOOP(k, n) {
    const int a = u[k], b = it[k];
    umin = min(umin, a);
    umax = max(umax, a);
    imin = min(imin, b);
    imax = max(imax, b);
  }
  for (int m = 32; m >= 1; m >>= 1) {
    umin = min(umin, __shfl_xor(umin, m, 64));
    umax = max(umax, __shfl_xor(umax, m, 64));
    imin = min(imin, __shfl_xor(imin, m, 64));
    imax = max(imax, __shfl_xor(imax, m, 64));
  }
  // few blocks (grid <= 2048): one set of 4 atomics per wave stays off the critical path (one
  // per 256 rows of a full grid serialised on the 4 words: 12 ms at 20M ratings)
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], umin);
    atomicMax(&mm[1], umax);
    atomicMin(&mm[2], imin);
    atomicMax(&mm[3], imax);
  }
}

__global__ void oap_als_init_mm(int* mm) {
  mm[0] = INT_MAX;
  mm[1] = INT_MIN;
  mm[2] = INT_MAX;
  mm[3] = INT_MIN;
}

__global__ void oap_als_flag(const int32_t* __restrict__ ids, int64_t n, int lo,
                             int32_t* __restrict__ flag) {
  OAP_GRID_LOOP(k, n) flag[ids[k] - lo] = 1;
}

__global__ void oap_als_compact_ids(const int32_t* __restrict__ flag,
                                    const int32_t* __restrict__ rank, int64_t range, int lo,
                                    int32_t* __restrict__ ids) {
  OAP_GRID_LOOP(x, range) if (flag[x]) ids[rank[x]] = int32_t(lo + x);
}

// packed keys of both CSRs and per-row counts
__global__ void oap_als_keys(const int32_t* __restrict__ u, const int32_t* __restrict__ it,
                             int64_t n, int ulo, int ilo, const int32_t* __restrict__ urank,
                             const int32_t* __restrict__ irank, int ubits, int ibits,
                             uint64_t* __restrict__ ku, uint64_t* __restrict__ ki,
                             int32_t* __restrict__ ucnt, int32_t* __restrict__ icnt) {
  OAP_GRID_LOOP(k, n) {
    const uint64_t ur = uint64_t(urank[u[k] - ulo]), ir = uint64_t(irank[it[k] - ilo]);
    ku[k] = (ur << ibits) | ir;
    ki[k] = (ir << ubits) | ur;
    atomicAdd(&ucnt[ur], 1);
    atomicAdd(&icnt[ir], 1);
  }
}

__global__ void oap_als_key_cols(const uint64_t* __restrict__ key, int64_t n, int cbits,
                                 int32_t* __restrict__ col) {
  const uint64_t m = (uint64_t(1) << cbits) - 1;
  OAP_GRID_LOOP(k, n) col[k] = int32_t(key[k] & m);
}

// ---- multi-rank setup kernels ---------------------------------------------------------------
// Owner rank of every rating: id mod P (bounds == nullptr) or the slab of a global index
// (upper_bound over the P + 1 rank offsets); per-owner counts through an LDS histogram.
__global__ void oap_als_owner(const int32_t* __restrict__ key, int64_t n, int P,
                              const int64_t* __restrict__ bounds, uint32_t* __restrict__ owner,
                              int32_t* __restrict__ iota, unsigned long long* __restrict__ counts) {
  extern __shared__ unsigned int hist[];
  for (int q = threadIdx.x; q < P; q += kThreads) hist[q] = 0;
  __syncthreads();
  OAP_GRID_LOOP(k, n) {
    const int64_t v = key[k];
    int q;
    if (bounds == nullptr) {
      q = int(((v % P) + P) % P);
    } else {
      int lo = 0, hi = P;  // largest q with bounds[q] <= v
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (bounds[mid] <= v) lo = mid;
        else hi = mid;
      }
      q = lo;
    }
    owner[k] = uint32_t(q);
    iota[k] = int32_t(k);
    atomicAdd(&hist[q], 1u);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < P; q += kThreads)
    if (hist[q]) atomicAdd(&counts[q], (unsigned long long)hist[q]);
}

// out_x[j] = x[perm[j]] for the three SoA columns of a rating
__global__ void oap_als_gather3(const int32_t* __restrict__ perm, int64_t n,
                                const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                                const float* __restrict__ r, int32_t* __restrict__ oa,
                                int32_t* __restrict__ ob, float* __restrict__ orr) {
  OAP_GRID_LOOP(j, n) {
    const int32_t k = perm[j];
    oa[j] = a[k];
    ob[j] = b[k];
    orr[j] = r[k];
  }
}

// ids[k] <- base + rank[ids[k] - lo] (global dense index of an owned id)
__global__ void oap_als_to_index(int32_t* __restrict__ ids, int64_t n, int lo,
                                 const int32_t* __restrict__ rank, int64_t base) {
  OAP_GRID_LOOP(k, n) ids[k] = int32_t(base + rank[ids[k] - lo]);
}

// CSR keys of owned rows: row = rank[rowid - lo] (rank != nullptr) or rowid - sub; col as given
__global__ void oap_als_csr_keys(const int32_t* __restrict__ rowid, const int32_t* __restrict__ col,
                                 int64_t n, const int32_t* __restrict__ rank, int lo, int64_t sub,
                                 int cbits, uint64_t* __restrict__ key,
                                 int32_t* __restrict__ cnt) {
  OAP_GRID_LOOP(k, n) {
    const int64_t row = rank ? int64_t(rank[rowid[k] - lo]) : int64_t(rowid[k]) - sub;
    key[k] = (uint64_t(row) << cbits) | uint64_t(uint32_t(col[k]));
    atomicAdd(&cnt[row], 1);
  }
}

// order-independent checksums of the three columns: sum of the 32-bit patterns (wrap-free for
// up to 2^31 ratings); the shuffle verifies that every rating arrived exactly once
__global__ void oap_als_checksum(const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                                 const float* __restrict__ r, int64_t n,
                                 unsigned long long* __restrict__ out) {
  unsigned long long sa = 0, sb = 0, sr = 0;
  OAP_GRID_LOOP(k, n) {
    sa += uint32_t(a[k]);
    sb += uint32_t(b[k]);
    sr += __float_as_uint(r[k]);
  }
  for (int m = 32; m >= 1; m >>= 1) {
    sa += __shfl_xor(sa, m, 64);
    sb += __shfl_xor(sb, m, 64);
    sr += __shfl_xor(sr, m, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&out[0], sa);
    atomicAdd(&out[1], sb);
    atomicAdd(&out[2], sr);
  }
}

__global__ void oap_als_copy_i32(const int32_t* __restrict__ src, int64_t n,
                                 int32_t* __restrict__ dst) {
  OAP_GRID_LOOP(k, n) dst[k] = src[k];
}

int bits_for(int64_t count) {  // bits to hold indices [0, count)
  int b = 1;
  while ((int64_t(1) << b) < count) ++b;
  return b;
}

template <typename T>
void exclusive_scan_dev(Context& ctx, const int32_t* in, T* out, size_t n, hipStream_t s) {
  size_t tb = 0;
  OAP_HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, in, out, T(0), n, rocprim::plus<T>(), s));
  Buffer tmp = ctx.alloc(std::max<size_t>(tb, 16));
  OAP_HIP_CHECK(rocprim::exclusive_scan(tmp.data(), tb, in, out, T(0), n, rocprim::plus<T>(), s));
}

// Dense index of the distinct ids among ids[0, n) within [lo, lo + range): rank (per id value,
// exclusive scan of presence flags) and the sorted distinct ids (device + host copies).
int64_t dense_index(Context& ctx, const int32_t* ids, int64_t n, int lo, int64_t range,
                    hipStream_t s, Buffer& rank, Buffer& dev_ids, std::vector<int32_t>& host_ids) {
  Buffer flag = ctx.alloc(size_t(range) * 4);
  rank = ctx.alloc(size_t(range) * 4);
  OAP_HIP_CHECK(hipMemsetAsync(flag.data(), 0, size_t(range) * 4, s));
  if (n > 0)
    hipLaunchKernelGGL(oap_als_flag, dim3(grid_of(n)), dim3(kThreads), 0, s, ids, n, lo,
                       flag.as<int32_t>());
  exclusive_scan_dev<int32_t>(ctx, flag.as<int32_t>(), rank.as<int32_t>(), size_t(range), s);
  int32_t last[2];
  ctx.copy_to_host(&last[0], rank.as<int32_t>() + range - 1, 4, s);
  ctx.copy_to_host(&last[1], flag.as<int32_t>() + range - 1, 4, s);
  const int64_t count = int64_t(last[0]) + last[1];
  dev_ids = ctx.alloc(std::max<size_t>(size_t(count) * 4, 16));
  hipLaunchKernelGGL(oap_als_compact_ids, dim3(grid_of(range)), dim3(kThreads), 0, s,
                     flag.as<int32_t>(), rank.as<int32_t>(), range, lo, dev_ids.as<int32_t>());
  OAP_HIP_CHECK(hipGetLastError());
  host_ids.resize(count);
  ctx.copy_to_host(host_ids.data(), dev_ids.data(), size_t(count) * 4, s);
  return count;
}

// Stable radix sort of (key, val) pairs -> cols (low cbits of the key), row pointers from the
// per-row counts (nrows + 1 entries, the last one 0).
void csr_from_keys(Context& ctx, Buffer& keys, const float* vals, int64_t n, int64_t nrows,
                   int bits, int cbits, Buffer& cnt, hipStream_t s, AlsDeviceCsr& csr) {
  csr.nrows = nrows;
  csr.val = ctx.alloc(std::max<size_t>(size_t(n) * 4, 16));
  csr.col = ctx.alloc(std::max<size_t>(size_t(n) * 4, 16));
  if (n > 0) {
    Buffer ksorted = ctx.alloc(size_t(n) * 8);
    size_t tb = 0;
    OAP_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tb, keys.as<uint64_t>(),
                                            ksorted.as<uint64_t>(), vals, csr.val.as<float>(),
                                            size_t(n), 0, bits, s));
    {
      Buffer tmp = ctx.alloc(std::max<size_t>(tb, 16));
      OAP_HIP_CHECK(rocprim::radix_sort_pairs(tmp.data(), tb, keys.as<uint64_t>(),
                                              ksorted.as<uint64_t>(), vals, csr.val.as<float>(),
                                              size_t(n), 0, bits, s));
    }
    keys = Buffer();
    hipLaunchKernelGGL(oap_als_key_cols, dim3(grid_of(n)), dim3(kThreads), 0, s,
                       ksorted.as<uint64_t>(), n, cbits, csr.col.as<int32_t>());
    OAP_HIP_CHECK(hipGetLastError());
  }
  csr.ptr = ctx.alloc(size_t(nrows + 1) * 8);
  exclusive_scan_dev<int64_t>(ctx, cnt.as<int32_t>(), csr.ptr.as<int64_t>(), size_t(nrows + 1),
                              s);
  csr.ptr_h.resize(nrows + 1);
  ctx.copy_to_host(csr.ptr_h.data(), csr.ptr.data(), size_t(nrows + 1) * 8, s);
  OAP_CHECK(csr.ptr_h[nrows] == n, "ALS device setup: row pointer total " << csr.ptr_h[nrows]
                                                                           << " != " << n);
}

}  // namespace

bool als_device_setup(Context& ctx, const int32_t* users, const int32_t* items,
                      const float* ratings, int64_t n, hipStream_t s, AlsDeviceSetup* out) {
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a) {
    return std::chrono::duration<double, std::milli>(clk::now() - a).count();
  };
  if (n <= 0 || n >= (int64_t(1) << 31)) return false;
  auto t0 = clk::now();
  Buffer du = ctx.alloc(size_t(n) * 4), di = ctx.alloc(size_t(n) * 4);
  Buffer dr = ctx.alloc(size_t(n) * 4);
  ctx.copy_to_backend(du.data(), users, size_t(n) * 4, s);
  ctx.copy_to_backend(di.data(), items, size_t(n) * 4, s);
  ctx.copy_to_backend(dr.data(), ratings, size_t(n) * 4, s);
  Buffer mmb = ctx.alloc(64);
  hipLaunchKernelGGL(oap_als_init_mm, dim3(1), dim3(1), 0, s, mmb.as<int>());
  hipLaunchKernelGGL(oap_als_minmax, dim3(std::min(grid_of(n), 2048)), dim3(kThreads), 0, s,
                     du.as<int32_t>(), di.as<int32_t>(), n, mmb.as<int>());
  OAP_HIP_CHECK(hipGetLastError());
  int mm[4];
  ctx.copy_to_host(mm, mmb.data(), sizeof(mm), s);
  out->upload_ms = ms(t0);
  const int64_t urange = int64_t(mm[1]) - mm[0] + 1, irange = int64_t(mm[3]) - mm[2] + 1;
  const int64_t cap = std::max<int64_t>(8 * n, int64_t(1) << 26);
  if (urange > cap || irange > cap || urange >= (int64_t(1) << 31) ||
      irange >= (int64_t(1) << 31))
    return false;

  auto t1 = clk::now();
  // ---- dense indices: presence flags -> exclusive scan (rank) -> distinct ids
  Buffer urank, irank, uids, iids;
  const int64_t nu = dense_index(ctx, du.as<int32_t>(), n, mm[0], urange, s, urank, uids,
                                 out->user_ids);
  const int64_t ni = dense_index(ctx, di.as<int32_t>(), n, mm[2], irange, s, irank, iids,
                                 out->item_ids);
  const int ubits = bits_for(nu), ibits = bits_for(ni);
  OAP_CHECK(ubits + ibits <= 64, "als_device_setup: index bits");
  Buffer ku = ctx.alloc(size_t(n) * 8), ki = ctx.alloc(size_t(n) * 8);
  Buffer ucnt = ctx.alloc(size_t(nu + 1) * 4), icnt = ctx.alloc(size_t(ni + 1) * 4);
  OAP_HIP_CHECK(hipMemsetAsync(ucnt.data(), 0, size_t(nu + 1) * 4, s));
  OAP_HIP_CHECK(hipMemsetAsync(icnt.data(), 0, size_t(ni + 1) * 4, s));
  hipLaunchKernelGGL(oap_als_keys, dim3(grid_of(n)), dim3(kThreads), 0, s, du.as<int32_t>(),
                     di.as<int32_t>(), n, mm[0], mm[2], urank.as<int32_t>(), irank.as<int32_t>(),
                     ubits, ibits, ku.as<uint64_t>(), ki.as<uint64_t>(), ucnt.as<int32_t>(),
                     icnt.as<int32_t>());
  OAP_HIP_CHECK(hipGetLastError());
  du = Buffer();
  di = Buffer();
  urank = Buffer();
  irank = Buffer();
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  out->index_ms = ms(t1);

  auto t2 = clk::now();
  // ---- per side: stable radix sort of (key, rating), cols from the keys, row pointers
  csr_from_keys(ctx, ku, dr.as<float>(), n, nu, ubits + ibits, ibits, ucnt, s, out->users);
  csr_from_keys(ctx, ki, dr.as<float>(), n, ni, ubits + ibits, ubits, icnt, s, out->items);
  out->sort_ms = ms(t2);
  return true;
}

// ------------------------------------------------------------------------- multi-rank setup
namespace {

// Ratings as three device columns (a = row-side id, b = col-side id / index, r = value).
struct Soa {
  Buffer a, b, r;
  int64_t n = 0;
  void alloc(Context& ctx, int64_t m) {
    n = m;
    const size_t bytes = std::max<size_t>(size_t(m) * 4, 16);
    a = ctx.alloc(bytes);
    b = ctx.alloc(bytes);
    r = ctx.alloc(bytes);
  }
};

// Routes every rating to the owner of its `a` column (by_a) or `b` column: owner = id mod P
// (bounds empty) or the rank slab holding a global index (bounds = P + 1 offsets).  The
// partition is a stable radix sort by owner, so each destination receives its records in source
// order, and the result is in source-rank order — the same order as the host exchange.
Soa shuffle(Context& ctx, Comm& comm, Soa& in, bool by_a, const std::vector<int64_t>& bounds,
            hipStream_t s) {
  const int P = comm.size(), me = comm.rank();
  const int64_t n = in.n;
  Buffer owner = ctx.alloc(std::max<size_t>(size_t(n) * 4, 16));
  Buffer iota = ctx.alloc(std::max<size_t>(size_t(n) * 4, 16));
  Buffer counts = ctx.alloc(size_t(P) * 8 + 8);
  Buffer dbounds;
  OAP_HIP_CHECK(hipMemsetAsync(counts.data(), 0, size_t(P) * 8, s));
  if (!bounds.empty()) {
    dbounds = ctx.alloc(bounds.size() * 8);
    ctx.copy_to_backend(dbounds.data(), bounds.data(), bounds.size() * 8, s);
  }
  hipLaunchKernelGGL(oap_als_owner, dim3(std::min(grid_of(n), 4096)), dim3(kThreads),
                     size_t(P) * 4, s, (by_a ? in.a : in.b).as<int32_t>(), n, P,
                     bounds.empty() ? nullptr : dbounds.as<int64_t>(), owner.as<uint32_t>(),
                     iota.as<int32_t>(), counts.as<unsigned long long>());
  OAP_HIP_CHECK(hipGetLastError());
  Soa send;
  send.alloc(ctx, n);
  if (n > 0) {
    Buffer okeys = ctx.alloc(size_t(n) * 4), perm = ctx.alloc(size_t(n) * 4);
    size_t tb = 0;
    const int obits = bits_for(std::max(P, 2));
    OAP_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tb, owner.as<uint32_t>(),
                                            okeys.as<uint32_t>(), iota.as<int32_t>(),
                                            perm.as<int32_t>(), size_t(n), 0, obits, s));
    {
      Buffer tmp = ctx.alloc(std::max<size_t>(tb, 16));
      OAP_HIP_CHECK(rocprim::radix_sort_pairs(tmp.data(), tb, owner.as<uint32_t>(),
                                              okeys.as<uint32_t>(), iota.as<int32_t>(),
                                              perm.as<int32_t>(), size_t(n), 0, obits, s));
    }
    hipLaunchKernelGGL(oap_als_gather3, dim3(grid_of(n)), dim3(kThreads), 0, s,
                       perm.as<int32_t>(), n, in.a.as<int32_t>(), in.b.as<int32_t>(),
                       in.r.as<float>(), send.a.as<int32_t>(), send.b.as<int32_t>(),
                       send.r.as<float>());
    OAP_HIP_CHECK(hipGetLastError());
  }
  in = Soa();
  // counts matrix (every rank's row of destinations), then the three column exchanges
  std::vector<int64_t> mine(P);
  ctx.copy_to_host(mine.data(), counts.data(), size_t(P) * 8, s);
  Buffer call = ctx.alloc(size_t(P) * P * 8);
  comm_allgather(ctx, comm, counts.data(), call.data(), size_t(P), DType::I64, s);
  std::vector<int64_t> all(size_t(P) * P);
  ctx.copy_to_host(all.data(), call.data(), all.size() * 8, s);
  std::vector<size_t> sc(P), rc(P);
  int64_t m = 0;
  for (int q = 0; q < P; ++q) {
    sc[q] = size_t(mine[q]);
    rc[q] = size_t(all[size_t(q) * P + me]);
    m += int64_t(rc[q]);
  }
  Soa recv;
  recv.alloc(ctx, m);
  comm_alltoallv(ctx, comm, send.a.data(), sc, recv.a.data(), rc, DType::I32, s);
  comm_alltoallv(ctx, comm, send.b.data(), sc, recv.b.data(), rc, DType::I32, s);
  comm_alltoallv(ctx, comm, send.r.data(), sc, recv.r.data(), rc, DType::F32, s);
  // integrity: the world's sent and received column checksums must agree
  Buffer ck = ctx.alloc(64);
  OAP_HIP_CHECK(hipMemsetAsync(ck.data(), 0, 64, s));
  const int cg = std::min(grid_of(std::max(n, m)), 1024);
  hipLaunchKernelGGL(oap_als_checksum, dim3(cg), dim3(kThreads), 0, s, send.a.as<int32_t>(),
                     send.b.as<int32_t>(), send.r.as<float>(), n, ck.as<unsigned long long>());
  hipLaunchKernelGGL(oap_als_checksum, dim3(cg), dim3(kThreads), 0, s, recv.a.as<int32_t>(),
                     recv.b.as<int32_t>(), recv.r.as<float>(), m, ck.as<unsigned long long>() + 3);
  OAP_HIP_CHECK(hipGetLastError());
  comm.wait(s);  // (the watchdog covers the exchange; send buffers are freed below)
  int64_t sums[6];
  ctx.copy_to_host(sums, ck.data(), sizeof(sums), s);
  comm_allreduce_host(ctx, comm, sums, 6, DType::I64, ReduceOp::Sum);
  if (!(sums[0] == sums[3] && sums[1] == sums[4] && sums[2] == sums[5]))
    OAP_THROW(CommError,
              "ALS device shuffle: checksum mismatch (ratings lost or corrupted in the exchange)");
  return recv;
}

// allgatherv of this rank's sorted distinct ids (device) in rank order -> host.
std::vector<int32_t> gather_ids(Context& ctx, Comm& comm, const Buffer& mine,
                                const std::vector<int64_t>& cnt, hipStream_t s) {
  const int P = comm.size(), me = comm.rank();
  int64_t mx = 1;
  for (int64_t c : cnt) mx = std::max(mx, c);
  Buffer send = ctx.alloc(size_t(mx) * 4), recv = ctx.alloc(size_t(mx) * P * 4);
  OAP_HIP_CHECK(hipMemsetAsync(send.data(), 0, size_t(mx) * 4, s));
  if (cnt[me] > 0)
    hipLaunchKernelGGL(oap_als_copy_i32, dim3(grid_of(cnt[me])), dim3(kThreads), 0, s,
                       mine.as<int32_t>(), cnt[me], send.as<int32_t>());
  comm_allgather(ctx, comm, send.data(), recv.data(), size_t(mx), DType::I32, s);
  std::vector<int32_t> all(size_t(mx) * P), out;
  ctx.copy_to_host(all.data(), recv.data(), all.size() * 4, s);
  int64_t total = 0;
  for (int64_t c : cnt) total += c;
  out.reserve(size_t(total));
  for (int q = 0; q < P; ++q)
    out.insert(out.end(), all.begin() + size_t(q) * mx, all.begin() + size_t(q) * mx + cnt[q]);
  return out;
}

}  // namespace

bool als_device_setup_dist(Context& ctx, Comm& comm, const int32_t* users, const int32_t* items,
                           const float* ratings, int64_t n, hipStream_t s, AlsDistSetup* out) {
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a) {
    return std::chrono::duration<double, std::milli>(clk::now() - a).count();
  };
  const int P = comm.size(), me = comm.rank();
  auto t0 = clk::now();
  Soa x;
  x.alloc(ctx, n);
  ctx.copy_to_backend(x.a.data(), users, size_t(n) * 4, s);
  ctx.copy_to_backend(x.b.data(), items, size_t(n) * 4, s);
  ctx.copy_to_backend(x.r.data(), ratings, size_t(n) * 4, s);
  // global id ranges and rating count: every rank takes the same device-or-host decision
  Buffer mmb = ctx.alloc(64);
  hipLaunchKernelGGL(oap_als_init_mm, dim3(1), dim3(1), 0, s, mmb.as<int>());
  if (n > 0)
    hipLaunchKernelGGL(oap_als_minmax, dim3(std::min(grid_of(n), 2048)), dim3(kThreads), 0, s,
                       x.a.as<int32_t>(), x.b.as<int32_t>(), n, mmb.as<int>());
  OAP_HIP_CHECK(hipGetLastError());
  int mm[4];
  ctx.copy_to_host(mm, mmb.data(), sizeof(mm), s);
  // [-umin, umax, -imin, imax, n] under one max-allreduce (n: a sum is not needed, the largest
  // local share bounds the 31-bit index space just as well as the total)
  double g[6] = {-double(mm[0]), double(mm[1]), -double(mm[2]), double(mm[3]), double(n), 0.0};
  comm_allreduce_host(ctx, comm, g, 5, DType::F64, ReduceOp::Max);
  const double ntot = comm_allreduce_scalar(ctx, comm, double(n), ReduceOp::Sum);
  out->upload_ms = ms(t0);
  if (ntot <= 0 || ntot >= double(int64_t(1) << 31)) return false;
  const int ulo = int(-g[0]), ilo = int(-g[2]);
  const int64_t urange = int64_t(g[1]) - ulo + 1, irange = int64_t(g[3]) - ilo + 1;
  const int64_t cap = std::max<int64_t>(8 * int64_t(ntot), int64_t(1) << 26);
  if (urange > cap || irange > cap || urange >= (int64_t(1) << 31) ||
      irange >= (int64_t(1) << 31))
    return false;  // rank-uniform: every input of this test was reduced over the world

  auto t1 = clk::now();
  double shuffle_ms = 0.0;
  auto timed_shuffle = [&](Soa& in, bool by_a, const std::vector<int64_t>& bounds) {
    auto ts = clk::now();
    Soa r = shuffle(ctx, comm, in, by_a, bounds, s);
    shuffle_ms += ms(ts);
    return r;
  };
  auto offsets = [&](int64_t mine_cnt, std::vector<int64_t>& cnt, std::vector<int64_t>& off) {
    cnt = comm_allgather_i64(ctx, comm, mine_cnt);
    off.assign(P + 1, 0);
    for (int q = 0; q < P; ++q) off[q + 1] = off[q] + cnt[q];
  };
  // ---- 1. ratings -> item owners (item mod P); dense item index of the owned items
  Soa r1 = timed_shuffle(x, false, {});
  Buffer irank, iids;
  std::vector<int32_t> my_items;
  const int64_t ni_loc =
      dense_index(ctx, r1.b.as<int32_t>(), r1.n, ilo, irange, s, irank, iids, my_items);
  offsets(ni_loc, out->icnt, out->ioff);
  const int64_t NI = out->ioff[P];
  if (r1.n > 0)  // b <- global item index
    hipLaunchKernelGGL(oap_als_to_index, dim3(grid_of(r1.n)), dim3(kThreads), 0, s,
                       r1.b.as<int32_t>(), r1.n, ilo, irank.as<int32_t>(), out->ioff[me]);
  irank = Buffer();
  // ---- 2. (user, global item, r) -> user owners; user CSR (cols = global item index)
  Soa r2 = timed_shuffle(r1, true, {});
  Buffer urank, uids;
  std::vector<int32_t> my_users;
  const int64_t nu_loc =
      dense_index(ctx, r2.a.as<int32_t>(), r2.n, ulo, urange, s, urank, uids, my_users);
  offsets(nu_loc, out->ucnt, out->uoff);
  const int64_t NU = out->uoff[P];
  const int ubits = bits_for(NU), ibits = bits_for(NI);
  OAP_CHECK(bits_for(nu_loc) + ibits <= 64 && bits_for(std::max<int64_t>(ni_loc, 1)) + ubits <= 64,
            "ALS device setup: index bits");
  {
    Buffer key = ctx.alloc(std::max<size_t>(size_t(r2.n) * 8, 16));
    Buffer cnt = ctx.alloc(size_t(nu_loc + 1) * 4);
    OAP_HIP_CHECK(hipMemsetAsync(cnt.data(), 0, size_t(nu_loc + 1) * 4, s));
    if (r2.n > 0)
      hipLaunchKernelGGL(oap_als_csr_keys, dim3(grid_of(r2.n)), dim3(kThreads), 0, s,
                         r2.a.as<int32_t>(), r2.b.as<int32_t>(), r2.n, urank.as<int32_t>(), ulo,
                         int64_t(0), ibits, key.as<uint64_t>(), cnt.as<int32_t>());
    OAP_HIP_CHECK(hipGetLastError());
    csr_from_keys(ctx, key, r2.r.as<float>(), r2.n, nu_loc, bits_for(nu_loc) + ibits, ibits, cnt,
                  s, out->users);
  }
  // a <- global user index; then (global item, global user, r) to the item slab owners
  if (r2.n > 0)
    hipLaunchKernelGGL(oap_als_to_index, dim3(grid_of(r2.n)), dim3(kThreads), 0, s,
                       r2.a.as<int32_t>(), r2.n, ulo, urank.as<int32_t>(), out->uoff[me]);
  urank = Buffer();
  std::swap(r2.a, r2.b);  // a = global item, b = global user
  // ---- 3. -> item slab owners; item CSR (rows = global item - ioff[me], cols = global user)
  Soa r3 = timed_shuffle(r2, true, out->ioff);
  {
    Buffer key = ctx.alloc(std::max<size_t>(size_t(r3.n) * 8, 16));
    Buffer cnt = ctx.alloc(size_t(ni_loc + 1) * 4);
    OAP_HIP_CHECK(hipMemsetAsync(cnt.data(), 0, size_t(ni_loc + 1) * 4, s));
    if (r3.n > 0)
      hipLaunchKernelGGL(oap_als_csr_keys, dim3(grid_of(r3.n)), dim3(kThreads), 0, s,
                         r3.a.as<int32_t>(), r3.b.as<int32_t>(), r3.n, nullptr, 0, out->ioff[me],
                         ubits, key.as<uint64_t>(), cnt.as<int32_t>());
    OAP_HIP_CHECK(hipGetLastError());
    csr_from_keys(ctx, key, r3.r.as<float>(), r3.n, ni_loc,
                  bits_for(std::max<int64_t>(ni_loc, 1)) + ubits, ubits, cnt, s, out->items);
  }
  // ---- global index -> id tables (rank order = global index order)
  out->user_ids = gather_ids(ctx, comm, uids, out->ucnt, s);
  out->item_ids = gather_ids(ctx, comm, iids, out->icnt, s);
  out->nnz = int64_t(
      comm_allreduce_scalar(ctx, comm, double(out->users.ptr_h.back()), ReduceOp::Sum));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  out->shuffle_ms = shuffle_ms;
  out->index_ms = ms(t1) - shuffle_ms;
  return true;
}

}  // namespace kern
}  // namespace oap
