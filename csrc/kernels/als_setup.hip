// Device-side ALS setup: dense id re-indexing and both CSR matrices on the GPU (see
// kernels/als_setup.h).  Ids are re-indexed through a presence bitmap over [min, max] and an
// exclusive scan (rank = index among the distinct ids, ascending); each rating becomes one
// packed 64-bit key (row << cbits | col) per CSR and a stable LSD radix sort (rocPRIM) orders
// the ratings by (row, col) — row pointers come from a per-row count and a scan.  Every pass is
// a streaming pass over HBM: ~50 ms of device time per CSR at 1B ratings.
#include "kernels/als_setup.h"

#include <hip/hip_runtime.h>

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

__global__ void oap_als_minmax(const int32_t* __restrict__ u, const int32_t* __restrict__ it,
                               int64_t n, int* mm) {
  int umin = INT_MAX, umax = INT_MIN, imin = INT_MAX, imax = INT_MIN;
  for (int64_t k = blockIdx.x * int64_t(kThreads) + threadIdx.x; k < n;
       k += int64_t(gridDim.x) * kThreads) {
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
  for (int64_t k = blockIdx.x * int64_t(kThreads) + threadIdx.x; k < n;
       k += int64_t(gridDim.x) * kThreads)
    flag[ids[k] - lo] = 1;
}

__global__ void oap_als_compact_ids(const int32_t* __restrict__ flag,
                                    const int32_t* __restrict__ rank, int64_t range, int lo,
                                    int32_t* __restrict__ ids) {
  for (int64_t x = blockIdx.x * int64_t(kThreads) + threadIdx.x; x < range;
       x += int64_t(gridDim.x) * kThreads)
    if (flag[x]) ids[rank[x]] = int32_t(lo + x);
}

// packed keys of both CSRs and per-row counts
__global__ void oap_als_keys(const int32_t* __restrict__ u, const int32_t* __restrict__ it,
                             int64_t n, int ulo, int ilo, const int32_t* __restrict__ urank,
                             const int32_t* __restrict__ irank, int ubits, int ibits,
                             uint64_t* __restrict__ ku, uint64_t* __restrict__ ki,
                             int32_t* __restrict__ ucnt, int32_t* __restrict__ icnt) {
  for (int64_t k = blockIdx.x * int64_t(kThreads) + threadIdx.x; k < n;
       k += int64_t(gridDim.x) * kThreads) {
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
  for (int64_t k = blockIdx.x * int64_t(kThreads) + threadIdx.x; k < n;
       k += int64_t(gridDim.x) * kThreads)
    col[k] = int32_t(key[k] & m);
}

int bits_for(int64_t count) {  // bits to hold indices [0, count)
  int b = 1;
  while ((int64_t(1) << b) < count) ++b;
  return b;
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
  auto index = [&](const Buffer& ids, int lo, int64_t range, Buffer& rank,
                   std::vector<int32_t>& host_ids) {
    Buffer flag = ctx.alloc(size_t(range) * 4);
    rank = ctx.alloc(size_t(range) * 4);
    OAP_HIP_CHECK(hipMemsetAsync(flag.data(), 0, size_t(range) * 4, s));
    hipLaunchKernelGGL(oap_als_flag, dim3(grid_of(n)), dim3(kThreads), 0, s, ids.as<int32_t>(),
                       n, lo, flag.as<int32_t>());
    size_t tb = 0;
    OAP_HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, flag.as<int32_t>(), rank.as<int32_t>(),
                                          int32_t(0), size_t(range), rocprim::plus<int32_t>(),
                                          s));
    Buffer tmp = ctx.alloc(std::max<size_t>(tb, 16));
    OAP_HIP_CHECK(rocprim::exclusive_scan(tmp.data(), tb, flag.as<int32_t>(), rank.as<int32_t>(),
                                          int32_t(0), size_t(range), rocprim::plus<int32_t>(),
                                          s));
    int32_t last[2];
    ctx.copy_to_host(&last[0], rank.as<int32_t>() + range - 1, 4, s);
    ctx.copy_to_host(&last[1], flag.as<int32_t>() + range - 1, 4, s);
    const int64_t count = int64_t(last[0]) + last[1];
    Buffer idb = ctx.alloc(std::max<size_t>(size_t(count) * 4, 16));
    hipLaunchKernelGGL(oap_als_compact_ids, dim3(grid_of(range)), dim3(kThreads), 0, s,
                       flag.as<int32_t>(), rank.as<int32_t>(), range, lo, idb.as<int32_t>());
    OAP_HIP_CHECK(hipGetLastError());
    host_ids.resize(count);
    ctx.copy_to_host(host_ids.data(), idb.data(), size_t(count) * 4, s);
    return count;
  };
  Buffer urank, irank;
  const int64_t nu = index(du, mm[0], urange, urank, out->user_ids);
  const int64_t ni = index(di, mm[2], irange, irank, out->item_ids);
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
  auto build = [&](Buffer& keys, int64_t nrows, int rbits, int cbits, Buffer& cnt,
                   AlsDeviceCsr& csr) {
    csr.nrows = nrows;
    Buffer ksorted = ctx.alloc(size_t(n) * 8);
    csr.val = ctx.alloc(size_t(n) * 4);
    size_t tb = 0;
    OAP_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tb, keys.as<uint64_t>(),
                                            ksorted.as<uint64_t>(), dr.as<float>(),
                                            csr.val.as<float>(), size_t(n), 0, rbits + cbits, s));
    {
      Buffer tmp = ctx.alloc(std::max<size_t>(tb, 16));
      OAP_HIP_CHECK(rocprim::radix_sort_pairs(tmp.data(), tb, keys.as<uint64_t>(),
                                              ksorted.as<uint64_t>(), dr.as<float>(),
                                              csr.val.as<float>(), size_t(n), 0, rbits + cbits,
                                              s));
    }
    keys = Buffer();
    csr.col = ctx.alloc(size_t(n) * 4);
    hipLaunchKernelGGL(oap_als_key_cols, dim3(grid_of(n)), dim3(kThreads), 0, s,
                       ksorted.as<uint64_t>(), n, cbits, csr.col.as<int32_t>());
    OAP_HIP_CHECK(hipGetLastError());
    csr.ptr = ctx.alloc(size_t(nrows + 1) * 8);
    size_t sb = 0;
    OAP_HIP_CHECK(rocprim::exclusive_scan(nullptr, sb, cnt.as<int32_t>(), csr.ptr.as<int64_t>(),
                                          int64_t(0), size_t(nrows + 1),
                                          rocprim::plus<int64_t>(), s));
    {
      Buffer tmp = ctx.alloc(std::max<size_t>(sb, 16));
      OAP_HIP_CHECK(rocprim::exclusive_scan(tmp.data(), sb, cnt.as<int32_t>(),
                                            csr.ptr.as<int64_t>(), int64_t(0),
                                            size_t(nrows + 1), rocprim::plus<int64_t>(), s));
    }
    csr.ptr_h.resize(nrows + 1);
    ctx.copy_to_host(csr.ptr_h.data(), csr.ptr.data(), size_t(nrows + 1) * 8, s);
    OAP_CHECK(csr.ptr_h[nrows] == n, "als_device_setup: row pointer total");
  };
  build(ku, nu, ubits, ibits, ucnt, out->users);
  build(ki, ni, ibits, ubits, icnt, out->items);
  out->sort_ms = ms(t2);
  return true;
}

}  // namespace kern
}  // namespace oap
