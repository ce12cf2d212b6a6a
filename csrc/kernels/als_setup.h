// Device-side ALS setup (kernels/als_setup.hip): dense re-indexing of user / item ids and both
// CSR matrices built on the GPU (the reference's ratings shuffle + CSR build,
// mllib-dal/src/main/native/ALSShuffle.cpp:62-127, scala/.../ALSDALImpl.scala:184-230, which
// here ran on one host thread and took 24 s at 1B ratings).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "comm/comm.h"
#include "runtime/context.h"

namespace oap {
namespace kern {

struct AlsDeviceCsr {
  int64_t nrows = 0;
  Buffer ptr;                  // int64 [nrows + 1]
  Buffer col;                  // int32 [nnz]: dense index of the other side
  Buffer val;                  // float [nnz]
  std::vector<int64_t> ptr_h;  // host copy of ptr (row lists are planned on the host)
};

struct AlsDeviceSetup {
  std::vector<int32_t> user_ids, item_ids;  // sorted distinct ids (dense index order)
  AlsDeviceCsr users, items;                // rows = users (cols = items) / items (cols = users)
  double upload_ms = 0.0, index_ms = 0.0, sort_ms = 0.0;
};

// Single-rank setup of n ratings (host arrays).  Within a row the entries are ordered by the
// other side's index (radix sort, stable: duplicates keep their input order), so the result is
// deterministic.  Returns false (nothing built) when an id range is too sparse for the dense
// index (range > max(8 n, 2^26)): the caller falls back to the host setup.
bool als_device_setup(Context& ctx, const int32_t* users, const int32_t* items,
                      const float* ratings, int64_t n, hipStream_t s, AlsDeviceSetup* out);

// Multi-rank setup (any non-trivial comm; device buffers throughout).  Items are owned by
// id mod P, users likewise; each side's dense global index is rank-major (rank q's owned ids,
// ascending, at [off[q], off[q + 1])), exactly as the host setup in drivers/als.cpp orders them.
struct AlsDistSetup {
  std::vector<int64_t> ucnt, uoff, icnt, ioff;  // per-rank owned counts / global offsets
  std::vector<int32_t> user_ids, item_ids;      // global index -> id (all ranks)
  AlsDeviceCsr users, items;  // owned rows; cols = the other side's global index
  int64_t nnz = 0;            // global rating count
  double upload_ms = 0.0, shuffle_ms = 0.0, index_ms = 0.0;
};

// Collective: every rank of `comm` must call it.  Returns false on every rank (nothing built)
// when a global id range is too sparse for the dense index (the caller uses the host setup).
bool als_device_setup_dist(Context& ctx, Comm& comm, const int32_t* users, const int32_t* items,
                           const float* ratings, int64_t n, hipStream_t s, AlsDistSetup* out);

}  // namespace kern
}  // namespace oap
