// DenseTable: the rank-local partition of a dense row-major dataset, resident on the context's
// backend.  The MI355X-native replacement for the reference's per-partition oneDAL
// HomogenNumericTable + RowMergedNumericTable (mllib-dal/src/main/scala/org/apache/spark/ml/
// util/OneDAL.scala:92-166, native/OneDAL.cpp:50-76): ingestion is a chunked, double-buffered
// pinned-host -> HBM stream with the dtype conversion and zero padding done on the device,
// instead of one JNI call per row.
#pragma once

#include <cstdint>
#include <vector>

#include "comm/comm.h"
#include "runtime/context.h"

namespace oap {

struct DenseTable {
  int64_t rows = 0;  // local rows
  int cols = 0;      // features
  int64_t ld = 0;    // row stride in elements (>= cols, zero padded)
  DType dtype = DType::F32;
  Buffer data;
  Backend backend = Backend::CPU;
  int64_t global_offset = -1;  // global row index of local row 0 (-1 = not yet known)
  int64_t global_rows = -1;
  // (no per-table statistics are cached across fits: every fit pays for what it reads)

  size_t bytes() const { return size_t(rows) * size_t(ld) * dtype_size(dtype); }
};

// Host (numpy) rows -> backend-resident table.  src_t in {F32, F64}; storage in {F32, F64, BF16}
// (F64 only on the CPU backend).  chunk_rows bounds the pinned staging footprint.
DenseTable upload_dense(Context& ctx, const void* host, DType src_t, int64_t rows, int cols,
                        int64_t src_ld, DType storage, int64_t ld, int64_t chunk_rows = 1 << 18);

// Deterministic synthetic Gaussian blobs generated directly on the backend (rows
// [row0, row0+rows) of a global dataset; identical values for any sharding).  `storage` F32 or
// BF16 (GPU: the table's dtype; CPU: f64 storage of the same f32 / bf16-rounded values).
DenseTable synth_blobs_table(Context& ctx, int64_t rows, int cols, int64_t ld, int64_t row0,
                             int ncenters, double box, double sigma, uint64_t seed,
                             DType storage = DType::F32);

// Fills global_offset / global_rows with an allgather of local row counts.
void assign_global_offsets(Context& ctx, Comm& comm, DenseTable& t);

// Per-column max |x| over the GLOBAL dataset (local kernel + allreduce MAX), one pass per call.
std::vector<double> global_column_absmax(Context& ctx, Comm& comm, DenseTable& t);

// sum_i |x_i|^2 over the LOCAL rows in fp64 (exact squares, fixed summation order), one pass per
// call; *rel_err receives its rounding bound relative to the sum.  NaN when
// no kernel covers the table's layout (GPU f32 rows with ld % 4 == 0 and ld <= 1024 only).
double local_row_sqnorm(Context& ctx, DenseTable& t, double* rel_err);

// Copies rows [r0, r0+n) (first `cols` columns) back to host as float64.
std::vector<double> table_rows_f64(Context& ctx, const DenseTable& t, int64_t r0, int64_t n);

}  // namespace oap
