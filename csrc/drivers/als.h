// Distributed implicit-feedback ALS driver.
//
// MI355X-native counterpart of the reference's ALS path: ratings shuffle (mllib-dal/src/main/
// native/ALSShuffle.cpp:62-127), CSR build (scala/.../ALSDALImpl.scala:184-230) and oneDAL's
// distributed implicit ALS (native/ALSDALImpl.cpp:216-438: 12 blocking collectives per
// iteration through a root).  Here:
//   * users and items are owned by rank id % P; a 3-step alltoallv gives every rank the CSR of
//     its owned users (columns = global item index) and of its owned items (columns = global
//     user index) — sparse and gapped IDs are handled by dense re-indexing;
//   * factor matrices are replicated ([n_users | n_items] x r_pad, fp32 in HBM);
//   * per half-iteration: Gramian of the owned source slice (MFMA SYRK) -> allreduce (r x r),
//     per-row normal equations + Cholesky (kernels/als.hip) for the owned destination rows,
//     then ONE allgather of the updated slices.
// Iteration order and solve semantics follow Spark's implicit ALS (ALS.scala:1036-1062,
// 1718-1800): items from users, then users from items.
#pragma once

#include <cstdint>
#include <vector>

#include "comm/comm.h"
#include "runtime/context.h"

namespace oap {

struct AlsParams {
  int rank = 10;
  int max_iter = 10;
  double reg = 0.1;
  double alpha = 1.0;
  bool implicit = true;
  uint64_t seed = 0;
  // optional initial user factors (resume from a checkpoint): ids sorted ascending,
  // factors [n_init][rank]; users not listed get the seeded random initialisation
  const int32_t* init_ids = nullptr;
  const float* init_factors = nullptr;
  int64_t n_init = 0;
  // fp64 host engine (thread pool, per-row Cholesky) even on a GPU context: the distributed
  // fallback for what the GPU kernels do not take (rank > kern::als_max_rank()); the ratings
  // stay sharded (same owner shuffle), only the factor slices are exchanged
  bool host_engine = false;
  // non-negative factors (Spark's nonnegative = true): NNLS per row, host engine
  bool nonnegative = false;
};

struct AlsResult {
  int rank = 0;
  std::vector<int32_t> user_ids, item_ids;      // global index order
  HostArray<float> user_factors, item_factors;    // [n][rank] row-major
  int64_t nnz = 0;                                // global ratings
  double setup_ms = 0.0, train_ms = 0.0;
  std::vector<double> iter_ms;                    // per iteration (both halves)
  double solve_ms = 0.0, gram_ms = 0.0, comm_ms = 0.0;  // summed device/host phase times
  // device comms: comm-stream time of the factor-chunk broadcasts (start -> end of each chunk's
  // grouped broadcast, summed) and the bytes every rank received through them
  double bcast_ms = 0.0;
  int64_t bcast_recv_bytes = 0;
  int64_t failed_rows = 0;                        // rows whose system was not SPD
  int64_t eig_unconverged = 0;  // Gramian eigensolves that stopped at max_sweeps (low-rank path)
};

// users/items/ratings: this rank's share of the ratings (any partition).
AlsResult als_fit(Context& ctx, Comm& comm, const int32_t* users, const int32_t* items,
                  const float* ratings, int64_t n, const AlsParams& p);

}  // namespace oap
