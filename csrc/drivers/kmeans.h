// Distributed K-Means driver (native Lloyd loop + k-means|| / random initialisation).
//
// MI355X-native counterpart of the reference's K-Means JNI driver
// (mllib-dal/src/main/native/KMeansDALImpl.cpp:34-249) and of the initialisation the reference
// leaves on Spark (spark-3.1.1/mllib/clustering/KMeans.scala:354-432).  Per iteration the
// reference does 4 blocking collectives through rank 0 (bcast length, bcast centroids,
// allgatherv partials, bcast converged — SURVEY.md §2.7 C2-C5); here each rank runs the fused
// assign kernel, ONE grouped allreduce of [fixed-point sums | counts] + cost, and the finalize
// kernel, and evaluates convergence redundantly — no root, no broadcast.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "comm/comm.h"
#include "runtime/context.h"
#include "runtime/table.h"

namespace oap {

enum class KMeansInit : int { Given = 0, Random = 1, Parallel = 2 };

struct KMeansParams {
  int k = 2;
  int max_iter = 20;
  double tol = 1e-4;
  KMeansInit init = KMeansInit::Parallel;
  int init_steps = 2;
  uint64_t seed = 1;
  // exact-fp32 MFMA distances only (default: bf16-split fast path + exact refinement, which
  // yields the same assignments)
  bool precise = false;
  // bound-based pruning of the distance work in Lloyd iterations after the first (GPU fast
  // path, d <= 128); exact: assignments, centers and costs are bitwise those without it
  bool prune = true;
  // with pruning on the single-launch path: iterations after the first keep the local
  // statistics and read only the rows of tiles whose labels may change (delta accumulation);
  // per-iteration costs are then computed only on full passes, the final cost by an exact
  // pass over the labels (cost_history holds NaN for the delta iterations before the last)
  bool delta = true;
  // per-iteration phase events (kmeans/assign_kernel and kmeans/allreduce metrics); off: one
  // event pair per batch of iterations (kmeans/iteration only), no event gaps between phases
  // (each record is a ~10 us gap in the stream, so the default is off)
  bool phase_events = false;
  // row-scan image passes: a sample of the rows (kern::kmeans_scan_decide) estimates the share
  // the Hamerly test would prune; below this share the pass runs dense (the pipelined image
  // kernel, ~15% faster than a scan pass that prunes nothing).  Result-neutral (either pass
  // writes every label and bound), so a local, per-rank choice.  0: always scan.
  double scan_min_prune = 0.2;
  // internal: the fixed-point bounds come from a column-maxima pass up front (set on the
  // restart after a failed provisional check, see kmeans.cpp fit_bounds)
  bool absmax_pass = false;
};

struct KMeansResult {
  std::vector<double> centers;  // k_eff x d, row-major
  int k = 0;                    // k_eff (may be < requested k when fewer distinct points)
  int d = 0;
  double cost = 0.0;            // cost of the last assignment step (Spark semantics)
  int num_iter = 0;
  bool converged = false;
  std::vector<double> cost_history;
  // per iteration: the largest center movement |c_new - c_old| (Euclidean) of that update
  std::vector<double> shift_history;
  std::vector<int64_t> last_counts;  // cluster sizes of the last assignment step
  double init_seconds = 0.0;
  double iter_seconds = 0.0;
  int64_t global_rows = 0;
  int64_t refine_tiles = 0;  // 32-row tiles re-decided by the exact pass (GPU fast path)
  int64_t tier3_tiles = 0;   // 32-row tiles whose tier-1 (one bf16 product) answer was unsure
  int64_t pruned_tiles = 0;  // 32-row tile passes whose distance work the bounds skipped
  int64_t deferred_rows = 0;  // rows the lean tier-1 pass left to the exact re-decision
  int64_t moved_rows = 0;     // rows the lean delta passes moved between clusters
  int64_t pruned_rows = 0;    // rows the row-level scan proved unchanged (summed over passes)
  int image_passes = 0;       // lean passes that took their operands from the fp16 row image
  int64_t image_bytes = 0;    // HBM of that image (0: not allocated)
  std::string assign_path = "cpu";  // the distance kernel path of the last iteration (GPU)
  // how a last assignment that computed no cost in its pass got one: "stats" (from the fit's
  // statistics, kmeans.cpp final_cost_from_stats), "rows" (a pass over the labels), "" (none
  // needed: the last pass computed it)
  std::string final_cost_path;
  // where the fixed-point column bounds came from: "centers" (provisional bounds from the
  // initial centers, verified by the first pass), "centers_checked" (verified by a column-maxima
  // pass after the first pass flagged a row), "absmax" (the column maxima), "restart" (the
  // provisional bounds failed: the fit was restarted with the column maxima)
  std::string scale_source;
};

// Initial centers (k_eff x d) for `params.init` in {Random, Parallel}.  Identical result for
// any world size / sharding (every random draw is keyed by the GLOBAL row index).
std::vector<double> kmeans_init_centers(Context& ctx, Comm& comm, DenseTable& x,
                                        const KMeansParams& params, int* k_eff);

// Full fit: init (unless params.init == Given, in which case init_centers is used) + Lloyd.
// Out-of-core fit (SURVEY.md §5 scale axis): the rank's rows stay in host memory (row-major
// f32, `rows` x `d`, page-locked for the duration when the driver allows) and every Lloyd
// iteration streams them through two HBM chunk buffers — pitched DMA of chunk c+1 on the H2D
// stream while chunk c is assigned and accumulated on the compute stream.  Given initial centers;
// the same fixed-point statistics as the resident fit, so the centers are bitwise equal to it.
KMeansResult kmeans_fit_streamed(Context& ctx, Comm& comm, const float* host, int64_t rows,
                                 int d, const std::vector<double>& init_centers,
                                 const KMeansParams& p, int64_t chunk_rows);

KMeansResult kmeans_fit(Context& ctx, Comm& comm, DenseTable& x,
                        const std::vector<double>& init_centers, const KMeansParams& params);

// Nearest-center labels and exact squared distances for the local rows (host outputs).
void kmeans_predict(Context& ctx, const DenseTable& x, const std::vector<double>& centers, int k,
                    int32_t* labels, double* dist2);

// Same on device-resident outputs (e.g. torch tensors): labels[rows] int32, dist2[rows] f32.
void kmeans_predict_device(Context& ctx, const DenseTable& x, const std::vector<double>& centers,
                           int k, int32_t* labels, float* dist2);

// Average device time (ms) of the fused assign kernel over `reps` launches with optional timing
// ablations (kern::KMeansAssignArgs::ablate) — the per-phase cost breakdown used for tuning.
double kmeans_assign_timing(Context& ctx, const DenseTable& x, const std::vector<double>& centers,
                            int k, int reps, bool precise, int ablate);
// Steady-state image-pass probe (see kmeans.cpp): ms of one delta pass over the fp16 operand
// image (lean kernel alone, and with the exact re-decision), its deferred / moved rows, and the
// resulting labels and statistics.  kernel: 0 kmeans_lloyd, 1 kmeans_lean_img (cfg, -1 default).
struct ImageTiming {
  double lean_ms = 0.0, pass_ms = 0.0;
  int64_t deferred_rows = 0, moved_rows = 0, image_passes = 0;
  std::vector<int32_t> labels;
  std::vector<uint64_t> stats;
  std::string path;
};
ImageTiming kmeans_image_timing(Context& ctx, const DenseTable& x,
                                const std::vector<double>& centers_a,
                                const std::vector<double>& centers_b, int k, int reps, int kernel,
                                int cfg, bool fallback);
// Workgroup shape of the lean tier-1 kernel (tuning; default from OAP_KMEANS_LEAN_VARIANT).
void kmeans_set_lean_variant(int v);
// Deferred rows per pass of the last lean-path timing (ablate bit 64).
double& last_timing_deferred();

// k-means++ over weighted candidates, then up to max_iter weighted Lloyd iterations (host,
// elementwise loops on `pool` when given; identical results for any pool size).
// Mirrors the semantics of Spark's LocalKMeans.kMeansPlusPlus (RNG stream is our own).
std::vector<double> local_kmeans_pp(const std::vector<double>& pts, const std::vector<double>& w,
                                    int d, int k, int max_iter, uint64_t seed,
                                    ThreadPool* pool = nullptr);

}  // namespace oap
