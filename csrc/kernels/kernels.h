// Host-side launch API for every hand-written CDNA4 (gfx950) kernel.  Kernel names are chosen
// to be greppable in `rocprofv3 --kernel-trace` output (prefix "oap_").
#pragma once

#include <cstdint>

#include "runtime/common.h"

namespace oap {
namespace kern {

// ----------------------------------------------------------------------------- data layout
// Row stride (elements) of the dense tables the K-Means kernels read (16-byte rows, zero padded:
// a multiple of 4 for f32, of 8 for bf16) and the padded feature count of the centroid layout
// (multiple of 16 when d <= 128).
int kmeans_ld(int d, bool bf16 = false);
int kmeans_dp(int d);
// Dense ingestion: src rows (f64 or f32, row stride src_ld) -> dst rows (f32 / bf16 / f64, row
// stride dst_ld, zero padded).  Both pointers are device pointers.
void convert_pad(const void* src, DType src_t, int64_t rows, int cols, int64_t src_ld, void* dst,
                 DType dst_t, int64_t dst_ld, hipStream_t s);
// Per-column max |x| over rows (atomicMax on the float bit pattern), out[cols] must be zeroed.
// x is f32 or bf16 (t).
void column_absmax(const void* x, DType t, int64_t rows, int cols, int64_t ld, float* out,
                   hipStream_t s);
// sum_i |x_i|^2 of f32 rows [rows][ld] (first `cols` columns) as kSqnormBlocks fp64 partials
// (deterministic; the caller sums them in order).  Returns the partial count, or -1 when the
// layout is not supported (ld % 4 != 0, ld > 1024, rows not 16-byte aligned) or rows == 0.
constexpr int kSqnormBlocks = 2048;
int row_sqnorm_partials(const float* x, int64_t rows, int cols, int64_t ld, double* part,
                        hipStream_t s);
// Deterministic synthetic Gaussian blobs (hash RNG): rows [row0, row0+rows) of a global dataset,
// x = center[label] + sigma * N(0,1) with centers uniform in [-box, box]^cols, stored as f32 or
// bf16 (t; bf16 = the f32 value rounded to nearest even).
void synth_blobs(void* x, DType t, int64_t rows, int cols, int64_t ld, int64_t row0, int ncenters,
                 float box, float sigma, uint64_t seed, hipStream_t s);

// Deterministic float sum: per-block partials into slab (returns #partials, <= 256).
int reduce_sum_f32(const float* v, int64_t n, double* slab, hipStream_t s);
// Sums in[0..m) in a fixed order into out[0].
void sum_f64(const double* in, int m, double* out, hipStream_t s);
// out[i][0..cols) = x[idx[i]][0..cols)   (x f32 or bf16)
void gather_rows(const void* x, DType t, int64_t ld, int cols, const int64_t* idx, int64_t m,
                 float* out, hipStream_t s);
// Appends i to out_idx for every flag[i] != 0 (unordered; *counter zeroed by the caller).
void compact_flags(const int32_t* flag, int64_t n, int64_t* out_idx, unsigned long long* counter,
                   hipStream_t s);
void elementwise_min(float* acc, const float* v, int64_t n, hipStream_t s);
// flag[i] = u(seed, step, row0+i) < factor * cost[i]   (u ~ U[0,1), keyed by global row)
void bernoulli_select(const float* cost, int64_t n, int64_t row0, double factor, uint64_t seed,
                      int step, int32_t* flag, hipStream_t s);

// ----------------------------------------------------------------------------- K-Means
struct KMeansAssignArgs {
  const void* x = nullptr;  // [n][ld] f32 or bf16 (xbf16), ld = kmeans_ld(d, xbf16)
  bool xbf16 = false;
  int64_t n = 0;
  int ld = 0;
  int d = 0;
  const float* centers = nullptr;  // [kpad][dp] f32, zero padded (kmeans_prepare_centers)
  const float* cnorm = nullptr;    // [kpad] f32 |c|^2, +inf for j >= k
  const float* cstat = nullptr;    // [1]: max_j |c_j| (bf16x3 refinement threshold)
  int k = 0;
  int kpad = 0;  // multiple of 32
  int base = 0;  // global index of centers[0] (chunked launches)
  const float* scale = nullptr;          // [d] fixed-point scales (powers of two)
  unsigned long long* sums = nullptr;    // [k][d] int64 fixed point (accumulate)
  unsigned long long* counts = nullptr;  // [k]
  double* cost_slab = nullptr;           // [grid] per-block cost (deterministic)
  int32_t* labels = nullptr;             // optional [n]
  float* mindist = nullptr;              // optional [n] exact |x - c_best|^2
  bool accumulate = true;                // counts (+ sums when sums_too)
  bool sums_too = true;
  bool precise = false;                  // exact-fp32 MFMA only (no bf16x3 fast path)
  bool merge = false;                    // keep labels/mindist from earlier chunks unless beaten
  // optional [2]: tiles that took the exact pass, tiles that took the 3-product tier (fast1)
  unsigned long long* refine_tiles = nullptr;
  bool fast1 = false;  // start at the 1-product tier (see kmeans_assign.hip)
  int ablate = 0;  // timing ablations only: 1 no accumulate, 2 no cost, 8 no distance work,
                   // 16 prefetch two tiles ahead instead of one, 32 no tier-1 first pass
  // Bound-based pruning (fast path, d <= 128; see kmeans_assign.hip "Pruning").  bounds [n]:
  // single launch: {upper bound on |x - c_label|, lower bound on the distance to every other
  // center}; chunked (merge) passes: {running lower bound (squared) on the non-best candidates,
  // row-skippable flag/lower bound written by the seed pass}.  drift / drift_max (set only when
  // bounds and labels hold the previous iteration's values): per-center movement of the fp32
  // centers since then (global index) and its maximum.
  float* bounds = nullptr;  // float2 pairs
  const float* drift = nullptr;
  const float* drift_max = nullptr;
  // optional counter of 32-row tiles whose distance work the bounds skipped
  unsigned long long* pruned_tiles = nullptr;
  // chunked passes after a pruning seed: the seed appends every tile holding a row that may
  // change its label to tile_list (count in *tile_count, zeroed before the seed); the passes
  // then visit only those tiles, so pruned tiles cost no row reads at all
  int32_t* tile_list = nullptr;
  unsigned* tile_count = nullptr;
  // merge passes: a tile holding a row whose pick inside this chunk is a near tie that could
  // still win is not escalated here but appended to defer_list; the driver re-runs the chunk on
  // those tiles after the last chunk, when the row's best-so-far usually rules the chunk out.
  // Segmented per workgroup: [grid][kmeans_defer_segment(n)] tiles, defer_count [grid] (zeroed);
  // the re-run passes the same arrays as tile_list / tile_count with seg_list set.
  int32_t* defer_list = nullptr;
  unsigned* defer_count = nullptr;
  bool seg_list = false;
  bool fresh_bound = true;  // merge + bounds: this pass starts the row's running bound afresh
  // Delta accumulation (single launch, Lloyd iterations > 0, with tile_list from
  // kmeans_prune_scan): sums / counts hold the previous iteration's local statistics and only
  // rows whose label changes add +x to the new and -x to the old cluster (fixed point: exactly
  // the full recount).  Pruned tiles are never read.
  bool delta = false;
  // optional [ceil(n/32)]: per 32-row tile, the largest |x|^2 as the assign kernel computes it
  // (the scan's pruning margin)
  float* xnorm = nullptr;
  // Row-list (refine) mode of the general kernel: the rows to process are the entries of this
  // workgroup's segment of row_list ([grid][row_seg_cap], count row_count[blockIdx.x]), taken 32
  // at a time — the rows the lean tier-1 kernel deferred.  No pruning test; delta reads each
  // row's previous label.
  const int32_t* row_list = nullptr;
  const unsigned* row_count = nullptr;  // [grid][16]: rows per sub-segment
  // Row-scan image pass (kmeans_lean_img, fused): the kernel applies the row scan's Hamerly test
  // to every row itself and runs only the rows it cannot prune.  img_scan_xnorm: per-tile max
  // |x|^2 (set: the fused scan is on); img_scan_drift: the centers' drift [k] and its maximum at
  // [k]; img_scan_pruned (optional): counter of pruned rows.
  const float* img_scan_xnorm = nullptr;
  const float* img_scan_drift = nullptr;
  unsigned long long* img_scan_pruned = nullptr;
  int64_t row_seg_cap = 0;
  int row_subs = 1;  // sub-segments per workgroup segment (each row_seg_cap / row_subs long)
  // Lean tier-1 kernel output: rows whose tier-1 top-2 gap is inside the tier's error bound are
  // appended to this workgroup's segment ([grid][row_seg_cap], count defer_row_count[block]).
  int32_t* defer_rows = nullptr;
  unsigned* defer_row_count = nullptr;
  // optional counters [deferred rows, moved rows staged by delta passes, passes that read the
  // operand image] (3 entries)
  unsigned long long* deferred_rows = nullptr;
  // Row-list (refine) mode: rows still unsure after the bf16x3 tier are appended to
  // exact_rows ([grid][8][exact_sub_cap], one sub-segment per wave, counts exact_count
  // [grid][8]) instead of re-deciding their whole 32-row group; kmeans_exact_rows finishes them.
  int32_t* exact_rows = nullptr;
  unsigned* exact_count = nullptr;
  int64_t exact_sub_cap = 0;
  // Centroid-chunked lean pass (kmeans_lloyd / kmeans_exact_rows, k too large for one LDS plan,
  // k <= 1024): a launch sees centers / cnorm / k / kpad of ONE chunk whose first center has
  // global index `base`.  chunk_mode 1 = first, 2 = middle chunk (only the running state is
  // written), 3 = last chunk (the outputs), 0 = not chunked.  lean_keys: the lean kernel's
  // running top-2 keys per row ([n][2]); xstate: the exact kernel's running (best, index) per
  // deferral-list slot ([grid * row_seg_cap][2]; no bounds in this mode); centers_all / kglob:
  // every center (the chosen center's exact cost) and the global k.
  int chunk_mode = 0;
  int kglob = 0;
  int32_t* lean_keys = nullptr;
  float* xstate = nullptr;
  // Resident fp16 operand image of f32 rows (lean kernel, single launch): row-major
  // [32 ceil(n/32)][16 KS] halves (kmeans_lloyd_image_bytes), the MFMA B operand of each row
  // with its bias slots, at the scale *img_beta.  img_mode 1: this full pass writes image and
  // scale; 2: this pass takes its operands from the image (f32 rows only for accumulation).
  void* ximg = nullptr;
  float* img_beta = nullptr;
  int img_mode = 0;
  const float* centers_all = nullptr;
  // Lean kernel, full passes over the f32 / bf16 rows (kmeans_lloyd): sq_slab [grid] receives
  // each workgroup's sum of its rows' fp32 |x|^2, summed in fp64 (the final cost's
  // sum_i |x_i|^2, fused into the fit's first pass); bound_flag (optional) gets 1 or'ed in when
  // a row has a value |x_f| >= bound_inf — the fit's provisional fixed-point bounds may not hold
  // — and bound_flag[1] receives the largest fp32 |x|^2 of the rows (float bits, atomicMax).
  double* sq_slab = nullptr;
  unsigned* bound_flag = nullptr;
  float bound_inf = 0.f;
  // Batched fits with a tolerance: a device word the finalize sets once the fit has converged;
  // the lean / image / exact / scan kernels of later iterations in the batch return at once.
  const int* halt = nullptr;
  // Image pass gate (kmeans_lean_img): the pass runs only when *img_gate == img_gate_on — a
  // row-scan pass (1) and a dense pass (0) are both enqueued and kmeans_scan_decide picks one on
  // the device.  Either writes every row's label and bounds, so the choice changes no result.
  const int* img_gate = nullptr;
  int img_gate_on = 0;
};
// Lean tier-1 Lloyd kernel (kmeans_lloyd.hip): applicable when the centroid hi plane + the
// fixed-point accumulator fit LDS and d + 4 bias features fit the padded width.
bool kmeans_lloyd_supported(int d, int k, bool accumulate, bool sums_too);
int kmeans_lloyd_grid(int64_t n, int num_cus);
// Waves per workgroup of a lean-kernel variant; per-workgroup capacity of its deferral list
// (rows; `waves` sub-segments of seg_cap / waves each, counts [grid][16]).
int kmeans_lloyd_waves(int variant);
int64_t kmeans_lloyd_seg_cap(int64_t n, int grid, int waves);
// One pass: rows whose tier-1 answer is sure are finished (labels / mindist / bounds / cost /
// fixed-point statistics, delta mode over tile_list); the others go to a.defer_rows.  variant
// selects the workgroup shape (6: 16 waves, 8: 12 waves).  Writes `grid` cost partials.
int kmeans_lloyd(const KMeansAssignArgs& a, int grid, int variant, hipStream_t s);
// Bytes of the lean kernel's fp16 operand image of n f32 rows of width d (0: not applicable).
size_t kmeans_lloyd_image_bytes(int64_t n, int d);
// Steady-state image pass (kmeans_lean_img.hip): the delta Lloyd pass over the resident fp16
// operand image as its own compile-time-specialised kernel (same outputs as kmeans_lloyd with
// img_mode 2).  `waves` must be the lean variant's (kmeans_lloyd_waves: the deferral
// sub-segments), cfg < 0 the default configuration.  When the image's scale cannot hold the
// current centers the kernel does nothing; kmeans_lloyd with img_mode 3 then runs the pass.
// the refined tier-1 deferral test of the image passes (kmeans_frag.h refined_tt): on unless
// OAP_KMEANS_REFINE=0 (timing A/B; labels and statistics are the same either way)
bool kmeans_refine_default();
bool kmeans_lean_img_supported(int d, int k, int waves, bool scan = false);
void kmeans_lean_img(const KMeansAssignArgs& a, int grid, int waves, int cfg, hipStream_t s);
// The scan-vs-dense choice of a row-scan image pass, on the device: the row scan's own Hamerly
// test on an even sample of the rows (bounds, labels, the drift the last finalize wrote); *gate
// = 1 (scan) when at least min_frac of the sample is prunable, else 0 (the dense pipelined pass,
// cheaper when few rows prune).  gate: [4] ints, gate[2..3] zero before the first call (the
// kernel's scratch).  Returns at once when *halt is set.
void kmeans_scan_decide(int64_t n, int k, int d, const float* bounds, const int32_t* labels,
                        const float* xnorm, const float* drift, const float* cstat,
                        float min_frac, int* gate, const int* halt, hipStream_t s);
// Largest centroid chunks (multiples of 32) of the chunked lean pass at dimension d: the lean
// kernel's fp16 plane and the exact kernel's fp32 centers (0: d not supported).
int kmeans_lloyd_chunk_kmax(int d);
int kmeans_exact_chunk_kmax(int d);
// The general fused kernel over the rows kmeans_lloyd deferred (a.row_list / row_count /
// row_seg_cap from its defer outputs), on the same `grid`.
void kmeans_assign_rows(const KMeansAssignArgs& a, int grid, hipStream_t s);
// Exact fp32 re-decision of the rows kmeans_lloyd deferred (a.row_list / row_count /
// row_seg_cap / row_subs = its defer outputs, same `grid`): one wave per row, the centers in
// LDS, every candidate's distance on the VALU in the exact MFMA kernel's arithmetic (bitwise its
// answer), then the row's cost, outputs and fixed-point statistics (global atomics).  Writes
// `grid` cost partials.
void kmeans_exact_rows(const KMeansAssignArgs& a, int grid, hipStream_t s);
// Tiles per lean workgroup (each owns a contiguous range).
int64_t kmeans_lloyd_tiles_per_block(int64_t n, int grid);
// Delta-mode pruning scan in the lean layout: tile_list [lean_grid][tiles_per_block] segments,
// tile_count [lean_grid] (zeroed here); otherwise as kmeans_prune_scan.
void kmeans_lean_scan(int64_t n, int k, int d, int lean_grid, float* bounds,
                      const int32_t* labels, const float* xnorm, const float* drift,
                      const float* drift_max, const float* cstat, int32_t* tile_list,
                      unsigned* tile_count, unsigned long long* pruned, hipStream_t s,
                      const int* halt = nullptr);

// Delta-mode pruning scan (single launch): per 32-row tile, tests every row's bounds (labels,
// xnorm, the centers' drift) exactly as the assign kernel's own pruning test does.  Tiles that
// provably keep all labels get their bounds advanced in place (u + drift, l - max drift, rounded
// outward) and are counted in *pruned; the others are appended to tile_list (*tile_count must be
// zero on entry).  Reads 12 bytes per row (+4 per tile) and no row data.
void kmeans_prune_scan(int64_t n, int k, int d, float* bounds, const int32_t* labels,
                       const float* xnorm, const float* drift, const float* drift_max,
                       const float* cstat, int32_t* tile_list, unsigned* tile_count,
                       unsigned long long* pruned, hipStream_t s);
// Upper bound on rows one assign workgroup processes for n local rows (device independent); the
// fixed-point scale keeps per-workgroup LDS partial sums below 2^53 with it.
int64_t kmeans_rows_per_block_bound(int64_t n);
// Largest centroid count one launch can hold in LDS for d features (0 => generic kernel).
int kmeans_lds_kmax(int d, bool precise);
// Returns the number of blocks used (== entries written to cost_slab).
int kmeans_assign(const KMeansAssignArgs& a, int num_cus, hipStream_t s);
// Chunked path (d <= 128): mindist[i] = |x_i - centers[labels[i]]|^2, bitwise as the assign
// kernel computes it, so later merge passes can skip chunks that cannot beat it.
void kmeans_seed_mindist(const KMeansAssignArgs& a, hipStream_t s);
// Exact cost of an assignment: sum_i |x_i - centers[labels[i]]|^2 with the assign kernel's
// per-row fp32 arithmetic, centers staged in LDS.  Writes at most max_blocks fp64 partials to
// slab and returns their number, or -1 when the centers do not fit LDS.
int kmeans_label_cost(const KMeansAssignArgs& a, double* slab, int max_blocks, hipStream_t s);
// *pruned += (ntiles - *listed) * passes (device side: no host round trip)
void kmeans_count_pruned(const unsigned* listed, int64_t ntiles, int passes,
                         unsigned long long* pruned, hipStream_t s);
int kmeans_cost_slab_size(int num_cus);
// Deferral list layout of one merge pass over n rows: workgroups x per-workgroup capacity.
void kmeans_defer_layout(int64_t n, int num_cus, int* grid, int64_t* seg_cap);
// sums/counts += rows grouped by labels (fixed point; used after chunked assignment).  Cluster
// ranges are owned by workgroup groups that each keep their slice of the sums in LDS, so every
// row element costs one LDS atomic instead of a global one (sums == nullptr: counts only).
void kmeans_accumulate(const void* x, bool xbf16, int64_t n, int ld, int d,
                       const int32_t* labels, int k, const float* scale,
                       unsigned long long* sums, unsigned long long* counts, hipStream_t s);

// Same result via rows binned by cluster range first (every accumulation lane works on a row
// of its range).  scratch: kmeans_bin_scratch_bytes(n, k).  Returns false (nothing launched)
// when the layout does not apply; the caller then uses kmeans_accumulate.
size_t kmeans_bin_scratch_bytes(int64_t n, int k);
// Delta accumulation of the rows whose label changed (old -> new): +x into the new cluster, -x
// into the old one (fixed point: exactly the full recount's change).  *entries = entries it
// needed (2 per moved row); returns false (nothing accumulated, the caller recounts) when they
// exceed the scratch's capacity.  Synchronizes `s` once (reads that count).
bool kmeans_accumulate_moved(const void* x, bool xbf16, int64_t n, int ld, int d,
                             const int32_t* old_labels, const int32_t* new_labels, int k,
                             const float* scale, unsigned long long* sums,
                             unsigned long long* counts, void* scratch, size_t scratch_bytes,
                             int64_t* entries, hipStream_t s);
bool kmeans_accumulate_binned(const void* x, bool xbf16, int64_t n, int ld, int d,
                              const int32_t* labels, int k, const float* scale,
                              unsigned long long* sums, unsigned long long* counts, void* scratch,
                              hipStream_t s);

struct KMeansFinalizeArgs {
  const unsigned long long* sums = nullptr;  // global (allreduced) fixed-point sums [k][d]
  const unsigned long long* counts = nullptr;
  const double* inv_scale = nullptr;  // [d]
  double* centers64 = nullptr;        // [k][d] in/out (empty clusters keep their center)
  float* centers32 = nullptr;         // [kpad][dp] out (padded layout)
  float* cnorm = nullptr;             // [kpad] out (entries >= k untouched)
  float* cstat = nullptr;             // [1] out: max |c|
  int k = 0;
  int d = 0;
  int dp = 0;
  double tol = 0.0;
  const double* cost_in = nullptr;  // allreduced cost (1 value)
  void* flags = nullptr;            // KMeansFlags out
  double* scratch = nullptr;        // [2k]: enables the multi-block finalize (else 1 block)
  // optional [k + 1] out: |centers32_new - centers32_old| per center (rounded up), [k] = max
  float* drift = nullptr;
  // multi-block finalize in ONE launch: the last cluster block to finish (this zero-initialised
  // counter, reset by it) reduces the flags — no second kernel
  unsigned* done = nullptr;
  // optional: zeroed once its value is in the flags (the next iteration's cost accumulator)
  double* cost_reset = nullptr;
  // optional (batched fits, tol >= 0): the finalize returns at once when *halt is set and sets it
  // when this iteration converged, so the iterations enqueued behind it change nothing
  int* halt = nullptr;
};
// dst = src (bytes, a multiple of 4) unless *halt is set (halt may be null).
void copy_guarded(void* dst, const void* src, size_t bytes, const int* halt, hipStream_t s);
// The adaptive controls of a K-Means batch (kmeans_fit), on the device so that they ride the
// batch's last grouped allreduce (Max over ranks) instead of scalar host round trips:
// out[0] = the share of re-decisions (tier-3 tile re-runs of the general kernel / deferred rows
// of the lean kernel) over the batch against their budgets, out[1] = -(pruned tile share of the
// batch's scan passes), out[2] = moved rows / rows, out[3] = the provisional bound flag, out[4] =
// sqrt of the largest fp32 |x|^2 (rounded up).  snap[3] holds the counters at the batch start
// (updated here).  Null counters count as 0.
struct KMeansCtlArgs {
  const unsigned long long* refine = nullptr;   // [1] = tier-3 tile re-runs
  const unsigned long long* ldstat = nullptr;   // [0] deferred rows, [1] moved rows
  const unsigned long long* pruned = nullptr;   // tiles pruned by the tile scan
  const unsigned* bound_flag = nullptr;         // [flag, largest |x|^2 bits]
  unsigned long long* snap = nullptr;           // [3] in/out
  double* out = nullptr;                        // [5]
  int64_t rows = 0;
  int nb_it = 1;
  int scan_iters = 0;
  int scan_local = 0;  // this rank runs the tile scan (else its pruned share counts as 1)
};
void kmeans_ctl(const KMeansCtlArgs& a, hipStream_t s);
struct KMeansFlags {
  int converged;
  int nonempty;
  double cost;
  double max_shift2;
};
void kmeans_finalize(const KMeansFinalizeArgs& a, hipStream_t s);
// centers32 (padded [kpad][dp]) = (float)centers64, cnorm = |c|^2 (+inf for j in [k, kpad)),
// cstat[0] = max |c|.
void kmeans_prepare_centers(const double* centers64, int k, int d, int dp, float* centers32,
                            float* cnorm, float* cstat, int kpad, hipStream_t s);

// ---- PCA (kernels/pca.hip) ------------------------------------------------------------------
struct PcaPlan {
  int tw = 128;    // output tile width (128 or 256)
  int nb = 0;      // tw-feature blocks
  int tiles = 0;   // upper-triangular 128x128 tiles
  int splits = 0;  // row splits (one fp64 slab each)
  int64_t rows_per_split = 0;
  size_t part_elems = 0, cpart_elems = 0, shift_elems = 0;
  int grid = 0;
};
PcaPlan pca_syrk_plan(int64_t n, int d, int num_cus);
// part/cpart: fp64 slabs of p.part_elems / p.cpart_elems; shift: [p.shift_elems] zero padded.
void pca_syrk(const float* x, int64_t n, int64_t ld, int d, const float* shift, const PcaPlan& p,
              double* part, double* cpart, bool four, int flush_rows, hipStream_t s);
// Exact (reference-precision) statistics: fp64 products and sums on v_mfma_f64_16x16x4_f64 of
// f32 or f64 rows (x_f64), 128-wide tiles; shift: fp64 [p.shift_elems] zero padded.  The slabs
// reduce with pca_reduce like the fast path's.
PcaPlan pca_syrk_plan_f64(int64_t n, int d, int num_cus);
void pca_syrk_f64(const void* x, bool x_f64, int64_t n, int64_t ld, int d, const double* shift,
                  const PcaPlan& p, double* part, double* cpart, hipStream_t s);
// Exact statistics of f32 rows on the int8 matrix cores (kernels/pca_ozaki.hip): 7 base-128
// digits per centred element, 28 digit products per product, exact int32 sums; the fp64 result
// differs from the exact S by at most n 2^(E_j + E_k - 49) (8.05 + fp64 rounding) per entry.
struct PcaOzakiPlan {
  int64_t n = 0;
  int d = 0, dp = 0, nb = 0, tiles = 0, splits = 0;
  int64_t nrb = 0, groups = 0, chunk_rb = 0, chunks = 0, cgroups = 0;
  int split_group = 1;  // the reduce sums the splits in groups of this many
  int fp64_adds = 0;    // longest chain of fp64 additions into one output (error bound)
  size_t slab_elems = 0;
  size_t off_slab = 0, off_mm = 0, off_e = 0, off_sc = 0, off_shift = 0, off_cpart = 0;
  size_t ws_bytes = 0;  // one device workspace (digit planes of one row chunk first)
};
// max_plane_bytes bounds the digit planes of one row chunk (7 d_pad bytes per row)
PcaOzakiPlan pca_ozaki_plan(int64_t n, int d, int num_cus, size_t max_plane_bytes);
// out: d x d S (both triangles), colsum: [d]; shift_host: fp64 [d] (read before the call
// returns); bound (device, 1 double): the bound on max |S - S_exact| over the entries, negative
// when the column scales taken from a row sample (exact_scales false, > 65536 rows) proved too
// small — then call again with exact_scales
void pca_syrk_ozaki(const float* x, int64_t ld, const double* shift_host, const PcaOzakiPlan& p,
                    void* ws, double* out, double* colsum, double* bound, bool exact_scales,
                    hipStream_t s);
// ---- ALS (kernels/als.hip) -------------------------------------------------------------------
struct AlsSolveArgs {
  const int64_t* rowptr = nullptr;  // [nrows+1] CSR of the destination rows
  const int32_t* cols = nullptr;    // source-row indices into src
  const float* vals = nullptr;      // ratings
  // rows with at most the long-row threshold of ratings, solved directly
  const int32_t* short_rows = nullptr;
  int64_t n_short = 0;
  // long rows: their ratings are split into chunks (partial Gramians, summed in chunk order)
  const int32_t* long_rows = nullptr;
  int64_t n_long = 0;
  const int64_t* long_chunk_ptr = nullptr;  // [n_long+1] chunk ranges per long row
  const int64_t* chunk_begin = nullptr;     // [n_chunks] rating ranges
  const int64_t* chunk_end = nullptr;
  int64_t n_chunks = 0;
  float* partials = nullptr;                // [n_chunks][als_partial_floats(r)]
  // long-row chunks: split-fp16 Gramian scaled from [max |rating|, max |source factor|]
  // (device, float bits, als_absmax); null: exact-fp32 MFMA products
  const unsigned* absmax = nullptr;
  // direct rows (short_rows by decreasing length): the first n_direct_x3 take the split-fp16
  // Gramian, the rest the fp32 one (-1: all split-fp16 when absmax is set)
  int64_t n_direct_x3 = -1;
  const float* src = nullptr;       // source factors [n_src][ld]
  int ld = 0, r = 0;
  const float* yty = nullptr;       // [r][r] Gramian of ALL source factors (implicit)
  float alpha = 1.f, lambda = 0.f;
  bool implicit = true;
  float* dst = nullptr;             // [nrows][ld], indexed by destination row
  unsigned long long* queue = nullptr;  // device scratch: 8 counters ([2] is the driver's fail)
  unsigned long long* fail = nullptr;   // device counter of non-SPD rows
  // Low-rank (Woodbury) path for implicit rows with <= als_lowrank_max_len() ratings
  // (kernels/als_lowrank.hip): short_rows[lr_off[0], lr_off[4]) are those rows by decreasing
  // length, [lr_off[j], lr_off[j+1]) holding 16 (3 - j) + 1 .. 16 (4 - j) ratings; the direct
  // kernel solves short_rows[0, lr_off[0]).  lr_off[0] = n_short disables the path.
  int64_t lr_off[5] = {0, 0, 0, 0, 0};
  const float* lr_src = nullptr;   // source factors in the eigenbasis of Y^T Y: [n_src][ld]
  const float* lr_eig = nullptr;   // [ld] eigenvalues of Y^T Y (padding 1)
  const float* lr_back = nullptr;  // [ld][ld] Q^T (row vectors x^T = x_q^T Q^T)
  float* lr_scratch = nullptr;     // [lr_off[4] - lr_off[0]][ld]
};
size_t als_partial_floats(int r);
int als_max_rank();
void als_solve(const AlsSolveArgs& a, int num_cus, hipStream_t s);
int als_lowrank_max_len();
void als_solve_lowrank(const AlsSolveArgs& a, int num_cus, hipStream_t s);
// out[out_rows ? out_rows[i] : i] = in[in_rows ? in_rows[i] : i] R for n rows (R: ld x ld)
void als_rotate(const float* in, const int32_t* in_rows, float* out, const int32_t* out_rows,
                int64_t n, const float* R, int ld, int num_cus, hipStream_t s);
void als_init_factors(const int32_t* ids, int64_t n, int r, int ld, uint64_t seed, float* out,
                      hipStream_t s);
void f64_to_f32(const double* in, float* out, int64_t n, hipStream_t s);
// *out = max(*out, max |x_i|) as float bits (caller zeroes *out first)
void als_absmax(const float* x, int64_t n, unsigned* out, hipStream_t s);
// ---- ALS Gramian eigenbasis on the device (kernels/als_eig.hip) ----------------------------
// gram: fp64 r x r symmetric (device).  Q / QT: float [ld][ld] (eigenvectors as columns of Q,
// identity padding), eig: float [ld] (max(lambda, 0), padding 1).  scratch: device bytes of
// als_gram_eig_scratch_bytes(r) (fp64 V when it does not fit in LDS next to A).
size_t als_gram_eig_scratch_bytes(int r);
// status (optional): incremented when the sweeps stop at max_sweeps short of the tolerance.
void als_gram_eig(const double* gram, int r, int ld, double* scratch, float* Q, float* QT,
                  float* eig, hipStream_t s, int max_sweeps = 30, double tol = 1e-14,
                  unsigned long long* status = nullptr);

// cov = (S - c c^T / n) / (n - 1) from pca_reduce's [S | c] output, on the device
void pca_cov(const double* stats, int d, int64_t n, double* cov, hipStream_t s);
// out: d x d symmetric (both triangles written), colsum: [d]
void pca_reduce(const PcaPlan& p, const double* part, const double* cpart, int d, double* out,
                double* colsum, hipStream_t s);

// ----------------------------------------------------------------------------- eigensolver
// Householder tridiagonalisation of a symmetric n x n fp64 matrix (device, row-major, full) by one
// persistent cooperative kernel with the matrix LDS-resident across the CUs (eig.hip).  Outputs:
// d[n], e[n] (e[n-2] last coupling; e[n-1] untouched), reflector rows vrows[n x n] and tau[n].
// scratch: eig_tridiag_scratch_doubles(n, num_cus) doubles; bar: 2 zeroed-by-the-call unsigned.
bool eig_tridiag_supported(int n, int num_cus);
int eig_tridiag_grid(int n, int num_cus);
size_t eig_tridiag_scratch_doubles(int n, int num_cus);
void eig_tridiag(const double* a, int n, int num_cus, double* d, double* e, double* vrows,
                 double* tau, double* scratch, unsigned* bar, hipStream_t s);
// All n eigenvalues (ascending) of the symmetric tridiagonal (d, e) by multisection; [lo, hi)
// must bracket the spectrum (Gershgorin), pivmin as LAPACK's.  Device pointers.
void eig_bisect(const double* d, const double* e, int n, double lo, double hi, double pivmin,
                double* out, hipStream_t s);
// Z (n x k row-major, device) <- Q Z with the reflectors of eig_tridiag.
void eig_apply_q(const double* vrows, const double* tau, int n, int k, double* z, hipStream_t s);
// Everything after eig_tridiag on the device, no host round trip: the Gershgorin bracket, every
// eigenvalue by multisection (lam [n], ascending), the `keep` of largest magnitude (stable order),
// their tridiagonal eigenvectors by inverse iteration with Gram-Schmidt inside clusters (the
// LAPACK dstein recipe), back-transformed by Q and sign-normalised: z [n x keep] row-major.
// scratch: eig_vectors_scratch_doubles(n, keep) doubles.
bool eig_vectors_supported(int n, int keep);
size_t eig_vectors_scratch_doubles(int n, int keep);
void eig_top_vectors(const double* d, const double* e, int n, int keep, const double* vrows,
                     const double* tau, double* lam, double* z, double* scratch, hipStream_t s);

}  // namespace kern
}  // namespace oap
