#include "drivers/kmeans.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <limits>
#include <map>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>

#include "kernels/kernels.h"
#include "kernels/kmeans_init.h"
#include "kernels/kmeans_wide.h"
#include "runtime/knobs.h"

namespace oap {

namespace {

using u64 = unsigned long long;

double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// Host buffer collectives that work with device- or host-buffer comms.
void host_allreduce(Context& ctx, Comm& comm, void* host, size_t count, DType dt, ReduceOp op) {
  comm_allreduce_host(ctx, comm, host, count, dt, op);
}

// Gathers a variable number of f64 rows (cols wide) from every rank, rank-major.
std::vector<double> host_allgatherv_rows(Context& ctx, Comm& comm, const std::vector<double>& mine,
                                         int cols) {
  int64_t my_rows = cols ? int64_t(mine.size()) / cols : 0;
  if (comm.trivial()) return mine;
  auto counts = comm_allgather_i64(ctx, comm, my_rows);
  int64_t mx = 0;
  for (auto c : counts) mx = std::max(mx, c);
  if (mx == 0) return {};
  std::vector<double> send(size_t(mx) * cols, 0.0), recv(size_t(mx) * cols * comm.size());
  std::copy(mine.begin(), mine.end(), send.begin());
  size_t cnt = size_t(mx) * cols;
  if (comm.on_device()) {
    Buffer ds = ctx.alloc(cnt * 8), dr = ctx.alloc(cnt * 8 * comm.size());
    hipStream_t s = ctx.comm_stream();
    OAP_HIP_CHECK(hipMemcpyAsync(ds.data(), send.data(), cnt * 8, hipMemcpyHostToDevice, s));
    comm.allgather(ds.data(), dr.data(), cnt, DType::F64, s);
    OAP_HIP_CHECK(
        hipMemcpyAsync(recv.data(), dr.data(), recv.size() * 8, hipMemcpyDeviceToHost, s));
    comm.wait(s);
  } else {
    comm.allgather(send.data(), recv.data(), cnt, DType::F64, nullptr);
  }
  std::vector<double> out;
  for (int r = 0; r < comm.size(); ++r)
    out.insert(out.end(), recv.begin() + size_t(r) * cnt,
               recv.begin() + size_t(r) * cnt + size_t(counts[r]) * cols);
  return out;
}

struct FixedPoint {
  std::vector<float> scale;       // 2^e_f
  std::vector<double> inv_scale;  // 2^-e_f
};

// Per-feature fixed-point exponents e_f: every |rint(x * 2^e_f)| summed over the whole dataset
// stays below 2^61 (int64 global sums, any rank count), and over one assign workgroup's rows
// below 2^52 (exact integer partial sums in the GPU kernel's fp64 LDS accumulator).  The same
// function serves both engines so CPU and GPU produce identical integers.
FixedPoint fixed_point_scales(const std::vector<double>& absmax, int64_t global_rows,
                              int64_t max_local_rows) {
  FixedPoint fp;
  int d = static_cast<int>(absmax.size());
  fp.scale.resize(d);
  fp.inv_scale.resize(d);
  auto clog2 = [](double v) { return static_cast<int>(std::ceil(std::log2(std::max(v, 2.0)))); };
  const int ln = clog2(double(global_rows));
  // (the per-block bound of the GLOBAL row count, not this world's largest shard: a bound for
  // every sharding, so the scales — and the integers — are the same for any world size)
  const int lb = clog2(double(kern::kmeans_rows_per_block_bound(
      std::max(max_local_rows, global_rows))));
  const int budget = std::min(61 - ln, 52 - lb);
  for (int f = 0; f < d; ++f) {
    int e = 0;
    if (absmax[f] > 0 && std::isfinite(absmax[f])) {
      int lm = static_cast<int>(std::ceil(std::log2(absmax[f])));
      e = budget - lm;
      e = std::max(-100, std::min(120, e));
    }
    fp.scale[f] = std::ldexp(1.0f, e);
    fp.inv_scale[f] = std::ldexp(1.0, -e);
  }
  return fp;
}

// The fixed point's per-column bounds.  Provisional bounds from the initial centers,
// B_f = 2^(ceil(log2 max_c |c_f|) + 3) (identical on every rank and engine: the centers are), are
// taken whenever every row satisfies |x_f| < B_f; otherwise the global column maxima.  The rule
// needs no pass over the rows up front: the GPU fit's first full pass checks a sufficient
// condition (every |x_f| below min_f B_f: max3 chains, 16 VALU per 32-row tile) and only a
// flagged row costs the column-maxima pass (then the rule is evaluated exactly on them).
// Either way the scale is a function of (init centers, global column maxima), so the CPU engine,
// the out-of-core fit and every world size derive the same integers.
std::vector<double> center_bounds(const std::vector<double>& centers, int k, int d) {
  std::vector<double> b(d, 0.0);
  for (int f = 0; f < d; ++f) {
    double m = 0.0;
    for (int c = 0; c < k; ++c) m = std::max(m, std::fabs(centers[size_t(c) * d + f]));
    b[f] = (m > 0.0 && std::isfinite(m)) ? std::ldexp(1.0, int(std::ceil(std::log2(m))) + 3) : 0.0;
  }
  return b;
}

// The provisional bounds cost up to 3 bits of the fixed point's resolution against the column
// maxima; they apply only where the pass they save is worth it: datasets of at least
// OAP_KMEANS_PROVISIONAL_MIN elements (global rows x features, default 2^28 — 1 GiB of f32).
bool provisional_allowed(int64_t global_rows, int d) {
  const double lim = knob_float("OAP_KMEANS_PROVISIONAL_MIN");  // (read per fit: tests set it)
  return double(global_rows) * double(d) >= lim;
}

std::vector<double> fit_bounds(const std::vector<double>& cb, const std::vector<double>& absmax,
                               int64_t global_rows, bool* from_centers) {
  bool ok = provisional_allowed(global_rows, int(cb.size()));
  for (size_t f = 0; f < cb.size(); ++f) ok = ok && absmax[f] < cb[f];
  *from_centers = ok;
  return ok ? cb : absmax;
}

inline double table_at(const DenseTable& t, int64_t r, int c) {
  return t.dtype == DType::F64 ? t.data.as<double>()[size_t(r) * t.ld + c]
                               : double(t.data.as<float>()[size_t(r) * t.ld + c]);
}

// ---------------------------------------------------------------------------- CPU engine
struct CpuAssignOut {
  std::vector<int64_t> sums;    // k*d fixed point (when accumulate)
  std::vector<int64_t> counts;  // k
  double cost = 0.0;
};

// Exact fp64 distances; lowest index wins ties (Spark findClosest semantics).
CpuAssignOut cpu_assign(Context& ctx, const DenseTable& x, const std::vector<double>& centers,
                        int k, const FixedPoint* fp, bool accumulate, bool sums_too,
                        int32_t* labels, double* dist2) {
  const int d = x.cols;
  const int P = ctx.pool().size();
  std::vector<CpuAssignOut> part(P);
  ctx.pool().parallel_for(x.rows, [&](int ci, int64_t b, int64_t e) {
    CpuAssignOut& o = part[ci];
    if (accumulate) {
      o.counts.assign(k, 0);
      if (sums_too) o.sums.assign(size_t(k) * d, 0);
    }
    std::vector<double> xr(d);
    for (int64_t r = b; r < e; ++r) {
      for (int f = 0; f < d; ++f) xr[f] = table_at(x, r, f);
      double best = std::numeric_limits<double>::infinity();
      int bi = 0;
      for (int c = 0; c < k; ++c) {
        const double* cr = centers.data() + size_t(c) * d;
        double acc = 0.0;
        for (int f = 0; f < d; ++f) {
          double df = xr[f] - cr[f];
          acc += df * df;
        }
        if (acc < best) {
          best = acc;
          bi = c;
        }
      }
      if (labels) labels[r] = bi;
      if (dist2) dist2[r] = best;
      o.cost += best;
      if (accumulate) {
        o.counts[bi] += 1;
        if (sums_too)
          for (int f = 0; f < d; ++f)
            o.sums[size_t(bi) * d + f] += static_cast<int64_t>(
                std::llrint(xr[f] * double(fp->scale[f])));
      }
    }
  });
  CpuAssignOut out;
  if (accumulate) {
    out.counts.assign(k, 0);
    if (sums_too) out.sums.assign(size_t(k) * d, 0);
  }
  for (auto& o : part) {  // chunk order => deterministic cost
    out.cost += o.cost;
    if (!accumulate || o.counts.empty()) continue;
    for (int c = 0; c < k; ++c) out.counts[c] += o.counts[c];
    if (sums_too)
      for (size_t i = 0; i < out.sums.size(); ++i)
        out.sums[i] = static_cast<int64_t>(static_cast<u64>(out.sums[i]) +
                                           static_cast<u64>(o.sums[i]));
  }
  return out;
}

// ---------------------------------------------------------------------------- GPU helpers
// Device-resident centers in the padded kernel layout.
struct GpuCenters {
  Buffer c32, cnorm, cstat;
  int k = 0, kpad = 0, dp = 0;
};

GpuCenters alloc_centers(Context& ctx, int k, int d) {
  GpuCenters g;
  g.k = k;
  g.kpad = static_cast<int>(round_up(std::max(k, 1), 32));
  g.dp = kern::kmeans_dp(d);
  g.c32 = ctx.alloc(sizeof(float) * size_t(g.kpad) * g.dp);
  g.cnorm = ctx.alloc(sizeof(float) * g.kpad);
  g.cstat = ctx.alloc(sizeof(float) * 4);
  return g;
}

GpuCenters upload_centers(Context& ctx, const std::vector<double>& centers, int k, int d) {
  GpuCenters g = alloc_centers(ctx, k, d);
  Buffer c64 = ctx.alloc(sizeof(double) * size_t(std::max(k, 1)) * d);
  ctx.copy_to_backend(c64.data(), centers.data(), sizeof(double) * size_t(k) * d);
  kern::kmeans_prepare_centers(c64.as<double>(), k, d, g.dp, g.c32.as<float>(),
                               g.cnorm.as<float>(), g.cstat.as<float>(), g.kpad, ctx.compute());
  OAP_HIP_CHECK(hipStreamSynchronize(ctx.compute()));
  return g;
}

// One assignment pass over the local rows.  Uses the fused single-launch kernel when the
// centroids fit the LDS plan, otherwise walks centroid chunks (merge mode: exact-cost argmin
// across chunks, earlier chunk wins ties) and accumulates from the labels afterwards.
struct AssignReq {
  bool accumulate = false;
  bool sums_too = true;
  bool precise = false;
  const float* scale = nullptr;
  u64* sums = nullptr;
  u64* counts = nullptr;
  int32_t* labels = nullptr;  // device, optional
  float* mindist = nullptr;   // device, optional
  double* cost_slab = nullptr;
  u64* refine_tiles = nullptr;
  // chunked path: `labels` already holds the previous assignment (a Lloyd iteration > 0), so
  // the merge passes start from its exact distance
  bool labels_valid = false;
  // chunked path: `mindist` already holds an upper bound that only a strictly closer center may
  // replace (k-means|| cost updates: the merge passes then compute min(old, new) in place)
  bool mindist_seeded = false;
  // start at the 1-product tier (the fit turns it off when tier-3 re-runs get frequent)
  bool fast1 = true;
  // pruning state (kmeans_assign.hip "Pruning"): bounds [rows] float2 pairs; drift / drift_max
  // only when bounds and `labels` hold the previous iteration's values
  float* bounds = nullptr;
  const float* drift = nullptr;
  const float* drift_max = nullptr;
  u64* pruned_tiles = nullptr;
  // chunked path with pruning: [ceil(rows/32)] active-tile list + its counter
  int32_t* tile_list = nullptr;
  unsigned* tile_count = nullptr;
  // chunked path: defer in-chunk near ties to a re-run after the last chunk (pays off when the
  // centers are distinct cluster centers — Lloyd / predict; k-means|| candidate sets hold
  // several near-identical points per cluster, whose ties are genuine, so init passes opt out)
  bool defer = true;
  // single launch, pruning on: delta accumulation over req.tile_list (see KMeansAssignArgs)
  bool delta = false;
  float* xnorm = nullptr;
  // single launch, fast1: the lean tier-1 kernel + the general kernel over its deferred rows
  // (kmeans_lloyd.hip); defer_rows / defer_count: persistent buffers (allocated per call if null)
  bool lean = true;
  int32_t* defer_rows = nullptr;
  unsigned* defer_count = nullptr;
  u64* deferred_rows = nullptr;
  int ablate = 0;  // timing ablations (kern::KMeansAssignArgs::ablate)
  // centroid-chunked lean pass: sums / counts persist across iterations (local statistics);
  // with prev_labels (the previous iteration's labels, a separate buffer) only the moved rows
  // are accumulated, otherwise the statistics are recounted from zero
  bool stats_persist = false;
  const int32_t* prev_labels = nullptr;
  int64_t* moved_rows = nullptr;  // host counter of the rows the delta accumulated
  // lean kernel's resident fp16 operand image (KMeansAssignArgs::ximg / img_beta / img_mode)
  void* ximg = nullptr;
  float* img_beta = nullptr;
  int img_mode = 0;
  // img_mode 2: also launch the f32-row fallback (kmeans_lloyd img_mode 3) after the image
  // kernel, for the case the image's scale cannot hold the current centers (the host clears it
  // once the rows' norms prove that impossible)
  bool img_fallback = true;
  int img_kernel = -1;      // timing probes: 0 kmeans_lloyd's image branch, else the image kernel
  int img_cfg = -1;         // timing probes: oap_kmeans_lean_img configuration (0 / 1; -1 default)
  bool skip_exact = false;  // timing probes: the lean pass only
  // image passes with the row scan fused into the image kernel (KMeansAssignArgs::img_scan_*)
  const float* img_scan_xnorm = nullptr;
  const float* img_scan_drift = nullptr;
  u64* img_scan_pruned = nullptr;
  // lean full pass: per-workgroup sum |x|^2 and the provisional-bound check (KMeansAssignArgs)
  double* sq_slab = nullptr;
  unsigned* bound_flag = nullptr;
  float bound_inf = 0.f;
  // batched fits with a tolerance: the kernels stand down once the fit converged
  const int* halt = nullptr;
  // fused row-scan image passes: a device word (kern::kmeans_scan_decide) picks the scan (1) or
  // the dense pass (0); both are enqueued (KMeansAssignArgs::img_gate)
  const int* img_gate = nullptr;
};

int& lean_variant_ref() {  // -1: by width (below); kmeans_set_lean_variant (timing probes)
  static int v = -1;
  return v;
}
// Workgroup shape of the lean kernel: variant 6 (16 waves, 4 per SIMD, 128 registers, fragment
// reads grouped ahead of each MFMA chain) unless the rows are 7-8 k-steps wide, where 128
// registers spill (config 5, d = 100: 232 B/lane of scratch) and variant 8 (12 waves, 168
// registers) measured 3.5% faster (396 -> 382 ms/iter at 1B rows).
int lean_variant(int d, int kpad) {
  (void)kpad;
  const int v = lean_variant_ref();
  if (v == 6 || v == 8) return v;
  return d + 4 > 96 ? 8 : 6;
}

// Whether gpu_assign takes the lean path for this request.
bool lean_applies(const DenseTable& x, int k, int kpad, const AssignReq& req) {
  return req.lean && req.fast1 && !req.precise && x.cols <= 128 && !req.mindist_seeded &&
         kern::kmeans_lloyd_supported(x.cols, k, req.accumulate, req.sums_too) &&
         !(req.bounds && req.drift && !req.delta);  // the in-kernel pruning test: general kernel
}

// Whether the centroid-chunked lean pass applies: k too large for one LDS plan of the general
// kernel, but small enough for 10-bit key indices; no pruning state (full passes).
bool lean_chunked_applies(const DenseTable& x, const GpuCenters& g, const AssignReq& req,
                          int kmax) {
  const bool off = knob_on("OAP_KMEANS_NO_LEAN_CHUNKED");
  return !off && req.lean && req.fast1 && !req.precise && !req.mindist_seeded && !req.bounds &&
         !req.delta && x.cols <= 128 && g.kpad > kmax && g.kpad <= 1024 &&
         kern::kmeans_lloyd_chunk_kmax(x.cols) >= 32 && kern::kmeans_exact_chunk_kmax(x.cols) >= 32;
}

size_t lean_defer_bytes(int64_t rows, int d, int kpad, int num_cus, int* grid, int64_t* cap) {
  *grid = kern::kmeans_lloyd_grid(rows, num_cus);
  *cap = kern::kmeans_lloyd_seg_cap(rows, *grid, kern::kmeans_lloyd_waves(lean_variant(d, kpad)));
  return sizeof(int32_t) * size_t(*grid) * size_t(*cap) + sizeof(unsigned) * 16 * size_t(*grid);
}

// The distance path the last gpu_assign of this thread took (reported with the fit result, so
// a benchmark names the kernel that actually ran).
thread_local const char* t_assign_path = "none";

// Returns the number of cost partials written to req.cost_slab.
int gpu_assign(Context& ctx, const DenseTable& x, const GpuCenters& g, const AssignReq& req,
               hipStream_t s) {
  kern::KMeansAssignArgs a;
  a.x = x.data.data();
  a.xbf16 = x.dtype == DType::BF16;
  a.n = x.rows;
  a.ld = static_cast<int>(x.ld);
  a.d = x.cols;
  a.centers = g.c32.as<float>();
  a.cnorm = g.cnorm.as<float>();
  a.cstat = g.cstat.as<float>();
  a.k = g.k;
  a.kpad = g.kpad;
  a.scale = req.scale;
  a.sums = req.sums;
  a.counts = req.counts;
  a.cost_slab = req.cost_slab;
  a.labels = req.labels;
  a.mindist = req.mindist;
  a.accumulate = req.accumulate;
  a.sums_too = req.sums_too;
  a.precise = req.precise;
  a.refine_tiles = req.refine_tiles;
  a.fast1 = req.fast1 && !req.precise;
  a.bounds = req.bounds;
  a.drift = req.drift;
  a.drift_max = req.drift_max;
  a.pruned_tiles = req.pruned_tiles;
  OAP_CHECK(!req.bounds || (x.cols <= 128 && !req.precise && req.labels),
            "kmeans pruning needs the fast path (d <= 128) and persistent labels");
  a.xnorm = req.xnorm;
  a.ablate = req.ablate;
  a.halt = req.halt;
  const int kmax = kern::kmeans_lds_kmax(x.cols, req.precise);
  if (x.rows > 0 && lean_applies(x, g.k, g.kpad, req)) {
    // ---- lean tier-1 pass, then the general kernel re-decides the deferred rows exactly
    int grid = 0;
    int64_t cap = 0;
    const size_t dbytes =
        lean_defer_bytes(x.rows, x.cols, g.kpad, ctx.info().cu_count, &grid, &cap);
    Buffer dbuf;
    int32_t* drows = req.defer_rows;
    unsigned* dcnt = req.defer_count;
    if (!drows) {
      dbuf = ctx.alloc(dbytes);
      drows = dbuf.as<int32_t>();
      dcnt = reinterpret_cast<unsigned*>(drows + size_t(grid) * size_t(cap));
    }
    a.defer_rows = drows;
    a.defer_row_count = dcnt;
    a.row_seg_cap = cap;
    a.deferred_rows = req.deferred_rows;
    a.tile_list = nullptr;
    a.tile_count = nullptr;
    a.ximg = req.ximg;
    a.img_beta = req.img_beta;
    a.img_mode = req.img_mode;
    a.img_scan_xnorm = req.img_mode == 2 ? req.img_scan_xnorm : nullptr;
    a.img_scan_drift = req.img_mode == 2 ? req.img_scan_drift : nullptr;
    a.img_scan_pruned = req.img_mode == 2 ? req.img_scan_pruned : nullptr;
    a.sq_slab = req.sq_slab;
    a.bound_flag = req.bound_flag;
    a.bound_inf = req.bound_inf;
    if (req.delta) {  // delta accumulation; over the scan's tile list when there is one
      OAP_CHECK(req.labels && req.labels_valid,
                "kmeans delta accumulation needs the previous iteration's labels");
      a.delta = true;
      if (req.tile_list) {
        OAP_CHECK(req.bounds && req.drift && req.tile_count, "scan pass without bounds");
        a.tile_list = req.tile_list;
        a.tile_count = req.tile_count;
      }
    }
    t_assign_path = req.img_mode == 2
                        ? (req.tile_list ? "lean_fp16_image_delta_scan" : "lean_fp16_image_delta")
                    : req.delta ? (req.tile_list ? "lean_fp16_delta_scan" : "lean_fp16_delta")
                                : "lean_fp16";
    const int lv = lean_variant(x.cols, a.kpad);
    const int lw = kern::kmeans_lloyd_waves(lv);
    const bool img_k = req.img_kernel != 0;
    if (req.img_mode == 2 && img_k &&
        kern::kmeans_lean_img_supported(x.cols, g.k, lw, a.img_scan_xnorm != nullptr)) {
      // configurations: 0 for row-scan passes (the scan's prefetched bounds fit the non-pipelined
      // loop's registers; the pipelined one spills 64 B/lane, 4.66 vs 5.14 ms/step), 1 (the
      // pipelined chunk loop) for dense passes
      const int dense_cfg = req.img_cfg >= 0 ? req.img_cfg : 1;
      const int cfg = req.img_cfg >= 0 ? req.img_cfg : a.img_scan_xnorm ? 0 : 1;
      if (a.img_scan_xnorm && req.img_gate) {
        // the scan pass and the dense pass, one of which runs (the device gate)
        kern::KMeansAssignArgs as = a;
        as.img_gate = req.img_gate;
        as.img_gate_on = 1;
        kern::kmeans_lean_img(as, grid, lw, cfg, s);
        kern::KMeansAssignArgs ad = a;
        ad.img_scan_xnorm = nullptr;
        ad.img_scan_drift = nullptr;
        ad.img_scan_pruned = nullptr;
        ad.img_gate = req.img_gate;
        ad.img_gate_on = 0;
        kern::kmeans_lean_img(ad, grid, lw, dense_cfg, s);
      } else {
        kern::kmeans_lean_img(a, grid, lw, cfg, s);
      }
      if (req.img_fallback) {
        kern::KMeansAssignArgs f = a;
        f.img_mode = 3;
        kern::kmeans_lloyd(f, grid, lv, s);
      }
      t_assign_path = a.img_scan_xnorm && req.img_gate
                          ? "lean_img_kernel_delta_fused_rowscan_gated"
                      : a.img_scan_xnorm ? "lean_img_kernel_delta_fused_rowscan"
                      : req.tile_list    ? "lean_img_kernel_delta_scan"
                                         : "lean_img_kernel_delta";
    } else {
      OAP_CHECK(!a.img_scan_xnorm, "kmeans: a row-scan image pass needs the image kernel");
      kern::kmeans_lloyd(a, grid, lv, s);
    }
    if (req.skip_exact) return 0;
    kern::KMeansAssignArgs b = a;
    b.ximg = nullptr;
    b.img_mode = 0;
    b.defer_rows = nullptr;
    b.defer_row_count = nullptr;
    b.deferred_rows = nullptr;
    b.row_list = drows;
    b.row_count = dcnt;
    b.row_subs = kern::kmeans_lloyd_waves(lean_variant(x.cols, a.kpad));
    b.tile_list = nullptr;
    b.tile_count = nullptr;
    b.xnorm = nullptr;
    b.img_scan_xnorm = nullptr;
    b.img_scan_drift = nullptr;
    b.img_scan_pruned = nullptr;
    b.sq_slab = nullptr;
    b.bound_flag = nullptr;
    b.cost_slab = a.cost_slab ? a.cost_slab + grid : nullptr;
    kern::kmeans_exact_rows(b, grid, s);
    return a.cost_slab ? 2 * grid : 0;
  }
  if (x.cols > 128 && x.rows > 0 && req.fast1 && !req.precise && !req.mindist_seeded &&
      !req.delta && kern::kmeans_wide_supported(x.cols, g.k) &&
      !knob_on("OAP_KMEANS_NO_WIDE")) {
    // ---- wide rows on MFMA (kmeans_wide.hip): tier-1 labels + exact re-decision, then the
    // label-driven accumulation and (when asked) the per-row cost
    Buffer lab, dbuf;
    int32_t* labels = req.labels;
    if (!labels) {
      lab = ctx.alloc(sizeof(int32_t) * size_t(x.rows));
      labels = lab.as<int32_t>();
    }
    a.labels = labels;
    t_assign_path = "wide_mfma";
    dbuf = ctx.alloc(sizeof(int32_t) * size_t(x.rows) + 64);
    unsigned* dcount = reinterpret_cast<unsigned*>(dbuf.as<int32_t>() + x.rows);
    kern::kmeans_wide_assign(a, ctx.info().cu_count, dbuf.as<int32_t>(), dcount, s);
    if (req.accumulate)
      kern::kmeans_accumulate(x.data.data(), x.dtype == DType::BF16, x.rows, int(x.ld), x.cols,
                              labels, g.k, req.scale, req.sums_too ? req.sums : nullptr,
                              req.counts, s);
    if (req.cost_slab)
      return kern::kmeans_wide_cost(a, req.cost_slab, kern::kmeans_cost_slab_size(
                                                          ctx.info().cu_count), s);
    if (req.mindist) {
      Buffer tmp = ctx.alloc(sizeof(double) * size_t(kern::kmeans_cost_slab_size(
                                                  ctx.info().cu_count)));
      kern::kmeans_wide_cost(a, tmp.as<double>(), kern::kmeans_cost_slab_size(
                                                      ctx.info().cu_count), s);
      OAP_HIP_CHECK(hipStreamSynchronize(s));  // (tmp is freed on return)
    }
    return 0;
  }
  if (x.cols > 128 || g.kpad <= kmax || kmax == 0) {
    if (req.delta) {
      OAP_CHECK(req.bounds && req.drift && req.tile_list && req.labels_valid,
                "kmeans delta accumulation needs the pruning scan's tile list");
      a.delta = true;
      a.tile_list = req.tile_list;
      a.tile_count = req.tile_count;
    }
    t_assign_path = req.precise ? "exact_fp32_mfma" : "tiered_bf16_mfma";
    return kern::kmeans_assign(a, ctx.info().cu_count, s);
  }
  OAP_CHECK(!req.delta, "kmeans delta accumulation is single-launch only");
  if (x.rows > 0 && lean_chunked_applies(x, g, req, kmax)) {
    // ---- centroid-chunked lean pass: the lean tier-1 kernel walks chunks of the fp16 centroid
    // plane carrying each row's top-2 keys (global indices) between launches; the last chunk
    // finishes the sure rows and defers the near ties; the exact re-decision walks chunks of
    // fp32 centers carrying (best, index); labels drive the binned accumulation.
    const int lk = kern::kmeans_lloyd_chunk_kmax(x.cols);
    const int ek = kern::kmeans_exact_chunk_kmax(x.cols);
    t_assign_path = req.stats_persist && req.prev_labels ? "lean_fp16_centroid_chunked_delta"
                                                         : "lean_fp16_centroid_chunked";
    auto split = [&](int cap, int* n) {
      *n = (g.k + cap - 1) / cap;
      return static_cast<int>(round_up((g.k + *n - 1) / *n, 32));
    };
    int nl = 0, ne = 0;
    const int lsz = split(lk, &nl), esz = split(ek, &ne);
    int grid = 0;
    int64_t cap = 0;
    Buffer dbuf =
        ctx.alloc(lean_defer_bytes(x.rows, x.cols, g.kpad, ctx.info().cu_count, &grid, &cap));
    int32_t* drows = dbuf.as<int32_t>();
    unsigned* dcnt = reinterpret_cast<unsigned*>(drows + size_t(grid) * size_t(cap));
    Buffer keys = ctx.alloc(sizeof(int32_t) * 2 * size_t(x.rows));
    Buffer xstate = ctx.alloc(sizeof(float) * 2 * size_t(grid) * size_t(cap));
    Buffer lab;
    int32_t* labels = req.labels;
    if (!labels && req.accumulate) {
      lab = ctx.alloc(sizeof(int32_t) * size_t(x.rows));
      labels = lab.as<int32_t>();
    }
    a.labels = labels;
    a.accumulate = false;
    a.defer_rows = drows;
    a.defer_row_count = dcnt;
    a.row_seg_cap = cap;
    a.lean_keys = keys.as<int32_t>();
    a.xstate = xstate.as<float>();
    a.centers_all = g.c32.as<float>();
    a.kglob = g.k;
    auto chunk = [&](kern::KMeansAssignArgs& b, int c, int size, int ci, int n) {
      const int kc = std::min(size, g.k - c);
      b.centers = g.c32.as<float>() + size_t(c) * g.dp;
      b.cnorm = g.cnorm.as<float>() + c;
      b.k = kc;
      b.kpad = static_cast<int>(round_up(kc, 32));
      b.base = c;
      b.chunk_mode = n == 1 ? 0 : (ci == 0 ? 1 : (ci == n - 1 ? 3 : 2));
      if (b.chunk_mode == 1 || b.chunk_mode == 2) {  // running state only
        b.labels = nullptr;
        b.mindist = nullptr;
        b.cost_slab = nullptr;
        b.deferred_rows = nullptr;
      }
    };
    for (int ci = 0; ci < nl; ++ci) {
      kern::KMeansAssignArgs b = a;
      b.deferred_rows = req.deferred_rows;
      chunk(b, ci * lsz, lsz, ci, nl);
      kern::kmeans_lloyd(b, grid, lean_variant(x.cols, g.kpad), s);
    }
    for (int ci = 0; ci < ne; ++ci) {
      kern::KMeansAssignArgs b = a;
      b.defer_rows = nullptr;
      b.defer_row_count = nullptr;
      b.deferred_rows = nullptr;
      b.row_list = drows;
      b.row_count = dcnt;
      b.row_subs = kern::kmeans_lloyd_waves(lean_variant(x.cols, g.kpad));
      b.cost_slab = a.cost_slab ? a.cost_slab + grid : nullptr;
      chunk(b, ci * esz, esz, ci, ne);
      kern::kmeans_exact_rows(b, grid, s);
    }
    if (req.accumulate) {
      // the pass buffers go first (config 5 keeps 208 GB of rows resident; stream-ordered reuse)
      keys = Buffer();
      xstate = Buffer();
      dbuf = Buffer();
      const size_t sbytes = kern::kmeans_bin_scratch_bytes(x.rows, g.k);
      Buffer bins = ctx.alloc(sbytes);
      bool done = false;
      if (req.stats_persist && req.prev_labels && req.sums_too && req.sums) {
        // delta: moved rows only (+x new, -x old); above a quarter of the rows moved the
        // scratch is too small and the statistics are recounted
        int64_t entries = 0;
        done = kern::kmeans_accumulate_moved(
            x.data.data(), x.dtype == DType::BF16, x.rows, static_cast<int>(x.ld), x.cols,
            req.prev_labels, labels, g.k, req.scale, req.sums, req.counts, bins.data(), sbytes,
            &entries, s);
        if (req.moved_rows) *req.moved_rows += entries / 2;
      }
      if (!done) {
        if (req.stats_persist)
          OAP_HIP_CHECK(hipMemsetAsync(req.sums, 0, sizeof(u64) * size_t(g.k) * (x.cols + 1), s));
        if (!kern::kmeans_accumulate_binned(x.data.data(), x.dtype == DType::BF16, x.rows,
                                            static_cast<int>(x.ld), x.cols, labels, g.k,
                                            req.scale, req.sums_too ? req.sums : nullptr,
                                            req.counts, bins.data(), s))
          kern::kmeans_accumulate(x.data.data(), x.dtype == DType::BF16, x.rows,
                                  static_cast<int>(x.ld), x.cols, labels, g.k, req.scale,
                                  req.sums_too ? req.sums : nullptr, req.counts, s);
      }
    }
    return a.cost_slab ? 2 * grid : 0;
  }
  // ---- chunked path (more centroids than one LDS plan holds)
  t_assign_path = "tiered_bf16_mfma_chunked";
  Buffer lab, dist;
  int32_t* labels = req.labels;
  float* mind = req.mindist;
  if (!labels) {
    lab = ctx.alloc(sizeof(int32_t) * std::max<int64_t>(x.rows, 1));
    labels = lab.as<int32_t>();
  }
  if (!mind) {
    dist = ctx.alloc(sizeof(float) * std::max<int64_t>(x.rows, 1));
    mind = dist.as<float>();
  }
  a.labels = labels;
  a.mindist = mind;
  a.accumulate = false;
  a.cost_slab = nullptr;
  // Every chunk runs in merge mode against the row's best exact (cost, index) so far: seeded
  // with the previous assignment's distance when there is one (most rows keep their label, so
  // chunks that cannot win skip the exact re-decision of their own near ties), else +huge.
  if (req.labels_valid && req.labels) {
    if (req.bounds && req.drift && req.tile_list) {
      OAP_HIP_CHECK(hipMemsetAsync(req.tile_count, 0, sizeof(unsigned), s));
      a.tile_list = req.tile_list;
      a.tile_count = req.tile_count;
    }
    kern::kmeans_seed_mindist(a, s);
    if (a.tile_list && req.pruned_tiles) {
      // pruned tile passes = (tiles - listed tiles) per chunk: counted on the device
      kern::kmeans_count_pruned(a.tile_count, (x.rows + 31) / 32,
                                (g.k + kmax - 1) / kmax, req.pruned_tiles, s);
    }
  } else if (req.bounds) {
    // no previous assignment: every row is processed; the merge passes build its bound from
    // scratch, the seed verdict reads as "recompute" (0xbf bytes: negative floats)
    OAP_HIP_CHECK(hipMemsetAsync(mind, 0x7f, sizeof(float) * x.rows, s));
    OAP_HIP_CHECK(hipMemsetAsync(labels, 0, sizeof(int32_t) * x.rows, s));
    OAP_HIP_CHECK(hipMemsetAsync(req.bounds, 0xbf, sizeof(float) * 2 * x.rows, s));
  } else if (req.mindist_seeded && req.mindist) {
    OAP_HIP_CHECK(hipMemsetAsync(labels, 0, sizeof(int32_t) * x.rows, s));
  } else {
    OAP_HIP_CHECK(hipMemsetAsync(mind, 0x7f, sizeof(float) * x.rows, s));  // 3.4e38, finite
    OAP_HIP_CHECK(hipMemsetAsync(labels, 0, sizeof(int32_t) * x.rows, s));
  }
  // balanced chunks: ceil(k / kmax) launches of equal 32-multiples (no thin last pass)
  const int nchunks = (g.k + kmax - 1) / kmax;
  const int csize = static_cast<int>(round_up((g.k + nchunks - 1) / nchunks, 32));
  // Near ties inside a chunk that could still win are deferred (KMeansAssignArgs::defer_list):
  // after the last chunk each chunk re-runs on its deferred tiles against the row's final best,
  // which rules most of them out without the 3-product / exact re-decision (an unseeded first
  // chunk would otherwise escalate nearly every tile).
  int dgrid = 0;
  int64_t dcap = 0;
  kern::kmeans_defer_layout(x.rows, ctx.info().cu_count, &dgrid, &dcap);
  const size_t per_chunk = size_t(dgrid) * size_t(dcap);  // list entries of one chunk
  const size_t cnt_stride = round_up(size_t(dgrid), 16);
  Buffer defer = ctx.alloc(sizeof(int32_t) * per_chunk * nchunks +
                           sizeof(unsigned) * cnt_stride * nchunks);
  auto dlist = [&](int ci) { return defer.as<int32_t>() + per_chunk * ci; };
  auto dcount = [&](int ci) {
    return reinterpret_cast<unsigned*>(defer.as<int32_t>() + per_chunk * nchunks) +
           cnt_stride * ci;
  };
  OAP_HIP_CHECK(hipMemsetAsync(dcount(0), 0, sizeof(unsigned) * cnt_stride * nchunks, s));
  auto run_chunk = [&](int ci, bool main_pass) {
    const int c = ci * csize;
    const int kc = std::min(csize, g.k - c);
    kern::KMeansAssignArgs b = a;
    b.centers = g.c32.as<float>() + size_t(c) * g.dp;
    b.cnorm = g.cnorm.as<float>() + c;
    b.k = kc;
    b.kpad = static_cast<int>(round_up(kc, 32));
    b.base = c;
    b.merge = true;
    b.fresh_bound = main_pass && ci == 0;
    if (main_pass) {
      if (req.defer && c + csize < g.k) {  // the last chunk already sees the final best
        b.defer_list = dlist(ci);
        b.defer_count = dcount(ci);
      }
    } else {
      b.tile_list = dlist(ci);
      b.tile_count = dcount(ci);
      b.seg_list = true;
      b.pruned_tiles = nullptr;
    }
    kern::kmeans_assign(b, ctx.info().cu_count, s);
  };
  for (int ci = 0; ci * csize < g.k; ++ci) run_chunk(ci, true);
  if (req.defer)
    for (int ci = 0; (ci + 1) * csize < g.k; ++ci) run_chunk(ci, false);
  if (req.accumulate) {
    Buffer bins = ctx.alloc(kern::kmeans_bin_scratch_bytes(x.rows, g.k));
    if (!kern::kmeans_accumulate_binned(x.data.data(), x.dtype == DType::BF16, x.rows,
                                        static_cast<int>(x.ld), x.cols, labels, g.k, req.scale,
                                        req.sums_too ? req.sums : nullptr, req.counts,
                                        bins.data(), s))
      kern::kmeans_accumulate(x.data.data(), x.dtype == DType::BF16, x.rows,
                              static_cast<int>(x.ld), x.cols, labels, g.k, req.scale,
                              req.sums_too ? req.sums : nullptr, req.counts, s);
  }
  if (req.cost_slab) return kern::reduce_sum_f32(mind, x.rows, req.cost_slab, s);
  return 0;
}

void check_gpu_table(const DenseTable& x) {
  OAP_CHECK(x.dtype == DType::F32 || x.dtype == DType::BF16,
            "GPU K-Means expects an f32 or bf16 table, got " << dtype_name(x.dtype));
  const int want = kern::kmeans_ld(x.cols, x.dtype == DType::BF16);
  OAP_CHECK(x.ld == want, "table row stride " << x.ld << " does not match the K-Means layout "
                                              << want);
}

// k-means|| cost updates and candidate counts (k within one LDS plan) on the lean fp16 pass +
// exact re-decision instead of the general kernel's bf16x3 tier: 100M x 50, k = 200 init
// 133 -> 85 ms.  Both are exact-argmin paths; per-row fp32 distances may differ in the last
// ulp between them (direct vs expanded form), which can move a Bernoulli draw, so
// OAP_KMEANS_INIT_PRECISE=1 keeps the previous path for A/B runs.
bool init_fast() { return !knob_on("OAP_KMEANS_INIT_PRECISE"); }

// Candidate sets beyond one LDS plan take super-chunks of at most 1024 candidates on the lean
// pass (the centroid-chunked one where a super-chunk still exceeds the plan), the per-row exact
// answers merged by distance (kmeans_merge_argmin), instead of the general chunked kernel's
// bf16x3 tiers: config 5's ~2000-4000 candidates.  OAP_KMEANS_INIT_SUPER=0: the previous path.
// (debug: =1 cost updates only, =2 candidate counts only)
bool init_super(const DenseTable& x, int m, int which) {
  const std::string e = knob_str("OAP_KMEANS_INIT_SUPER");
  if (!e.empty() && (e[0] == '0' || (e[0] == '1' && which != 1) || (e[0] == '2' && which != 2)))
    return false;
  return init_fast() && x.cols <= 128 && x.rows > 0 &&
         int(round_up(size_t(m), 32)) > kern::kmeans_lds_kmax(x.cols, false) &&
         kern::kmeans_lloyd_chunk_kmax(x.cols) >= 32 && kern::kmeans_exact_chunk_kmax(x.cols) >= 32;
}

// super-chunk [base, base + size) of m candidates: sizes of at most 1024, multiples of 32
int super_size(int m) {
  const int n = (m + 1023) / 1024;
  return int(round_up(size_t((m + n - 1) / n), 32));
}

std::vector<double> centers_slice(const std::vector<double>& c, int d, int base, int size) {
  return std::vector<double>(c.begin() + size_t(base) * d, c.begin() + size_t(base + size) * d);
}

// Operations the initialisers need, on either backend.
class InitOps {
 public:
  InitOps(Context& ctx, DenseTable& x) : ctx_(ctx), x_(x) {
    if (ctx.is_gpu()) {
      check_gpu_table(x);
      costs_ = ctx.alloc(sizeof(float) * std::max<int64_t>(x.rows, 1));
      tmp_ = ctx.alloc(sizeof(float) * std::max<int64_t>(x.rows, 1));
      slab_ = ctx.alloc(sizeof(double) * std::max(kern::kmeans_cost_slab_size(256), 512));
      ctx.memset(costs_.data(), 0x7f, sizeof(float) * std::max<int64_t>(x.rows, 1));
    } else {
      hcost_.assign(x.rows, std::numeric_limits<double>::infinity());
    }
  }

  // costs = min(costs, dist^2 to `centers`)
  void update_costs(const std::vector<double>& centers, int m) {
    if (m == 0 || x_.rows == 0) return;
    if (ctx_.is_gpu() && init_super(x_, m, 1)) {
      const int ss = super_size(m), d = x_.cols;
      for (int base = 0; base < m; base += ss) {
        const int sz = std::min(ss, m - base);
        GpuCenters g = upload_centers(ctx_, centers_slice(centers, d, base, sz), sz, d);
        AssignReq req;
        req.mindist = tmp_.as<float>();
        req.fast1 = true;
        gpu_assign(ctx_, x_, g, req, ctx_.compute());
        kern::elementwise_min(costs_.as<float>(), tmp_.as<float>(), x_.rows, ctx_.compute());
        OAP_HIP_CHECK(hipStreamSynchronize(ctx_.compute()));  // (g is freed on return)
      }
    } else if (ctx_.is_gpu()) {
      GpuCenters g = upload_centers(ctx_, centers, m, x_.cols);
      AssignReq req;
      if (x_.cols <= 128 && g.kpad > kern::kmeans_lds_kmax(x_.cols, false)) {
        // chunked: merge straight into the running costs (chunks that cannot lower a row's cost
        // skip their exact re-decisions)
        req.mindist = costs_.as<float>();
        req.defer = false;
        req.fast1 = false;  // candidate sets: near ties are the rule (see count_closest)
        req.mindist_seeded = true;
        gpu_assign(ctx_, x_, g, req, ctx_.compute());
      } else {
        req.mindist = tmp_.as<float>();
        req.fast1 = init_fast();
        gpu_assign(ctx_, x_, g, req, ctx_.compute());
        kern::elementwise_min(costs_.as<float>(), tmp_.as<float>(), x_.rows, ctx_.compute());
      }
      OAP_HIP_CHECK(hipStreamSynchronize(ctx_.compute()));
    } else {
      std::vector<double> d2(x_.rows);
      cpu_assign(ctx_, x_, centers, m, nullptr, false, false, nullptr, d2.data());
      for (int64_t i = 0; i < x_.rows; ++i) hcost_[i] = std::min(hcost_[i], d2[i]);
    }
  }

  double local_cost_sum() {
    if (x_.rows == 0) return 0.0;
    if (ctx_.is_gpu()) {
      Buffer out = ctx_.alloc(sizeof(double));
      int m = kern::reduce_sum_f32(costs_.as<float>(), x_.rows, slab_.as<double>(),
                                   ctx_.compute());
      kern::sum_f64(slab_.as<double>(), m, out.as<double>(), ctx_.compute());
      double v = 0.0;
      ctx_.copy_to_host(&v, out.data(), sizeof(double));
      return v;
    }
    double s = 0.0;
    for (double c : hcost_) s += c;
    return s;
  }

  // Local row indices whose Bernoulli draw succeeds, sorted ascending.
  std::vector<int64_t> select(double factor, uint64_t seed, int step) {
    std::vector<int64_t> idx;
    if (x_.rows == 0) return idx;
    if (ctx_.is_gpu()) {
      Buffer flag = ctx_.alloc(sizeof(int32_t) * x_.rows);
      Buffer out = ctx_.alloc(sizeof(int64_t) * x_.rows);
      Buffer cnt = ctx_.alloc(sizeof(u64));
      ctx_.memset(cnt.data(), 0, sizeof(u64));
      kern::bernoulli_select(costs_.as<float>(), x_.rows, x_.global_offset, factor, seed, step,
                             flag.as<int32_t>(), ctx_.compute());
      kern::compact_flags(flag.as<int32_t>(), x_.rows, out.as<int64_t>(), cnt.as<u64>(),
                          ctx_.compute());
      u64 n = 0;
      ctx_.copy_to_host(&n, cnt.data(), sizeof(u64));
      idx.resize(n);
      ctx_.copy_to_host(idx.data(), out.data(), sizeof(int64_t) * n);
      std::sort(idx.begin(), idx.end());
      return idx;
    }
    for (int64_t i = 0; i < x_.rows; ++i) {
      uint64_t h = mix64(seed ^ (uint64_t(step) << 48) ^ uint64_t(x_.global_offset + i));
      double u = double(h >> 11) * (1.0 / 9007199254740992.0);
      // same float rounding of the cost as the GPU path keeps the two engines aligned
      if (u < factor * double(float(hcost_[i]))) idx.push_back(i);
    }
    return idx;
  }

  std::vector<double> rows(const std::vector<int64_t>& local_idx) {
    const int d = x_.cols;
    std::vector<double> out(local_idx.size() * d);
    if (local_idx.empty()) return out;
    if (ctx_.is_gpu()) {
      Buffer di = ctx_.alloc(sizeof(int64_t) * local_idx.size());
      Buffer dv = ctx_.alloc(sizeof(float) * local_idx.size() * d);
      ctx_.copy_to_backend(di.data(), local_idx.data(), sizeof(int64_t) * local_idx.size());
      kern::gather_rows(x_.data.data(), x_.dtype, x_.ld, d, di.as<int64_t>(),
                        int64_t(local_idx.size()), dv.as<float>(), ctx_.compute());
      std::vector<float> h(local_idx.size() * d);
      ctx_.copy_to_host(h.data(), dv.data(), sizeof(float) * h.size());
      for (size_t i = 0; i < h.size(); ++i) out[i] = h[i];
      return out;
    }
    for (size_t i = 0; i < local_idx.size(); ++i)
      for (int f = 0; f < d; ++f) out[i * d + f] = table_at(x_, local_idx[i], f);
    return out;
  }

  std::vector<int64_t> count_closest(const std::vector<double>& centers, int m) {
    std::vector<int64_t> cnt(m, 0);
    if (x_.rows == 0) return cnt;
    if (ctx_.is_gpu() && init_super(x_, m, 2)) {
      const int ss = super_size(m), d = x_.cols;
      Buffer lab_b = ctx_.alloc(sizeof(int32_t) * x_.rows);
      Buffer lab_s = ctx_.alloc(sizeof(int32_t) * x_.rows);
      Buffer best = ctx_.alloc(sizeof(float) * x_.rows);  // the running nearest distance
      for (int base = 0; base < m; base += ss) {
        const int sz = std::min(ss, m - base);
        GpuCenters g = upload_centers(ctx_, centers_slice(centers, d, base, sz), sz, d);
        AssignReq req;
        req.labels = lab_s.as<int32_t>();
        req.mindist = tmp_.as<float>();
        req.fast1 = true;
        gpu_assign(ctx_, x_, g, req, ctx_.compute());
        kern::kmeans_merge_argmin(best.as<float>(), lab_b.as<int32_t>(), tmp_.as<float>(),
                                  lab_s.as<int32_t>(), base, x_.rows, base == 0, ctx_.compute());
        OAP_HIP_CHECK(hipStreamSynchronize(ctx_.compute()));
      }
      Buffer dc = ctx_.alloc(sizeof(u64) * m);
      ctx_.memset(dc.data(), 0, sizeof(u64) * m);
      kern::kmeans_accumulate(x_.data.data(), x_.dtype == DType::BF16, x_.rows,
                              static_cast<int>(x_.ld), x_.cols, lab_b.as<int32_t>(), m, nullptr,
                              nullptr, dc.as<u64>(), ctx_.compute());
      ctx_.copy_to_host(cnt.data(), dc.data(), sizeof(u64) * m);
      return cnt;
    }
    if (ctx_.is_gpu()) {
      GpuCenters g = upload_centers(ctx_, centers, m, x_.cols);
      Buffer dc = ctx_.alloc(sizeof(u64) * m);
      ctx_.memset(dc.data(), 0, sizeof(u64) * m);
      AssignReq req;
      req.accumulate = true;
      req.sums_too = false;
      req.defer = false;
      // k-means|| candidates sit several per cluster (near ties are common): the lean fp16 pass
      // still wins — its deferred rows go straight to the exact re-decision (init_fast)
      req.fast1 = init_fast();
      req.counts = dc.as<u64>();
      gpu_assign(ctx_, x_, g, req, ctx_.compute());
      ctx_.copy_to_host(cnt.data(), dc.data(), sizeof(u64) * m);
      return cnt;
    }
    auto o = cpu_assign(ctx_, x_, centers, m, nullptr, true, false, nullptr, nullptr);
    return o.counts;
  }

 private:
  Context& ctx_;
  DenseTable& x_;
  Buffer costs_, tmp_, slab_;
  std::vector<double> hcost_;
};

// Fetch rows by GLOBAL index; every rank ends with all of them (owner fills, allreduce SUM).
std::vector<double> fetch_global_rows(Context& ctx, Comm& comm, DenseTable& x, InitOps& ops,
                                      const std::vector<int64_t>& gidx) {
  const int d = x.cols;
  std::vector<double> out(gidx.size() * d, 0.0);
  std::vector<int64_t> mine;
  std::vector<size_t> pos;
  for (size_t i = 0; i < gidx.size(); ++i) {
    int64_t l = gidx[i] - x.global_offset;
    if (l >= 0 && l < x.rows) {
      mine.push_back(l);
      pos.push_back(i);
    }
  }
  auto vals = ops.rows(mine);
  for (size_t i = 0; i < mine.size(); ++i)
    std::copy(vals.begin() + i * d, vals.begin() + (i + 1) * d, out.begin() + pos[i] * d);
  host_allreduce(ctx, comm, out.data(), out.size(), DType::F64, ReduceOp::Sum);
  return out;
}

std::vector<double> distinct_rows(const std::vector<double>& pts, int d) {
  std::vector<double> out;
  std::set<std::vector<double>> seen;
  size_t m = d ? pts.size() / d : 0;
  for (size_t i = 0; i < m; ++i) {
    std::vector<double> r(pts.begin() + i * d, pts.begin() + (i + 1) * d);
    for (auto& v : r)
      if (v == 0.0) v = 0.0;  // -0.0 == 0.0 as in Spark's Vector equality
    if (seen.insert(r).second) out.insert(out.end(), r.begin(), r.end());
  }
  return out;
}

// Uniform sample of m distinct indices of [0, n) in draw order (partial Fisher-Yates).
std::vector<int64_t> sample_without_replacement(int64_t n, int64_t m, uint64_t seed) {
  std::mt19937_64 rng(mix64(seed));
  std::unordered_map<int64_t, int64_t> swp;
  std::vector<int64_t> out;
  m = std::min(m, n);
  for (int64_t i = 0; i < m; ++i) {
    std::uniform_int_distribution<int64_t> u(i, n - 1);
    int64_t j = u(rng);
    int64_t vi = swp.count(i) ? swp[i] : i;
    int64_t vj = swp.count(j) ? swp[j] : j;
    swp[j] = vi;
    out.push_back(vj);
  }
  return out;
}

}  // namespace

// ------------------------------------------------------------------------ local k-means++
namespace {
// Elementwise loops over the candidate points run on the pool; every reduction over points is
// sequential in point order, so results are identical for any pool size (and to the serial code).
void for_points(ThreadPool* pool, size_t n, const std::function<void(size_t, size_t)>& fn) {
  if (!pool || pool->size() <= 1 || n < 256) {
    fn(0, n);
    return;
  }
  pool->parallel_for(int64_t(n), [&](int, int64_t b, int64_t e) { fn(size_t(b), size_t(e)); });
}

// Squared distances with every distance summed feature by feature in order (sub, mul, add; no
// contraction in this unit), the order of a plain per-pair loop, so the values are bitwise that
// loop's; the loops run across centers / points instead, which vectorises (independent sums) where
// the per-pair loop is one add-latency chain per distance (~4x faster at d = 100).
//   dist[j * k + c] = |p_j - c|^2 for the G points p (row-major, d) against ct (d x k, transposed)
template <int G>
void dist_rows_to_centers(const double* const* p, const double* ct, int d, int k, double* dist) {
  for (int j = 0; j < G; ++j)
    for (int c = 0; c < k; ++c) dist[size_t(j) * k + c] = 0.0;
  for (int f = 0; f < d; ++f) {
    const double* cf = ct + size_t(f) * k;
    for (int j = 0; j < G; ++j) {
      const double pf = p[j][f];
      double* dj = dist + size_t(j) * k;
      for (int c = 0; c < k; ++c) {
        const double df = pf - cf[c];
        dj[c] += df * df;
      }
    }
  }
}

// acc[i - b] = |p_i - c|^2 for points [b, e) of pt (d x n, transposed)
void dist_points_to_center(const double* pt, size_t n, int d, const double* c, size_t b, size_t e,
                           double* acc) {
  for (size_t i = b; i < e; ++i) acc[i - b] = 0.0;
  for (int f = 0; f < d; ++f) {
    const double* pf = pt + size_t(f) * n;
    const double cf = c[f];
    for (size_t i = b; i < e; ++i) {
      const double df = pf[i] - cf;
      acc[i - b] += df * df;
    }
  }
}

// One greedy k-means++ seeding (2 + ln k candidate draws per step, keep the one that lowers the
// weighted potential most) followed by weighted Lloyd; returns the weighted cost.
// pt: the points transposed (d x n).
double kmeans_pp_once(const std::vector<double>& pts, const std::vector<double>& pt,
                      const std::vector<double>& w, int d, int k, int max_iter,
                      std::mt19937_64& rng, std::vector<double>& centers, ThreadPool* pool) {
  const size_t n = pts.size() / d;
  constexpr size_t kBlk = 512;  // points per block of the across-points loops (L1-resident sums)
  std::uniform_real_distribution<double> U(0.0, 1.0);
  // Spark pickWeighted semantics: the first j with cum_j = mass_0 + .. + mass_{j-1} >= r (summed
  // in index order), minus one.  The running sums are formed once per mass vector (prefix) and
  // each draw is a binary search in them — the same sums in the same order, so the same pick as
  // the per-draw scan, without a serial scan per draw.
  std::vector<double> prefix(n + 1);
  auto prefix_of = [&](const std::vector<double>& mass) {
    double cum = 0.0;
    prefix[0] = 0.0;
    for (size_t j = 0; j < n; ++j) prefix[j + 1] = (cum += mass[j]);
  };
  auto pick = [&]() {  // (after prefix_of; masses are >= 0, so prefix is non-decreasing)
    const double r = U(rng) * prefix[n];
    const size_t j = size_t(std::lower_bound(prefix.begin(), prefix.end(), r) - prefix.begin());
    const size_t jj = std::min(j, n);
    return jj == 0 ? size_t(0) : jj - 1;
  };
  centers.assign(size_t(k) * d, 0.0);
  auto set_center = [&](int c, size_t i) {
    std::copy(pts.begin() + i * d, pts.begin() + (i + 1) * d, centers.begin() + size_t(c) * d);
  };
  prefix_of(w);
  set_center(0, pick());
  std::vector<double> cost(n), mass(n);
  for_points(pool, n, [&](size_t b, size_t e) {
    for (size_t i0 = b; i0 < e; i0 += kBlk)
      dist_points_to_center(pt.data(), n, d, centers.data(), i0, std::min(e, i0 + kBlk),
                            cost.data() + i0);
  });
  const int trials = 2 + static_cast<int>(std::log(double(k)));
  std::vector<size_t> cand(trials);
  std::vector<std::vector<double>> trial(trials, std::vector<double>(n));
  for (int c = 1; c < k; ++c) {
    for (size_t i = 0; i < n; ++i) mass[i] = w[i] * cost[i];
    prefix_of(mass);
    for (int t = 0; t < trials; ++t) cand[t] = pick();  // same RNG order as drawing per trial
    for_points(pool, n, [&](size_t b, size_t e) {
      for (int t = 0; t < trials; ++t) {
        const double* cc = pts.data() + cand[t] * d;
        double* tr = trial[t].data();
        for (size_t i0 = b; i0 < e; i0 += kBlk) {
          const size_t i1 = std::min(e, i0 + kBlk);
          dist_points_to_center(pt.data(), n, d, cc, i0, i1, tr + i0);
          for (size_t i = i0; i < i1; ++i) tr[i] = std::min(cost[i], tr[i]);
        }
      }
    });
    int best_t = 0;
    double best_pot = std::numeric_limits<double>::infinity();
    // every trial's potential summed in point order, the trials' sums interleaved (independent
    // add chains in one sweep instead of one latency-bound chain after another)
    std::vector<double> pots(trials, 0.0);
    for (size_t i = 0; i < n; ++i)
      for (int t = 0; t < trials; ++t) pots[t] += w[i] * trial[t][i];
    for (int t = 0; t < trials; ++t) {
      const double pot = pots[t];
      if (pot < best_pot) {
        best_pot = pot;
        best_t = t;
      }
    }
    set_center(c, cand[best_t]);
    cost.swap(trial[best_t]);
  }
  std::vector<int> old(n, -1), lab(n, 0);
  std::vector<double> ct(size_t(k) * d);
  auto transpose_centers = [&]() {
    for (int c = 0; c < k; ++c)
      for (int f = 0; f < d; ++f) ct[size_t(f) * k + c] = centers[size_t(c) * d + f];
  };
  // fn(i, dist row of point i) for every point, 4 points per sweep of the centers
  auto each_point_dists = [&](const std::function<void(size_t, const double*)>& fn) {
    for_points(pool, n, [&](size_t b, size_t e) {
      std::vector<double> dist(size_t(4) * k);
      size_t i = b;
      for (; i + 4 <= e; i += 4) {
        const double* p[4] = {&pts[i * d], &pts[(i + 1) * d], &pts[(i + 2) * d],
                              &pts[(i + 3) * d]};
        dist_rows_to_centers<4>(p, ct.data(), d, k, dist.data());
        for (int j = 0; j < 4; ++j) fn(i + j, dist.data() + size_t(j) * k);
      }
      for (; i < e; ++i) {
        const double* p[1] = {&pts[i * d]};
        dist_rows_to_centers<1>(p, ct.data(), d, k, dist.data());
        fn(i, dist.data());
      }
    });
  };
  bool moved = true;
  for (int it = 0; moved && it < max_iter; ++it) {
    moved = false;
    transpose_centers();
    each_point_dists([&](size_t i, const double* dv) {
      int best = 0;
      double bd = std::numeric_limits<double>::infinity();
      for (int c = 0; c < k; ++c)
        if (dv[c] < bd) {
          bd = dv[c];
          best = c;
        }
      lab[i] = best;
    });
    std::vector<double> cnt(k, 0.0), sums(size_t(k) * d, 0.0);
    for (size_t i = 0; i < n; ++i) {
      const int best = lab[i];
      for (int f = 0; f < d; ++f) sums[size_t(best) * d + f] += w[i] * pts[i * d + f];
      cnt[best] += w[i];
      if (best != old[i]) {
        moved = true;
        old[i] = best;
      }
    }
    for (int c = 0; c < k; ++c) {
      if (cnt[c] == 0.0) {
        std::uniform_int_distribution<size_t> ui(0, n - 1);
        set_center(c, ui(rng));
      } else {
        for (int f = 0; f < d; ++f) centers[size_t(c) * d + f] = sums[size_t(c) * d + f] / cnt[c];
      }
    }
  }
  std::vector<double> bdist(n);
  transpose_centers();
  each_point_dists([&](size_t i, const double* dv) {
    double bd = std::numeric_limits<double>::infinity();
    for (int c = 0; c < k; ++c) bd = std::min(bd, dv[c]);
    bdist[i] = bd;
  });
  double total = 0.0;
  for (size_t i = 0; i < n; ++i) total += w[i] * bdist[i];
  return total;
}
}  // namespace

// Spark's LocalKMeans.kMeansPlusPlus runs ONE plain k-means++ seeding + Lloyd; here the seeding
// is greedy (sklearn-style local trials) and the best of 3 restarts by weighted cost is kept —
// a strictly better local optimum for the same candidate set (deterministic given the seed, for
// any pool size).
std::vector<double> local_kmeans_pp(const std::vector<double>& pts, const std::vector<double>& w,
                                    int d, int k, int max_iter, uint64_t seed, ThreadPool* pool) {
  const size_t n = d ? pts.size() / d : 0;
  OAP_CHECK(n > 0 && w.size() == n, "local_kmeans_pp: bad inputs");
  std::mt19937_64 rng(mix64(seed));
  std::vector<double> pt(n * size_t(d));  // the points transposed (d x n): across-points loops
  for (size_t i = 0; i < n; ++i)
    for (int f = 0; f < d; ++f) pt[size_t(f) * n + i] = pts[i * d + f];
  std::vector<double> best, cur;
  double best_cost = std::numeric_limits<double>::infinity();
  for (int r = 0; r < 3; ++r) {
    double c = kmeans_pp_once(pts, pt, w, d, k, max_iter, rng, cur, pool);
    if (c < best_cost) {
      best_cost = c;
      best = cur;
    }
  }
  return best;
}

// ------------------------------------------------------------------------------- init
std::vector<double> kmeans_init_centers(Context& ctx, Comm& comm, DenseTable& x,
                                        const KMeansParams& p, int* k_eff) {
  TraceRange tr(&ctx.metrics(), "kmeans/init");
  if (x.global_offset < 0) assign_global_offsets(ctx, comm, x);
  const int d = x.cols;
  const int64_t N = x.global_rows;
  OAP_CHECK(N > 0, "K-Means needs at least one row");
  InitOps ops(ctx, x);
  const uint64_t seed = mix64(p.seed ^ 0x5DEECE66Dull);
  std::vector<double> centers;
  if (p.init == KMeansInit::Random) {
    auto gidx = sample_without_replacement(N, p.k, seed);
    centers = distinct_rows(fetch_global_rows(ctx, comm, x, ops, gidx), d);
  } else {
    auto first = sample_without_replacement(N, 1, seed);
    std::vector<double> cand = fetch_global_rows(ctx, comm, x, ops, first);
    std::vector<double> newc = cand;
    for (int step = 0; step < p.init_steps; ++step) {
      {
        TraceRange tu(&ctx.metrics(), "kmeans/init/update_costs");
        ops.update_costs(newc, static_cast<int>(newc.size() / d));
      }
      double sum = comm_allreduce_scalar(ctx, comm, ops.local_cost_sum(), ReduceOp::Sum);
      if (!(sum > 0.0)) break;  // every point already a center
      TraceRange ts(&ctx.metrics(), "kmeans/init/sample");
      auto local = ops.select(2.0 * p.k / sum, seed, step);
      newc = host_allgatherv_rows(ctx, comm, ops.rows(local), d);
      cand.insert(cand.end(), newc.begin(), newc.end());
      if (newc.empty()) break;
    }
    centers = distinct_rows(cand, d);
    int m = static_cast<int>(centers.size() / d);
    if (m > p.k) {
      std::vector<int64_t> cnt;
      {
        TraceRange tc(&ctx.metrics(), "kmeans/init/count_closest");
        cnt = ops.count_closest(centers, m);
        host_allreduce(ctx, comm, cnt.data(), cnt.size(), DType::I64, ReduceOp::Sum);
      }
      std::vector<double> w(cnt.begin(), cnt.end());
      TraceRange tl(&ctx.metrics(), "kmeans/init/local_kmeans_pp");
      centers = local_kmeans_pp(centers, w, d, p.k, 30, seed ^ 0x1234567ull, &ctx.pool());
    }
  }
  *k_eff = static_cast<int>(centers.size() / d);
  std::ostringstream os;
  os << "\"k\":" << p.k << ",\"k_eff\":" << *k_eff << ",\"mode\":" << int(p.init);
  Logger::instance().log(LogLevel::Info, "kmeans/init", os.str());
  return centers;
}

// ------------------------------------------------------------------------------- fit
// The exact cost of the last assignment from the fit's own statistics, without a pass over
// the rows:  sum_i |x_i - c_l(i)|^2 = sum_i |x_i|^2 - 2 sum_c c.S_c + sum_c n_c |c|^2, with
// sum_i |x_i|^2 summed by the fit's first pass (the rows' fp32 norms, fp64 sum; a pass of its
// own when the first pass was not the lean kernel), S_c and n_c the global fixed-point
// statistics the last finalize used and c the fp32 centers that assignment used.  The rigorous
// error bound — the norms' fp32 rounding, fixed-point quantisation of S_c (|S~ - S| <= n_c q_f / 2
// per feature) plus fp64 rounding — must stay within kStatsCostRel of the result, else (rows far
// from the origin, a table layout without the norm kernel) it returns false and the caller runs
// the per-row pass.  Rank-uniform: every input is global (the norm
// sum is allreduced), so every rank takes the same branch.
// (accepted when its rigorous bound is within 1e-5 of the result: the per-row fp32 cost pass it
// replaces carries (d + 1) 2^-24 per row — ~3e-6 at d = 50 — in the worst case too)
constexpr double kStatsCostRel = 1e-5;
// OAP_KMEANS_HOST_MARKS=1: host timestamps at the fit's phase boundaries, to stderr (where a
// fit's wall clock goes when its kernels do not fill it: allocations, syncs, read-backs)
namespace {
// Drains a stream when the scope unwinds by an exception: the pooled pinned buffers a fit reads
// back into (flags, counters) go back to the pool on destruction, and an async copy still in
// flight must not land in a block another caller already holds (runtime/memory.h contract).
struct StreamDrainOnUnwind {
  hipStream_t s;
  int n0 = std::uncaught_exceptions();
  ~StreamDrainOnUnwind() {
    if (std::uncaught_exceptions() > n0) (void)hipStreamSynchronize(s);
  }
};
struct HostMarks {
  bool on = false;
  std::chrono::steady_clock::time_point t0;
  std::string out;
  HostMarks() {
    on = knob_on("OAP_KMEANS_HOST_MARKS");
    t0 = std::chrono::steady_clock::now();
  }
  void mark(const char* what) {
    if (!on) return;
    const double us =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    out += std::string(" ") + what + "=" + std::to_string(int64_t(us));
  }
  ~HostMarks() {
    if (on) std::fprintf(stderr, "kmeans_fit host marks (us):%s\n", out.c_str());
  }
};
}  // namespace

static bool final_cost_from_stats(Context& ctx, Comm& comm, DenseTable& x, const u64* sums_d,
                           const u64* counts_d, const float* centers_d, int k, int d, int dp,
                           const std::vector<double>& inv_scale, const double* fused_T,
                           double* cost) {
  double t_err = 0.0;
  // sum |x|^2: fused into the fit's first pass when it ran the lean kernel (fused_T = {sum,
  // relative bound}), else one pass over the rows now
  double T = fused_T ? fused_T[0] : local_row_sqnorm(ctx, x, &t_err);
  if (fused_T) t_err = fused_T[1];
  double terr_abs = std::isfinite(T) ? t_err * T : std::numeric_limits<double>::quiet_NaN();
  if (!comm.trivial()) {
    T = comm_allreduce_scalar(ctx, comm, T, ReduceOp::Sum);
    terr_abs = comm_allreduce_scalar(ctx, comm, terr_abs, ReduceOp::Sum);
  }
  if (!std::isfinite(T) || !std::isfinite(terr_abs)) return false;
  const size_t kd = size_t(k) * d;
  std::vector<u64> sh(kd), nh(k);
  std::vector<float> ch(size_t(k) * dp);
  ctx.copy_to_host(sh.data(), sums_d, sizeof(u64) * kd);
  ctx.copy_to_host(nh.data(), counts_d, sizeof(u64) * k);
  ctx.copy_to_host(ch.data(), centers_d, sizeof(float) * ch.size());
  double A = 0.0, A_abs = 0.0, B = 0.0, q_err = 0.0;
  for (int c = 0; c < k; ++c) {
    const double n = double(static_cast<long long>(nh[c]));
    double a = 0.0, aa = 0.0, b = 0.0, qe = 0.0;
    for (int f = 0; f < d; ++f) {
      const double cf = ch[size_t(c) * dp + f];
      const double s = double(static_cast<long long>(sh[size_t(c) * d + f])) * inv_scale[f];
      a += cf * s;
      aa += std::fabs(cf * s);
      b += cf * cf;
      qe += std::fabs(cf) * inv_scale[f];
    }
    A += a;
    A_abs += aa;
    B += n * b;
    q_err += n * qe;  // 2 |c| (n q / 2)
  }
  const double v = T - 2.0 * A + B;
  const double u = 1.12e-16;
  const double err = terr_abs + q_err + double(kd + k + 8) * u * (2.0 * A_abs + B) +
                     4.0 * u * (T + 2.0 * A_abs + B);
  if (!(v > 0.0) || err > kStatsCostRel * v) return false;
  *cost = v;
  return true;
}

// One fit attempt.  When the provisional fixed-point bounds fail (a row past its column's bound)
// it stores the initial centers in *restart_with and returns at once; kmeans_fit then reruns the
// fit with the column maxima's scales after this frame — and every buffer it held — has unwound.
static KMeansResult kmeans_fit_once(Context& ctx, Comm& comm, DenseTable& x,
                                    const std::vector<double>& init_centers,
                                    const KMeansParams& p, std::vector<double>* restart_with) {
  OAP_CHECK(p.k > 1 || p.init == KMeansInit::Given, "k must be > 1");
  OAP_CHECK(p.max_iter >= 0, "maxIter must be >= 0");
  if (ctx.is_gpu()) check_gpu_table(x);
  ctx.activate();
  HostMarks hm;
  KMeansResult res;
  const int d = x.cols;
  res.d = d;
  auto t_init = std::chrono::steady_clock::now();
  if (x.global_offset < 0) assign_global_offsets(ctx, comm, x);
  res.global_rows = x.global_rows;
  std::vector<double> centers;
  int k = 0;
  if (p.init == KMeansInit::Given) {
    OAP_CHECK(!init_centers.empty() && init_centers.size() % d == 0,
              "initial centers must be k x d");
    centers = init_centers;
    k = static_cast<int>(centers.size() / d);
  } else {
    centers = kmeans_init_centers(ctx, comm, x, p, &k);
  }
  res.init_seconds = seconds_since(t_init);
  res.k = k;

  // fixed-point scales (fit_bounds): provisional bounds from the initial centers, or the global
  // column maxima where a pass over the rows has to decide
  const std::vector<double> cbound = center_bounds(centers, k, d);
  const int64_t max_local =
      static_cast<int64_t>(comm_allreduce_scalar(ctx, comm, double(x.rows), ReduceOp::Max));
  std::vector<double> absmax;  // the global column maxima, once a pass computed them
  FixedPoint fp;
  auto bounds_from_absmax = [&]() {
    absmax = global_column_absmax(ctx, comm, x);
    bool fc = false;
    fp = fixed_point_scales(fit_bounds(cbound, absmax, x.global_rows, &fc), x.global_rows,
                            max_local);
    res.scale_source = fc ? "centers_checked" : "absmax";
  };
  if (!ctx.is_gpu()) bounds_from_absmax();
  const size_t kd = size_t(k) * d;
  hm.mark("setup");
  auto t_iter = std::chrono::steady_clock::now();
  Metrics& M = ctx.metrics();

  if (!ctx.is_gpu()) {
    // ------------------------------------------------------------------ CPU engine
    std::vector<int64_t> stats(kd + k);
    for (int it = 0; it < p.max_iter; ++it) {
      maybe_inject_fault(comm.rank(), "kmeans_iter", it);
      TraceRange tr(&M, "kmeans/iteration");
      auto o = cpu_assign(ctx, x, centers, k, &fp, true, true, nullptr, nullptr);
      std::copy(o.sums.begin(), o.sums.end(), stats.begin());
      std::copy(o.counts.begin(), o.counts.end(), stats.begin() + kd);
      double cost = o.cost;
      {
        TraceRange tc(&M, "kmeans/allreduce", int64_t(stats.size() * 8 + 8));
        host_allreduce(ctx, comm, stats.data(), stats.size(), DType::I64, ReduceOp::Sum);
        host_allreduce(ctx, comm, &cost, 1, DType::F64, ReduceOp::Sum);
      }
      bool conv = true;
      double max_sh = 0.0;
      for (int c = 0; c < k; ++c) {
        int64_t cnt = stats[kd + c];
        if (cnt <= 0) continue;
        double sh = 0.0;
        for (int f = 0; f < d; ++f) {
          double nv = double(stats[size_t(c) * d + f]) * fp.inv_scale[f] / double(cnt);
          double df = nv - centers[size_t(c) * d + f];
          sh += df * df;
          centers[size_t(c) * d + f] = nv;
        }
        if (sh > p.tol * p.tol) conv = false;
        max_sh = std::max(max_sh, sh);
      }
      res.cost = cost;
      res.cost_history.push_back(cost);
      res.shift_history.push_back(std::sqrt(max_sh));
      res.last_counts.assign(stats.begin() + kd, stats.end());
      res.num_iter = it + 1;
      if (conv && p.tol >= 0) {  // tol < 0: run exactly max_iter iterations
        res.converged = true;
        break;
      }
    }
    res.centers = centers;
    res.iter_seconds = seconds_since(t_iter);
    return res;
  }

  // -------------------------------------------------------------------- GPU engine
  hipStream_t s = ctx.compute();
  GpuCenters g = alloc_centers(ctx, k, d);
  Buffer c64 = ctx.alloc(sizeof(double) * kd);
  Buffer stats = ctx.alloc(sizeof(u64) * (kd + k));
  const int nslab = kern::kmeans_cost_slab_size(ctx.info().cu_count);
  Buffer slab = ctx.alloc(sizeof(double) * nslab);
  Buffer cost_d = ctx.alloc(sizeof(double));
  Buffer scale = ctx.alloc(sizeof(float) * (round_up(d, 4) + 4));
  Buffer inv_scale = ctx.alloc(sizeof(double) * d);
  // one flags slot per iteration of a batch (read back once per batch), the finalize's
  // last-block counter, the cost accumulator (zeroed by the finalize that reads it)
  Buffer flags_d = ctx.alloc(sizeof(kern::KMeansFlags) * 32);
  Buffer fin_done = ctx.alloc(sizeof(unsigned));
  ctx.memset(fin_done.data(), 0, sizeof(unsigned), s);
  ctx.memset(cost_d.data(), 0, sizeof(double), s);
  Buffer refine_d = ctx.alloc(2 * sizeof(u64));  // [exact re-decisions, tier-3 re-runs]
  Buffer counts_h = ctx.alloc_pinned(sizeof(u64) * k);
  Buffer refine_h = ctx.alloc_pinned(2 * sizeof(u64));
  ctx.memset(scale.data(), 0, sizeof(float) * (round_up(d, 4) + 4), s);
  ctx.memset(refine_d.data(), 0, 2 * sizeof(u64), s);
  ctx.copy_to_backend(c64.data(), centers.data(), sizeof(double) * kd, s);
  kern::kmeans_prepare_centers(c64.as<double>(), k, d, g.dp, g.c32.as<float>(),
                               g.cnorm.as<float>(), g.cstat.as<float>(), g.kpad, s);
  u64* sums = stats.as<u64>();
  u64* counts = sums + kd;

  AssignReq req;
  req.accumulate = true;
  req.sums_too = true;
  req.precise = p.precise;
  req.scale = scale.as<float>();
  req.sums = sums;
  req.counts = counts;
  req.cost_slab = slab.as<double>();
  req.refine_tiles = refine_d.as<u64>();
  if (!knob_str("OAP_KMEANS_CHUNK_DEFER").empty())
    req.defer = knob_int("OAP_KMEANS_CHUNK_DEFER") != 0;
  // chunked (large-k) path: labels/mindist persist across iterations to seed the merge passes
  Buffer lab_keep, mind_keep;
  const bool chunked = x.cols <= 128 && g.kpad > kern::kmeans_lds_kmax(x.cols, p.precise);
  if (chunked && x.rows > 0) {
    lab_keep = ctx.alloc(sizeof(int32_t) * x.rows);
    mind_keep = ctx.alloc(sizeof(float) * x.rows);
    req.labels = lab_keep.as<int32_t>();
    req.mindist = mind_keep.as<float>();
  }
  // the centroid-chunked lean pass runs full passes (no pruning state)
  const bool lean_chunked =
      chunked && !p.precise && g.kpad <= 1024 && !knob_on("OAP_KMEANS_NO_LEAN_CHUNKED") &&
      kern::kmeans_lloyd_chunk_kmax(x.cols) >= 32 && kern::kmeans_exact_chunk_kmax(x.cols) >= 32;
  // pruning: per-row bounds (+ labels) persist across iterations, finalize reports the drift
  const bool prune = p.prune && !p.precise && x.cols <= 128 && x.rows > 0 && !lean_chunked;
  // chunked lean pass with delta accumulation: local statistics persist, the labels alternate
  // between two buffers so the previous assignment is at hand (moved rows only)
  const bool cdelta = lean_chunked && p.delta && x.rows > 0;
  // (rank-uniform form) chunked lean iterations compute the cost only where it is reported, as
  // the single-launch delta path does: the first and a known last iteration, otherwise one
  // exact pass over the labels after the loop (a costless last chunk runs the kernel without
  // the per-row f32 distance: ~12% of the pass at 1B rows, k = 1000)
  const bool cfree_all = lean_chunked && p.delta;
  Buffer cloc_b, lab_prev_b;
  int32_t* lab_prev = nullptr;
  int64_t cmoved = 0;
  if (cdelta) {
    cloc_b = ctx.alloc(sizeof(u64) * (kd + k));
    lab_prev_b = ctx.alloc(sizeof(int32_t) * x.rows);
    lab_prev = lab_prev_b.as<int32_t>();
    req.sums = cloc_b.as<u64>();
    req.counts = cloc_b.as<u64>() + kd;
    req.stats_persist = true;
    req.moved_rows = &cmoved;
  }
  Buffer bounds_b, drift_b, pruned_d, tiles_b;
  if (prune) {
    bounds_b = ctx.alloc(sizeof(float) * 2 * x.rows);
    drift_b = ctx.alloc(sizeof(float) * (k + 1));
    pruned_d = ctx.alloc(sizeof(u64));
    ctx.memset(pruned_d.data(), 0, sizeof(u64), s);
    if (!req.labels) {
      lab_keep = ctx.alloc(sizeof(int32_t) * x.rows);
      req.labels = lab_keep.as<int32_t>();
    }
    req.bounds = bounds_b.as<float>();
    req.pruned_tiles = pruned_d.as<u64>();
    if (chunked) {
      tiles_b = ctx.alloc(sizeof(int32_t) * ((x.rows + 31) / 32) + 64);
      req.tile_list = tiles_b.as<int32_t>();
      req.tile_count = reinterpret_cast<unsigned*>(tiles_b.as<char>() +
                                                   sizeof(int32_t) * ((x.rows + 31) / 32));
    }
  }

  // delta accumulation (single launch + pruning): persistent local statistics, max |x|^2 per tile,
  // the scan's tile list, and the centers each iteration assigned against (final exact cost)
  // (rank-uniform form: a rank with no rows still joins the final-cost collective)
  // Delta accumulation (lean kernel): iterations after the first keep each rank's local
  // statistics and add only the rows whose label changed (+x to the new, -x to the old cluster;
  // integers, so bitwise the full recount).  Two forms per iteration: a full pass (every row
  // assigned and costed, unmoved rows not re-accumulated) or, with pruning, a scan pass (the
  // bounds scan lists the tiles that may change; only those are read, the cost is not
  // computed).  delta_all / scan_all are rank-uniform (a rank with no rows still joins the
  // final-cost collective).
  const bool delta_all = !p.precise && x.cols <= 128 && !chunked && p.delta &&
                         kern::kmeans_lloyd_supported(d, k, true, true);
  const bool scan_all = delta_all && p.prune;
  const bool delta = delta_all && x.rows > 0;
  const bool scan = scan_all && prune;
  if (delta && !req.labels) {
    lab_keep = ctx.alloc(sizeof(int32_t) * x.rows);
    req.labels = lab_keep.as<int32_t>();
  }
  // Provisional fixed-point bounds (fit_bounds): the lean single-launch fit's first full pass
  // checks every row against them (and sums |x|^2 for the final cost), so no pass over the rows
  // runs before the first iteration.  Decided from the shape and parameters (rank-uniform).
  // (a feature that is 0 in every initial center has bound 0, which every row would fail: the
  // check could only flag and restart, so such a fit takes the column maxima up front — the
  // rule fit_bounds evaluates then is the same on every engine)
  double cb_min = std::numeric_limits<double>::infinity();
  for (int f = 0; f < d; ++f) cb_min = std::min(cb_min, cbound[f]);
  const bool provisional = !p.absmax_pass && !knob_on("OAP_KMEANS_ABSMAX_PASS") && delta_all &&
                           provisional_allowed(x.global_rows, d) && cb_min > 0.0 &&
                           x.dtype == DType::F32 && lean_applies(x, k, g.kpad, req);
  Buffer bflag_b, sq_slab_b;
  if (provisional) {
    fp = fixed_point_scales(cbound, x.global_rows, max_local);
    res.scale_source = "centers";
    bflag_b = ctx.alloc(2 * sizeof(unsigned));  // [flag, largest fp32 |x|^2 (bits)]
    ctx.memset(bflag_b.data(), 0, 2 * sizeof(unsigned), s);
  } else {
    bounds_from_absmax();
  }
  ctx.copy_to_backend(scale.data(), fp.scale.data(), sizeof(float) * d, s);
  ctx.copy_to_backend(inv_scale.data(), fp.inv_scale.data(), sizeof(double) * d, s);
  bool prov_pending = provisional;  // the first batch's check is still to be read
  Buffer loc_b, xnorm_b, dlist_b, cbak_b;
  const int lgrid = kern::kmeans_lloyd_grid(x.rows, ctx.info().cu_count);
  // sum |x|^2 of the local rows, fused into the first full pass (the final cost's statistics
  // form): one fp64 partial per lean workgroup
  if (delta_all && x.rows > 0 && x.dtype == DType::F32 && lean_applies(x, k, g.kpad, req))
    sq_slab_b = ctx.alloc(sizeof(double) * lgrid);
  bool sq_ready = false;
  const int64_t ltiles = kern::kmeans_lloyd_tiles_per_block(x.rows, lgrid);
  if (delta) {
    loc_b = ctx.alloc(sizeof(u64) * (kd + k));
    req.sums = loc_b.as<u64>();
    req.counts = loc_b.as<u64>() + kd;
  }
  if (scan) {
    const int64_t nt = (x.rows + 31) / 32;
    xnorm_b = ctx.alloc(sizeof(float) * nt);
    dlist_b = ctx.alloc(sizeof(int32_t) * size_t(lgrid) * size_t(ltiles) +
                        sizeof(unsigned) * size_t(lgrid) + 64);
    req.xnorm = xnorm_b.as<float>();
  }
  if (delta || cdelta) cbak_b = ctx.alloc(sizeof(float) * size_t(g.kpad) * g.dp);
  // Row-level scan (image passes): per row, the Hamerly test the tile scan applies to whole
  // 32-row tiles; the image kernel then gathers only the rows it could not prune.  On overlapping
  // clusters a tile almost always holds a row near a boundary, while most rows are far from one
  // (headline data: tiles 0-13% prunable, rows up to 93%: profiles/r4/row_prune_potential.jsonl).
  // Bounds are then written by every pass.  The scan runs inside the image kernel (each wave
  // tests its own rows and queues the unpruned ones in LDS) where the kernel's LDS plan has room
  // for it; knob OAP_KMEANS_ROW_SCAN=0 takes the tile scan.  (A separate scan kernel writing
  // row lists through HBM cost more than it saved: profiles/r4/trace_bench_r4f_separate_scan.txt.)
  Buffer rpruned_b, scan_gate_b;
  const bool row_scan = scan && !chunked && knob_int("OAP_KMEANS_ROW_SCAN") != 0;
  if (row_scan) {
    rpruned_b = ctx.alloc(sizeof(u64));
    ctx.memset(rpruned_b.data(), 0, sizeof(u64), s);
    scan_gate_b = ctx.alloc(sizeof(int) * 4);
    ctx.memset(scan_gate_b.data(), 0, sizeof(int) * 4, s);
  }
  unsigned* dcount =
      scan ? reinterpret_cast<unsigned*>(dlist_b.as<int32_t>() + size_t(lgrid) * size_t(ltiles))
           : nullptr;
  bool last_scanned = false;  // the last iteration was a scan pass (its cost is not computed)
  // lean tier-1 path: persistent deferral list + a counter of deferred rows (adaptive tier)
  Buffer ldefer_b, ldstat_b, ldstat_h;
  if (x.rows > 0 && lean_applies(x, k, g.kpad, req)) {
    int lg = 0;
    int64_t lcap = 0;
    ldefer_b =
        ctx.alloc(lean_defer_bytes(x.rows, x.cols, g.kpad, ctx.info().cu_count, &lg, &lcap));
    req.defer_rows = ldefer_b.as<int32_t>();
    req.defer_count = reinterpret_cast<unsigned*>(req.defer_rows + size_t(lg) * size_t(lcap));
  }
  if (x.rows > 0 && (req.defer_rows || lean_chunked)) {
    // [deferred rows, moved rows staged, passes that read the operand image]
    ldstat_b = ctx.alloc(5 * sizeof(u64));
    ldstat_h = ctx.alloc_pinned(5 * sizeof(u64));
    ctx.memset(ldstat_b.data(), 0, 5 * sizeof(u64), s);
    req.deferred_rows = ldstat_b.as<u64>();
  }
  u64 deferred_seen = 0, moved_seen = 0;
  // Resident fp16 operand image (f32 rows, delta path): the first full lean pass writes each
  // tile's MFMA B operand (fp16 of beta x + bias slots, 2 B per padded feature instead of 4) and
  // the delta passes after it stream that instead of the f32 rows — 128 instead of 208 B per
  // row at d = 50 — reading f32 rows only for moved rows and the exact re-decisions.  Taken
  // when the image fits beside the arena's other buffers with a quarter of its budget to spare.
  Buffer img_b, img_beta_b;
  bool img_ready = false;
  // (the fallback check: the image scale read back into pinned memory)
  Buffer imgchk_h = ctx.alloc_pinned(sizeof(float));
  bool imgchk_pending = false;
  // >= every row's |x| on every rank: the global column maxima's norm, or (provisional bounds)
  // the smallest bound, which the first pass's check proves above every row's norm
  auto norm_cap_of = [](const std::vector<double>& am) {
    double c = 0.0;
    for (double v : am) c += v * v;
    return std::isfinite(c) ? std::sqrt(c) : 1e300;
  };
  double row_norm_cap = provisional ? norm_cap_of(cbound) : norm_cap_of(absmax);
  double init_cmax = 0.0;  // the largest |c| of the initial centers
  for (int c = 0; c < k; ++c) {
    double s2 = 0.0;
    for (int f = 0; f < d; ++f) s2 += centers[size_t(c) * d + f] * centers[size_t(c) * d + f];
    init_cmax = std::max(init_cmax, std::sqrt(s2));
  }
  {
    const size_t ib = kern::kmeans_lloyd_image_bytes(x.rows, x.cols);
    DeviceArena* ar = ctx.backend() == Backend::GPU ? ctx.arena() : nullptr;
    if (delta && req.defer_rows && x.dtype == DType::F32 && ib > 0 &&
        knob_int("OAP_KMEANS_IMAGE") != 0 && ar &&
        ar->used() + ib + ar->budget() / 4 <= ar->budget()) {
      img_b = ctx.alloc(ib);
      img_beta_b = ctx.alloc(sizeof(float) * 4);
      res.image_bytes = static_cast<int64_t>(ib);
    }
  }
  // (row-scan mode needs the image and the image kernel at this shape; rank-uniform in practice:
  // every rank decides from the same shape, and a rank without rows scans nothing)
  bool row_scan_ok = false;
  if (row_scan && img_b.data()) {
    const int lw = kern::kmeans_lloyd_waves(lean_variant(d, g.kpad));
    row_scan_ok = kern::kmeans_lean_img_supported(d, k, lw, true);
  }
  // the same decision for the whole world (it changes which iterations compute a cost and
  // scan tiles, and so which collectives run): every rank with rows must have the image and the
  // kernel (a rank without rows abstains) — one scalar Min-allreduce per fit; a rank whose own
  // image is there still leaves the row scan off when a peer's is not
  double rs_vote = (x.rows == 0 || row_scan_ok) ? 1.0 : 0.0;
  if (!comm.trivial()) rs_vote = comm_allreduce_scalar(ctx, comm, rs_vote, ReduceOp::Min);
  const bool row_scan_all = scan_all && !chunked && rs_vote > 0.5 &&
                            (row_scan_ok || x.rows == 0 || !comm.trivial());
  row_scan_ok = row_scan_ok && row_scan_all;
  // with the adaptive scan off, full passes write the per-row bounds (8 B/row) only where a
  // following iteration may scan, and the per-tile max |x|^2 (constant) once
  float* const bounds_full = req.bounds;
  float* const xnorm_full = req.xnorm;
  bool xnorm_ready = false;
  // adaptive delta: when the scan prunes few tiles (overlapping clusters), its pass and the
  // delta bookkeeping cost more than they save — run full passes (which refresh labels and
  // bounds) and probe the scan again every few iterations
  // (a scan that prunes nothing backs off exponentially: probes every probe_gap batches, the
  // gap doubling after each failed probe, so an overlapping-cluster fit pays for at most a few
  // scans and otherwise runs exactly the unpruned delta path)
  bool delta_on = true;
  bool probing = false;  // delta_on was set by a probe: scan one iteration, then decide
  int delta_probe = 0;
  // With a tolerance (tol >= 0) the fit batches too where every kernel of an iteration can stand
  // down on the device: the finalize of a converged iteration sets `halt`, and the lean / image /
  // exact / scan kernels, the finalize and the guarded copies of the iterations enqueued behind
  // it return at once — so the host reads the flags once per batch, not once per iteration.
  // That needs the delta form of the lean path: the local statistics persist and reach the
  // global ones by an out-of-place reduction (or a copy before an in-place one), so an iteration
  // that does nothing leaves every result as the converged one left it.  (A host communicator
  // still syncs inside each allreduce; batching saves it the per-iteration flag read-backs and
  // scalar collectives.)  Rank-uniform: delta_all and req.fast1 (decided from allreduced values)
  // are the same on every rank.
  const bool tol_batch_ok = p.tol >= 0 && delta_all;
  const int probe_gap0 = p.tol < 0 || tol_batch_ok ? 1 : 4;  // (batches vs single iterations)
  int probe_gap = probe_gap0;

  kern::KMeansFinalizeArgs fa;
  // a single-rank delta fit finalizes straight from its local statistics (no copy into the
  // allreduce buffer: there is no allreduce)
  const bool fin_direct = delta && comm.trivial();
  u64* const fin_counts = fin_direct ? loc_b.as<u64>() + kd : counts;
  fa.sums = fin_direct ? loc_b.as<u64>() : sums;
  fa.counts = fin_counts;
  fa.inv_scale = inv_scale.as<double>();
  fa.centers64 = c64.as<double>();
  fa.centers32 = g.c32.as<float>();
  fa.cnorm = g.cnorm.as<float>();
  fa.cstat = g.cstat.as<float>();
  fa.k = k;
  fa.d = d;
  fa.dp = g.dp;
  fa.tol = p.tol;
  fa.cost_in = cost_d.as<double>();
  fa.cost_reset = cost_d.as<double>();
  fa.flags = flags_d.data();
  Buffer fin_scratch = ctx.alloc(sizeof(double) * 2 * std::max(k, 1));
  fa.scratch = fin_scratch.as<double>();
  fa.done = fin_done.as<unsigned>();
  if (prune) fa.drift = drift_b.as<float>();
  // per-phase events (assign / allreduce / rest) in every iteration, or only one pair per
  // batch: an event record is a gap of ~10 us in the stream, a measurable share of an
  // iteration on a 12.5M-row shard
  const bool pev = p.phase_events;

  RcclComm* rccl = dynamic_cast<RcclComm*>(&comm);
  const int64_t flops_per_iter = 2 * int64_t(x.rows) * k * d;
  // With a tolerance the host must see each iteration's convergence flag before deciding to
  // launch the next one (batch of 1).  tol < 0 means "exactly max_iter iterations": then up to
  // kBatch iterations are enqueued back to back (kernels + collective, no host round trip in
  // between) and their flags / timings are read once per batch — the host re-checks the
  // adaptive distance tier at every batch boundary.
  // (32: a 20-iteration fit has 2 batch boundaries — each a host round trip, ~130 us with its
  // read-backs; flags_d slots)
  constexpr int kBatch = 32;
  auto batch_size = [&]() { return p.tol < 0 || (tol_batch_ok && req.fast1) ? kBatch : 1; };
  Buffer halt_b;
  if (tol_batch_ok) {
    halt_b = ctx.alloc(sizeof(int) * 4);
    ctx.memset(halt_b.data(), 0, sizeof(int) * 4, s);
  }
  // the batch's adaptive controls (kern::kmeans_ctl), Max-allreduced with its last iteration
  Buffer ctl_b = ctx.alloc(sizeof(double) * 8);
  Buffer ctl_snap = ctx.alloc(sizeof(u64) * 4);
  Buffer ctl_h = ctx.alloc_pinned(sizeof(double) * 8);
  ctx.memset(ctl_snap.data(), 0, sizeof(u64) * 4, s);
  struct IterEvents {
    Event e0, e1, e2, e3;
  };
  std::vector<IterEvents> ev(kBatch);
  Buffer flags_hb = ctx.alloc_pinned(sizeof(kern::KMeansFlags) * kBatch);
  // (declared after every pinned read-back buffer of the fit: destroyed before them)
  StreamDrainOnUnwind drain_on_unwind{s};
  auto* flh = flags_hb.as<kern::KMeansFlags>();
  bool stop = false;
  bool restart = false;  // the provisional fixed-point bounds failed (see prov_pending)
  int scan_iters = 0;  // scan passes in the current batch
  std::vector<char> it_scanned(kBatch, 0), it_costless(kBatch, 0);
  bool last_costless = false;  // the last iteration computed no cost (rank-uniform)
  hm.mark("buffers");
  for (int it0 = 0, nb_it = 0; it0 < p.max_iter && !stop; it0 += nb_it) {
    // the first batch is short so the adaptive choices (tier, scan) are made early
    // (with the scan on, the first batch ends after the first delta iteration: its moved-row
    // share gates the first scan probe)
    const int Bn = batch_size();
    nb_it = std::min(it0 == 0 && Bn > 3 ? (scan_all ? 2 : 3) : Bn, p.max_iter - it0);
    scan_iters = 0;
    // (the halt word applies to batches of more than one iteration with a tolerance)
    int* const halt = tol_batch_ok && Bn > 1 ? halt_b.as<int>() : nullptr;
    req.halt = halt;
    fa.halt = halt;
    for (int b = 0; b < nb_it; ++b) {
      const int it = it0 + b;
      maybe_inject_fault(comm.rank(), "kmeans_iter", it);
      roctx_push("kmeans/iteration");
      if (pev || b == 0) ev[b].e0.record(s);
      // (req.fast1: the lean kernel runs; only it does delta accumulation)
      const bool delta_it = delta && it > 0 && req.fast1;
      // (a probe batch scans its first iteration only: the next batch decides from it)
      // (the first batch scans its third iteration only: one right after the init's large
      // move rarely prunes)
      // (rank-uniform: row_scan_all, not row_scan_ok — the latter also needs this rank's rows
      // and its image allocation, so a rank without rows or without room for the image would
      // count tile-scan iterations its peers do not, and the per-batch collectives below that
      // scan_iters gates would pair up differently across ranks)
      const bool scan_it_all = scan_all && it > 1 && req.fast1 && delta_on && !row_scan_all &&
                               (!probing || b == 0);
      const bool scan_it = scan_it_all && scan;
      last_scanned = scan_it_all;
      it_scanned[b] = scan_it_all;
      scan_iters += scan_it_all ? 1 : 0;
      if (!delta_it && !cdelta)  // (the chunked lean pass zeroes its own on a recount)
        OAP_HIP_CHECK(hipMemsetAsync(delta ? loc_b.data() : stats.data(), 0,
                                     sizeof(u64) * (kd + k), s));
      req.labels_valid = it > 0;
      if (cdelta) {
        if (req.fast1) {  // the chunked lean pass runs: it writes the other label buffer
          std::swap(req.labels, lab_prev);
          req.prev_labels = it > 0 ? lab_prev : nullptr;
        } else {  // the general chunked path (adaptive tier off) accumulates from zero
          req.prev_labels = nullptr;
          OAP_HIP_CHECK(hipMemsetAsync(cloc_b.data(), 0, sizeof(u64) * (kd + k), s));
        }
      }
      if (scan_all && prune) {
        const bool next_may_scan =
            it >= 1 && (b < nb_it - 1 ? delta_on && !probing
                                      : delta_on || delta_probe + 1 >= probe_gap);
        req.bounds = (scan_it || next_may_scan || row_scan_ok) ? bounds_full : nullptr;
        req.xnorm = xnorm_ready ? nullptr : xnorm_full;
      }
      if (prune) {
        // the general kernel's in-kernel pruning test (lean off) or the scan read the drift;
        // a lean full pass refreshes labels and bounds without it
        const bool drift_in = it > 0 && (scan_it || !req.fast1 || !delta_all);
        req.drift = drift_in ? drift_b.as<float>() : nullptr;
        req.drift_max = drift_in ? drift_b.as<float>() + k : nullptr;
      }
      req.delta = delta_it;
      // lean iterations compute the exact cost only where it is reported: the first and a
      // known last iteration (fixed count); otherwise the final cost comes from one exact pass
      // over the labels after the loop
      // (with the row scan, a known last iteration is a scan pass too: the exact cost pass over
      // the labels after the loop reads the f32 rows once, cheaper than a full f32 cost pass)
      const bool cost_it = !req.fast1 || !(delta_all || cfree_all) || it == 0 ||
                           (p.tol < 0 && it == p.max_iter - 1 && !row_scan_all);
      req.cost_slab = cost_it ? slab.as<double>() : nullptr;
      it_costless[b] = !cost_it || scan_it_all;
      last_costless = it_costless[b];
      if (scan_it) {
        OAP_CHECK(xnorm_ready, "kmeans scan before any full pass");
        kern::kmeans_lean_scan(x.rows, k, d, lgrid, req.bounds, req.labels, xnorm_full,
                               req.drift, req.drift_max, g.cstat.as<float>(),
                               dlist_b.as<int32_t>(), dcount, req.pruned_tiles, s, halt);
        req.tile_list = dlist_b.as<int32_t>();
        req.tile_count = dcount;
      } else if (!chunked) {
        req.tile_list = nullptr;
        req.tile_count = nullptr;
      }
      // row-level scan ahead of an image pass (the drift finalize wrote for the previous step)
      const bool row_scan_it = row_scan_ok && delta_it && it > 1 && img_ready && !cost_it &&
                               req.fast1 && !req.tile_list;
      req.img_scan_xnorm = nullptr;
      req.img_scan_drift = nullptr;
      req.img_scan_pruned = nullptr;
      req.img_gate = nullptr;
      if (row_scan_it) {
        OAP_CHECK(xnorm_ready && bounds_full, "kmeans row scan before any full pass");
        req.img_scan_xnorm = xnorm_full;
        req.img_scan_drift = drift_b.as<float>();
        req.img_scan_pruned = rpruned_b.as<u64>();
        if (p.scan_min_prune > 0.0) {
          // scan or dense, decided on the device from a sample of the rows
          kern::kmeans_scan_decide(x.rows, k, d, bounds_full, req.labels, xnorm_full,
                                   drift_b.as<float>(), g.cstat.as<float>(),
                                   float(p.scan_min_prune), scan_gate_b.as<int>(), halt, s);
          req.img_gate = scan_gate_b.as<int>();
        }
      }
      // operand image: written by the first full lean pass, read by costless delta passes
      req.ximg = img_b.data();
      req.img_beta = img_beta_b.as<float>();
      req.img_mode = 0;
      if (img_b.data() && lean_applies(x, k, g.kpad, req)) {
        if (!img_ready && !req.tile_list && req.cost_slab)
          req.img_mode = 1;
        else if (img_ready && delta_it && !req.cost_slab && !req.mindist && !req.xnorm)
          req.img_mode = 2;
      }
      // (the lean chunked pass keeps its running state in its own buffers: no per-row distance
      // unless a cost is asked for; the general chunked path re-seeds its own each iteration)
      if (lean_chunked && x.rows > 0) req.mindist = req.fast1 ? nullptr : mind_keep.as<float>();
      // the first full pass: sum |x|^2 (final cost) and the provisional-bound check
      const bool first_full = it == 0 && !req.tile_list && !req.delta && req.fast1;
      req.sq_slab = first_full && sq_slab_b.data() ? sq_slab_b.as<double>() : nullptr;
      req.bound_flag = first_full && prov_pending ? bflag_b.as<unsigned>() : nullptr;
      req.bound_inf = float(cb_min);  // (a power of two, or 0 / inf)
      OAP_CHECK(!(it == 0 && prov_pending && x.rows > 0) ||
                    (req.bound_flag && lean_applies(x, k, g.kpad, req)),
                "kmeans: the provisional fixed-point bounds need the lean first pass");
      int nb = gpu_assign(ctx, x, g, req, s);
      if (req.sq_slab) sq_ready = true;
      req.sq_slab = nullptr;
      req.bound_flag = nullptr;
      if (req.img_mode == 1) {
        img_ready = true;
        // the image's scale, read back with the batch: whether the f32 fallback launch
        // after every image pass can be retired (below)
        OAP_HIP_CHECK(hipMemcpyAsync(imgchk_h.data(), img_beta_b.data(), sizeof(float),
                                     hipMemcpyDeviceToHost, s));
        imgchk_pending = true;
      }
      if (cdelta) {
        OAP_HIP_CHECK(hipMemcpyAsync(stats.data(), cloc_b.data(), sizeof(u64) * (kd + k),
                                     hipMemcpyDeviceToDevice, s));
        if (p.tol >= 0 || it == p.max_iter - 1)  // (the final exact-cost pass's centers)
          OAP_HIP_CHECK(hipMemcpyAsync(cbak_b.data(), g.c32.data(),
                                       sizeof(float) * size_t(g.kpad) * g.dp,
                                       hipMemcpyDeviceToDevice, s));
      }
      if (req.xnorm && !req.tile_list) xnorm_ready = true;
      // (a device communicator reduces the local statistics out of place into stats)
      const bool stats_oop = delta && !fin_direct && comm.on_device();
      if (delta) {
        if (!fin_direct && !stats_oop)
          OAP_HIP_CHECK(hipMemcpyAsync(stats.data(), loc_b.data(), sizeof(u64) * (kd + k),
                                       hipMemcpyDeviceToDevice, s));
        // the centers this iteration assigned against, for the final exact-cost pass — only
        // when it may follow this iteration (a convergence test, or the last iteration); in a
        // batch behind a converged iteration it must keep that iteration's centers
        if (p.tol >= 0 || it == p.max_iter - 1) {
          if (halt)
            kern::copy_guarded(cbak_b.data(), g.c32.data(), sizeof(float) * size_t(g.kpad) * g.dp,
                               halt, s);
          else
            OAP_HIP_CHECK(hipMemcpyAsync(cbak_b.data(), g.c32.data(),
                                         sizeof(float) * size_t(g.kpad) * g.dp,
                                         hipMemcpyDeviceToDevice, s));
        }
      }
      // (otherwise cost_d holds the zero the last finalize left: a costless iteration's cost
      // is not reported)
      if (nb > 0) kern::sum_f64(slab.as<double>(), nb, cost_d.as<double>(), s);
      if (pev) ev[b].e1.record(s);
      // the batch's adaptive controls, from the device counters, ride its last allreduce
      const bool ctl_it = b == nb_it - 1;
      if (ctl_it) {
        kern::KMeansCtlArgs ca;
        ca.refine = refine_d.as<u64>();
        ca.ldstat = ldstat_b.data() ? ldstat_b.as<u64>() : nullptr;
        ca.pruned = scan ? pruned_d.as<u64>() : nullptr;
        ca.bound_flag = prov_pending ? bflag_b.as<unsigned>() : nullptr;
        ca.snap = ctl_snap.as<u64>();
        ca.out = ctl_b.as<double>();
        ca.rows = x.rows;
        ca.nb_it = nb_it;
        ca.scan_iters = scan_iters;
        ca.scan_local = scan ? 1 : 0;
        kern::kmeans_ctl(ca, s);
      }
      if (!comm.trivial()) {
        if (comm.on_device()) {
          if (rccl) rccl->group_start();
          if (stats_oop)
            comm.allreduce_oop(loc_b.data(), stats.data(), kd + k, DType::I64, ReduceOp::Sum,
                               s);
          else
            comm.allreduce(stats.data(), kd + k, DType::I64, ReduceOp::Sum, s);
          comm.allreduce(cost_d.data(), 1, DType::F64, ReduceOp::Sum, s);
          if (ctl_it) comm.allreduce(ctl_b.data(), 5, DType::F64, ReduceOp::Max, s);
          if (rccl) rccl->group_end();
        } else {
          comm_allreduce(ctx, comm, stats.data(), kd + k, DType::I64, ReduceOp::Sum, s);
          comm_allreduce(ctx, comm, cost_d.data(), 1, DType::F64, ReduceOp::Sum, s);
          if (ctl_it) comm_allreduce(ctx, comm, ctl_b.data(), 5, DType::F64, ReduceOp::Max, s);
        }
      }
      if (pev) ev[b].e2.record(s);
      fa.flags = flags_d.as<kern::KMeansFlags>() + b;
      kern::kmeans_finalize(fa, s);
      if (pev || b == nb_it - 1) ev[b].e3.record(s);
      roctx_pop();
    }
    OAP_HIP_CHECK(hipMemcpyAsync(flh, flags_d.data(), sizeof(kern::KMeansFlags) * nb_it,
                                 hipMemcpyDeviceToHost, s));
    OAP_HIP_CHECK(
        hipMemcpyAsync(counts_h.data(), fin_counts, sizeof(u64) * k, hipMemcpyDeviceToHost, s));
    OAP_HIP_CHECK(hipMemcpyAsync(refine_h.data(), refine_d.data(), 2 * sizeof(u64),
                                 hipMemcpyDeviceToHost, s));
    OAP_HIP_CHECK(
        hipMemcpyAsync(ctl_h.data(), ctl_b.data(), 5 * sizeof(double), hipMemcpyDeviceToHost, s));
    const double* ctl = ctl_h.as<double>();
    if (ldstat_b.data())
      OAP_HIP_CHECK(hipMemcpyAsync(ldstat_h.data(), ldstat_b.data(), 5 * sizeof(u64),
                                   hipMemcpyDeviceToHost, s));
    comm.wait(s);
    if (prov_pending) {
      // the first pass's check of the provisional bounds (rank-uniform: allreduced); a flagged
      // row costs one column-maxima pass, which evaluates the rule exactly — the bounds either
      // hold (continue) or the fit restarts from its initial centers with the column maxima
      prov_pending = false;
      // (allreduced with the batch: the flag, and every row's norm on every rank — the largest
      // fp32 |x|^2, relative error <= (d + 1) 2^-24, kern::kmeans_ctl)
      const double fl = ctl[3];
      const double ncap = ctl[4];
      if (std::isfinite(ncap)) row_norm_cap = std::min(row_norm_cap, ncap);
      if (fl > 0.0) {
        absmax = global_column_absmax(ctx, comm, x);
        bool fc = false;
        (void)fit_bounds(cbound, absmax, x.global_rows, &fc);
        if (!fc) {
          restart = true;
          break;
        }
        res.scale_source = "centers_checked";
        row_norm_cap = norm_cap_of(absmax);
      }
    }
    if (imgchk_pending) {
      // every later center is a mean of rows (of any rank) or a center that never moved, so
      // its norm stays below the larger of the global column-max bound on the rows' norms and
      // the initial centers' largest (margin for the fp32 means): then the image's scale holds
      // every later plane and kmeans_lloyd's img_mode-3 fallback (a launch that would exit at
      // once) is not needed
      imgchk_pending = false;
      if (double(imgchk_h.as<float>()[0]) * std::max(row_norm_cap, init_cmax) * 1.001 <= 512.0)
        req.img_fallback = false;
    }
    const float ms_batch = pev ? 0.f : Event::elapsed_ms(ev[0].e0, ev[nb_it - 1].e3);
    for (int b = 0; b < nb_it; ++b) {
      const int it = it0 + b;
      const float ms_assign = pev ? Event::elapsed_ms(ev[b].e0, ev[b].e1) : 0.f,
                  ms_comm = pev ? Event::elapsed_ms(ev[b].e1, ev[b].e2) : 0.f,
                  ms_all = pev ? Event::elapsed_ms(ev[b].e0, ev[b].e3) : ms_batch / nb_it;
      if (pev) {
        M.add("kmeans/assign_kernel", ms_assign * 1e3, int64_t(x.bytes()));
        M.add("kmeans/allreduce", ms_comm * 1e3, int64_t(kd + k) * 8 + 8);
      }
      M.add("kmeans/iteration", ms_all * 1e3);
      const kern::KMeansFlags& fl = flh[b];
      if (Logger::instance().level() <= LogLevel::Info) {
        std::ostringstream os;
        os << "\"iter\":" << it << ",\"cost\":" << fl.cost << ",\"assign_us\":" << ms_assign * 1e3
           << ",\"allreduce_us\":" << ms_comm * 1e3 << ",\"tflops\":"
           << (ms_assign > 0 ? double(flops_per_iter) / (ms_assign * 1e-3) / 1e12 : 0.0);
        Logger::instance().log(LogLevel::Info, "kmeans/iteration", os.str());
      }
      // scan iterations sum the cost of the tiles they read only: not a cost
      const double c_it = it_costless[b] ? std::numeric_limits<double>::quiet_NaN() : fl.cost;
      res.cost = c_it;
      res.cost_history.push_back(c_it);
      res.shift_history.push_back(std::sqrt(std::max(fl.max_shift2, 0.0)));
      res.num_iter = it + 1;
      if (fl.converged && p.tol >= 0) {
        // (iterations enqueued past it in the batch stood down on the device: halt)
        res.converged = true;
        last_costless = it_costless[b];
        stop = true;
        break;
      }
    }
    if (req.fast1 && !stop) {
      // adaptive tier (rank-uniform: the largest local share decides): tier-1 first pays off
      // only while the re-decisions it leaves stay rare — tier-3 tile re-runs (general kernel)
      // or deferred rows (lean kernel)
      // (the batch's largest local share over the ranks, kern::kmeans_ctl)
      const double share = ctl[0];
      if (ldstat_b.data() && Logger::instance().level() <= LogLevel::Info) {
        Logger::instance().log(
            LogLevel::Info, "kmeans/batch_rows",
            "\"iters\":[" + std::to_string(it0) + "," + std::to_string(it0 + nb_it - 1) +
                "],\"deferred\":" + std::to_string(ldstat_h.as<u64>()[0] - deferred_seen) +
                ",\"moved\":" + std::to_string(ldstat_h.as<u64>()[1] - moved_seen));
      }
      if (ldstat_b.data()) {
        deferred_seen = ldstat_h.as<u64>()[0];
        moved_seen = ldstat_h.as<u64>()[1];
      }
      if (share > 1.0) {
        req.fast1 = false;
        Logger::instance().log(LogLevel::Info, "kmeans/tier1_off",
                               "\"iter\":" + std::to_string(res.num_iter - 1));
      }
    }
    if (scan_all && !stop) {  // adaptive scan (decided per batch from its pruned share);
      // rank-uniform: ranks see the same drift but their own rows, so the smallest local share
      // decides (a rank without rows reports 1)
      // (the smallest local pruned share over the ranks, kern::kmeans_ctl)
      const double frac = scan_iters > 0 ? -ctl[1] : 0.0;
      // (one scan right after a large move says little: turn off on two, or on a hopeless one)
      const bool was_probe = probing;
      probing = false;
      // first batch (iterations 0-1, no scan yet): with more than 3% of the rows moving in the
      // first delta iteration at most (0.97)^32 of the 32-row tiles can be free of movers — the
      // first scan would prune almost nothing (overlapping clusters) and costs a bound write,
      // a scan and a listed pass: back off as after a hopeless probe
      if (it0 == 0 && scan_iters == 0 && delta_on && nb_it >= 2) {  // (rank-uniform)
        const double mv = ctl[2];  // (the largest moved share over the ranks)
        if (mv > 0.03) {
          delta_on = false;
          delta_probe = 0;
          probe_gap = std::min(std::max(probe_gap * 2, 4 * probe_gap0), 64);
        }
      }
      if (delta_on && scan_iters > 0 &&
          (frac < 0.02 || ((scan_iters > 1 || was_probe) && frac < 0.2))) {
        delta_on = false;
        delta_probe = 0;
        // nothing pruned: wait 4x the base gap before probing again; each failed probe doubles
        if (frac < 0.02) probe_gap = std::min(std::max(probe_gap * 2, 4 * probe_gap0), 64);
        else if (was_probe) probe_gap = std::min(probe_gap * 2, 16 * probe_gap0);
      } else if (delta_on && scan_iters > 0) {
        probe_gap = probe_gap0;
      } else if (!delta_on && ++delta_probe >= probe_gap) {
        delta_on = true;  // probe: the centers may have settled
        probing = batch_size() > 1;
      }
    }
  }
  hm.mark("loop");
  if (restart) {
    // a row beyond the provisional bounds: the first batch's integers may have wrapped — the
    // fit runs again from its initial centers with the column maxima's scales (rare: rows
    // far outside every initial center's coordinate range)
    OAP_HIP_CHECK(hipStreamSynchronize(s));
    OAP_CHECK(restart_with != nullptr, "kmeans: the restarted fit failed its bounds again");
    *restart_with = centers;
    return res;
  }
  if ((delta_all || cfree_all) && last_costless && res.num_iter > 1) {
    // exact cost of a last scan iteration: every row against the centers it was assigned to,
    // with the assign kernel's per-row fp32 arithmetic (kmeans_label_cost), summed in fp64
    TraceRange tc(&M, "kmeans/final_cost", int64_t(x.bytes()));
    Buffer md;  // outlives the copy_to_host below (which synchronizes the stream)
    // (rank-uniform: the dtype, the shape and the env are; the helper's inputs are global)
    double c_stats = 0.0;
    // (knob OAP_KMEANS_FINAL_COST=rows: the per-row pass)
    const bool try_stats =
        delta_all && x.dtype == DType::F32 && knob_str("OAP_KMEANS_FINAL_COST")[0] != 'r';
    double fused_T[2] = {0.0, 0.0};  // {sum |x|^2 of the local rows, its relative bound}
    const bool fused = sq_ready || x.rows == 0;
    if (sq_ready) {
      std::vector<double> h(lgrid);
      ctx.copy_to_host(h.data(), sq_slab_b.data(), sizeof(double) * lgrid, s);
      for (double v : h) fused_T[0] += v;  // (fixed order)
      // each row's fp32 |x|^2 errs by <= (8 KS + 1) 2^-24 of itself (its fma chain over a half
      // row, the two halves' add; KS <= 8); then fp64 additions of non-negative terms: one per
      // tile a lane ran (>= 8 waves per workgroup), the wave's shuffle tree, the workgroup's
      // waves, the host's workgroups
      const double chain = double((ltiles + 7) / 8 + 6 + 16 + lgrid + 2);
      fused_T[1] = double(8 * ((d + 4 + 15) / 16) + 1) * 5.97e-8 * (1.0 + 1e-6) +
                   chain * 1.12e-16;
    }
    if (try_stats && final_cost_from_stats(ctx, comm, x, fa.sums, fa.counts, cbak_b.as<float>(),
                                           k, d, g.dp, fp.inv_scale, fused ? fused_T : nullptr,
                                           &c_stats)) {
      res.cost = c_stats;
      res.cost_history.back() = c_stats;
      res.final_cost_path = "stats";
    } else {
      res.final_cost_path = "rows";
      if (!delta && !cdelta) {
        OAP_HIP_CHECK(hipMemsetAsync(cost_d.data(), 0, sizeof(double), s));
      } else {
        kern::KMeansAssignArgs ca;
        ca.x = x.data.data();
        ca.xbf16 = x.dtype == DType::BF16;
        ca.n = x.rows;
        ca.ld = static_cast<int>(x.ld);
        ca.d = x.cols;
        ca.centers = cbak_b.as<float>();
        ca.k = k;
        ca.kpad = g.kpad;
        ca.labels = req.labels;
        int nb = kern::kmeans_label_cost(ca, slab.as<double>(), std::min(nslab, 2048), s);
        if (nb < 0) {  // centers beyond LDS: per-row costs through the seed kernel
          if (!mind_keep.data()) md = ctx.alloc(sizeof(float) * x.rows);
          ca.mindist = mind_keep.data() ? mind_keep.as<float>() : md.as<float>();
          kern::kmeans_seed_mindist(ca, s);
          nb = kern::reduce_sum_f32(ca.mindist, x.rows, slab.as<double>(), s);
        }
        kern::sum_f64(slab.as<double>(), nb, cost_d.as<double>(), s);
      }
      if (!comm.trivial()) {
        comm_allreduce(ctx, comm, cost_d.data(), 1, DType::F64, ReduceOp::Sum, s);
        if (comm.on_device()) comm.wait(s);  // the watchdog covers this collective too
      }
      double c = 0.0;
      ctx.copy_to_host(&c, cost_d.data(), sizeof(double), s);
      res.cost = c;
      res.cost_history.back() = c;
    }
  }
  hm.mark("final_cost");
  res.last_counts.assign(counts_h.as<u64>(), counts_h.as<u64>() + k);
  res.centers.resize(kd);
  ctx.copy_to_host(res.centers.data(), c64.data(), sizeof(double) * kd, s);
  ctx.copy_to_host(refine_h.data(), refine_d.data(), 2 * sizeof(u64), s);
  res.refine_tiles = static_cast<int64_t>(refine_h.as<u64>()[0]);
  res.tier3_tiles = static_cast<int64_t>(refine_h.as<u64>()[1]);
  if (prune) {
    u64 pt = 0;
    ctx.copy_to_host(&pt, pruned_d.data(), sizeof(u64), s);
    res.pruned_tiles = static_cast<int64_t>(pt);
  }
  if (rpruned_b.data()) {
    u64 pr = 0;
    ctx.copy_to_host(&pr, rpruned_b.data(), sizeof(u64), s);
    res.pruned_rows = static_cast<int64_t>(pr);
  }
  if (ldstat_b.data()) {
    u64 dr[5] = {0, 0, 0, 0, 0};
    ctx.copy_to_host(dr, ldstat_b.data(), 5 * sizeof(u64), s);
    res.deferred_rows = static_cast<int64_t>(dr[0]);
    res.moved_rows = static_cast<int64_t>(dr[1]) + cmoved;
    res.image_passes = static_cast<int>(dr[2]);  // counted by the passes that read the image
  }
  hm.mark("results");
  res.iter_seconds = seconds_since(t_iter);
  M.set_value("kmeans/iter_seconds", res.iter_seconds);
  M.set_value("kmeans/refine_tiles", double(res.refine_tiles));
  M.set_value("kmeans/samples_per_sec",
              res.iter_seconds > 0 ? double(x.global_rows) * res.num_iter / res.iter_seconds : 0);
  res.assign_path = t_assign_path;
  return res;
}

KMeansResult kmeans_fit(Context& ctx, Comm& comm, DenseTable& x,
                        const std::vector<double>& init_centers, const KMeansParams& p) {
  std::vector<double> again;
  KMeansResult r = kmeans_fit_once(ctx, comm, x, init_centers, p, &again);
  if (again.empty()) return r;
  // a row past the provisional bounds: the first batch's integers may have wrapped — the fit
  // runs again from its initial centers with the column maxima's scales (rare: rows far outside
  // every initial center's coordinate range), after the first attempt released its buffers
  KMeansParams q = p;
  q.absmax_pass = true;
  q.init = KMeansInit::Given;
  KMeansResult r2 = kmeans_fit_once(ctx, comm, x, again, q, nullptr);
  r2.init_seconds = r.init_seconds;
  r2.scale_source = "restart";
  return r2;
}

void kmeans_predict_device(Context& ctx, const DenseTable& x, const std::vector<double>& centers,
                           int k, int32_t* labels, float* dist2) {
  OAP_CHECK(ctx.is_gpu(), "kmeans_predict_device needs a GPU context");
  OAP_CHECK(centers.size() == size_t(k) * x.cols, "centers must be k x d");
  OAP_CHECK(labels && dist2, "device output pointers required");
  check_gpu_table(x);
  ctx.activate();
  if (x.rows == 0) return;
  TraceRange tr(&ctx.metrics(), "kmeans/predict_device");
  GpuCenters g = upload_centers(ctx, centers, k, x.cols);
  AssignReq req;
  req.labels = labels;
  req.mindist = dist2;
  gpu_assign(ctx, x, g, req, ctx.compute());
  OAP_HIP_CHECK(hipStreamSynchronize(ctx.compute()));
}

void kmeans_predict(Context& ctx, const DenseTable& x, const std::vector<double>& centers, int k,
                    int32_t* labels, double* dist2) {
  OAP_CHECK(centers.size() == size_t(k) * x.cols, "centers must be k x d");
  TraceRange tr(&ctx.metrics(), "kmeans/predict");
  if (!ctx.is_gpu()) {
    cpu_assign(ctx, x, centers, k, nullptr, false, false, labels, dist2);
    return;
  }
  check_gpu_table(x);
  ctx.activate();
  if (x.rows == 0) return;
  GpuCenters g = upload_centers(ctx, centers, k, x.cols);
  Buffer dl = ctx.alloc(sizeof(int32_t) * x.rows);
  Buffer dd = ctx.alloc(sizeof(float) * x.rows);
  AssignReq req;
  req.labels = dl.as<int32_t>();
  req.mindist = dd.as<float>();
  gpu_assign(ctx, x, g, req, ctx.compute());
  if (labels) ctx.copy_to_host(labels, dl.data(), sizeof(int32_t) * x.rows);
  if (dist2) {
    std::vector<float> h(x.rows);
    ctx.copy_to_host(h.data(), dd.data(), sizeof(float) * x.rows);
    for (int64_t i = 0; i < x.rows; ++i) dist2[i] = h[i];
  }
}

// ---------------------------------------------------------------- streamed (out-of-core) fit
KMeansResult kmeans_fit_streamed(Context& ctx, Comm& comm, const float* host, int64_t rows,
                                 int d, const std::vector<double>& init_centers,
                                 const KMeansParams& p, int64_t chunk_rows) {
  OAP_CHECK(ctx.is_gpu(), "kmeans_fit_streamed needs a GPU context");
  OAP_CHECK(d >= 1 && !init_centers.empty() && init_centers.size() % size_t(d) == 0,
            "kmeans_fit_streamed: initial centers must be k x d");
  OAP_CHECK(chunk_rows >= 32, "kmeans_fit_streamed: chunk_rows must be >= 32");
  ctx.activate();
  const int k = static_cast<int>(init_centers.size() / d);
  const size_t kd = size_t(k) * d;
  KMeansResult res;
  res.d = d;
  res.k = k;
  std::vector<double> centers = init_centers;
  hipStream_t s = ctx.compute(), hs = ctx.h2d() ? ctx.h2d() : s;
  // global rows and per-column |x| max (host pass over the rows, thread pool)
  const int64_t g_rows = static_cast<int64_t>(
      comm_allreduce_scalar(ctx, comm, double(rows), ReduceOp::Sum));
  const int64_t max_local = static_cast<int64_t>(
      comm_allreduce_scalar(ctx, comm, double(rows), ReduceOp::Max));
  res.global_rows = g_rows;
  std::vector<double> absmax(d, 0.0);
  {
    const int nt = ctx.pool().size();
    std::vector<std::vector<double>> part(nt, std::vector<double>(d, 0.0));
    ctx.pool().parallel_for(rows, [&](int ci, int64_t b, int64_t e) {
      std::vector<double>& m = part[ci];
      for (int64_t i = b; i < e; ++i)
        for (int f = 0; f < d; ++f)
          m[f] = std::max(m[f], std::fabs(double(host[size_t(i) * d + f])));
    });
    for (const auto& m : part)
      for (int f = 0; f < d; ++f) absmax[f] = std::max(absmax[f], m[f]);
    comm_allreduce_host(ctx, comm, absmax.data(), size_t(d), DType::F64, ReduceOp::Max);
  }
  bool from_centers = false;  // (the resident fit's rule: bitwise its integers)
  FixedPoint fp = fixed_point_scales(fit_bounds(center_bounds(centers, k, d), absmax, g_rows,
                                                &from_centers),
                                     g_rows, max_local);
  res.scale_source = from_centers ? "centers_checked" : "absmax";
  auto t_iter = std::chrono::steady_clock::now();

  // two device chunk buffers, filled by pitched DMA from the (registered) host rows on the H2D
  // stream while the other chunk is assigned on the compute stream
  const int64_t ld = kern::kmeans_ld(d);
  const int64_t cr = std::min<int64_t>(chunk_rows, std::max<int64_t>(rows, 1));
  Buffer dev[2] = {ctx.alloc(size_t(cr) * ld * 4), ctx.alloc(size_t(cr) * ld * 4)};
  for (auto& b : dev) OAP_HIP_CHECK(hipMemsetAsync(b.data(), 0, size_t(cr) * ld * 4, s));
  // the caller's rows stay page-locked for the fit only: the guard unregisters them on every
  // exit path (a CommError or an injected fault from the loop included)
  struct HostRegistration {
    void* p = nullptr;
    hipStream_t s0 = nullptr, s1 = nullptr;  // drained first: no DMA may still read the rows
    ~HostRegistration() {
      if (!p) return;
      (void)hipStreamSynchronize(s0);
      (void)hipStreamSynchronize(s1);
      (void)hipHostUnregister(p);
    }
  } registration{nullptr, s, hs};
  if (rows > 0 && hipHostRegister(const_cast<float*>(host), size_t(rows) * d * 4,
                                  hipHostRegisterDefault) == hipSuccess)
    registration.p = const_cast<float*>(host);
  (void)hipGetLastError();  // (a refused registration leaves pageable DMA)
  Event loaded[2], used[2];
  used[0].record(s);
  used[1].record(s);

  GpuCenters g = alloc_centers(ctx, k, d);
  Buffer c64 = ctx.alloc(sizeof(double) * kd);
  Buffer stats = ctx.alloc(sizeof(u64) * (kd + k));
  const int nslab = kern::kmeans_cost_slab_size(ctx.info().cu_count);
  Buffer slab = ctx.alloc(sizeof(double) * nslab);
  const int64_t nchunks = (rows + cr - 1) / cr;
  Buffer costs = ctx.alloc(sizeof(double) * size_t(std::max<int64_t>(nchunks, 1)) + 8);
  Buffer cost_d = ctx.alloc(sizeof(double));
  Buffer scale = ctx.alloc(sizeof(float) * (round_up(d, 4) + 4));
  Buffer inv_scale = ctx.alloc(sizeof(double) * d);
  Buffer flags_d = ctx.alloc(sizeof(kern::KMeansFlags));
  Buffer fin_scratch = ctx.alloc(sizeof(double) * 2 * std::max(k, 1));
  ctx.memset(scale.data(), 0, sizeof(float) * (round_up(d, 4) + 4), s);
  ctx.copy_to_backend(c64.data(), centers.data(), sizeof(double) * kd, s);
  ctx.copy_to_backend(scale.data(), fp.scale.data(), sizeof(float) * d, s);
  ctx.copy_to_backend(inv_scale.data(), fp.inv_scale.data(), sizeof(double) * d, s);
  kern::kmeans_prepare_centers(c64.as<double>(), k, d, g.dp, g.c32.as<float>(),
                               g.cnorm.as<float>(), g.cstat.as<float>(), g.kpad, s);
  u64* sums = stats.as<u64>();
  u64* counts = sums + kd;
  kern::KMeansFinalizeArgs fa;
  fa.sums = sums;
  fa.counts = counts;
  fa.inv_scale = inv_scale.as<double>();
  fa.centers64 = c64.as<double>();
  fa.centers32 = g.c32.as<float>();
  fa.cnorm = g.cnorm.as<float>();
  fa.cstat = g.cstat.as<float>();
  fa.k = k;
  fa.d = d;
  fa.dp = g.dp;
  fa.tol = p.tol;
  fa.cost_in = cost_d.as<double>();
  fa.flags = flags_d.data();
  fa.scratch = fin_scratch.as<double>();
  kern::KMeansFlags fl{};
  for (int it = 0; it < p.max_iter; ++it) {
    maybe_inject_fault(comm.rank(), "kmeans_iter", it);
    TraceRange tr(&ctx.metrics(), "kmeans/iteration_streamed");
    OAP_HIP_CHECK(hipMemsetAsync(stats.data(), 0, sizeof(u64) * (kd + k), s));
    for (int64_t c = 0; c < nchunks; ++c) {
      const int b = int(c & 1);
      const int64_t r0 = c * cr, nr = std::min(cr, rows - r0);
      used[b].wait_on(hs);  // the chunk that last used this buffer is assigned
      OAP_HIP_CHECK(hipMemcpy2DAsync(dev[b].data(), size_t(ld) * 4, host + size_t(r0) * d,
                                     size_t(d) * 4, size_t(d) * 4, size_t(nr),
                                     hipMemcpyHostToDevice, hs));
      loaded[b].record(hs);
      loaded[b].wait_on(s);
      DenseTable view;
      view.rows = nr;
      view.cols = d;
      view.ld = ld;
      view.dtype = DType::F32;
      view.backend = Backend::GPU;
      view.data = Buffer::view(dev[b].data(), size_t(nr) * ld * 4);
      view.global_offset = r0;
      view.global_rows = g_rows;
      AssignReq req;
      req.accumulate = true;
      req.sums_too = true;
      req.precise = p.precise;
      req.scale = scale.as<float>();
      req.sums = sums;
      req.counts = counts;
      req.cost_slab = slab.as<double>();
      const int nb = gpu_assign(ctx, view, g, req, s);
      if (nb > 0)
        kern::sum_f64(slab.as<double>(), nb, costs.as<double>() + c, s);
      else
        OAP_HIP_CHECK(hipMemsetAsync(costs.as<double>() + c, 0, sizeof(double), s));
      used[b].record(s);
    }
    // chunk costs in chunk order (deterministic), then one grouped allreduce + finalize
    if (nchunks > 0)
      kern::sum_f64(costs.as<double>(), int(nchunks), cost_d.as<double>(), s);
    else
      OAP_HIP_CHECK(hipMemsetAsync(cost_d.data(), 0, sizeof(double), s));
    if (!comm.trivial()) {
      comm_allreduce(ctx, comm, stats.data(), kd + k, DType::I64, ReduceOp::Sum, s);
      comm_allreduce(ctx, comm, cost_d.data(), 1, DType::F64, ReduceOp::Sum, s);
      if (comm.on_device()) comm.wait(s);
    }
    kern::kmeans_finalize(fa, s);
    ctx.copy_to_host(&fl, flags_d.data(), sizeof(fl), s);
    res.cost = fl.cost;
    res.cost_history.push_back(fl.cost);
    res.shift_history.push_back(std::sqrt(std::max(fl.max_shift2, 0.0)));
    res.num_iter = it + 1;
    if (fl.converged && p.tol >= 0) {
      res.converged = true;
      break;
    }
  }
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  res.centers.resize(kd);
  ctx.copy_to_host(res.centers.data(), c64.data(), sizeof(double) * kd, s);
  std::vector<u64> cnt(k);
  ctx.copy_to_host(cnt.data(), counts, sizeof(u64) * k, s);
  res.last_counts.assign(cnt.begin(), cnt.end());
  res.iter_seconds = seconds_since(t_iter);
  return res;
}

}  // namespace oap

namespace oap {

void kmeans_set_lean_variant(int v) { lean_variant_ref() = v; }

double& last_timing_deferred() {
  static double v = 0.0;
  return v;
}

double kmeans_assign_timing(Context& ctx, const DenseTable& x, const std::vector<double>& centers,
                            int k, int reps, bool precise, int ablate) {
  OAP_CHECK(ctx.is_gpu(), "kmeans_assign_timing needs a GPU context");
  check_gpu_table(x);
  ctx.activate();
  const int d = x.cols;
  GpuCenters g = upload_centers(ctx, centers, k, d);
  std::vector<double> absmax(d, 1.0);
  for (int f = 0; f < d; ++f) absmax[f] = 64.0;
  FixedPoint fp = fixed_point_scales(absmax, x.rows, x.rows);
  Buffer scale = ctx.alloc(sizeof(float) * (round_up(d, 4) + 4));
  ctx.memset(scale.data(), 0, sizeof(float) * (round_up(d, 4) + 4));
  ctx.copy_to_backend(scale.data(), fp.scale.data(), sizeof(float) * d);
  Buffer stats = ctx.alloc(sizeof(u64) * (size_t(k) * d + k));
  Buffer slab = ctx.alloc(sizeof(double) * kern::kmeans_cost_slab_size(ctx.info().cu_count));
  kern::KMeansAssignArgs a;
  a.x = x.data.data();
  a.xbf16 = x.dtype == DType::BF16;
  a.n = x.rows;
  a.ld = static_cast<int>(x.ld);
  a.d = d;
  a.centers = g.c32.as<float>();
  a.cnorm = g.cnorm.as<float>();
  a.cstat = g.cstat.as<float>();
  a.k = k;
  a.kpad = g.kpad;
  a.scale = scale.as<float>();
  a.sums = stats.as<u64>();
  a.counts = stats.as<u64>() + size_t(k) * d;
  a.cost_slab = slab.as<double>();
  a.precise = precise;
  a.fast1 = !precise && !(ablate & 32);
  a.ablate = ablate;
  hipStream_t s = ctx.compute();
  Event e0, e1;
  if (ablate & 64) {  // the Lloyd fit's path: lean tier-1 pass + exact re-decision of its rows
    AssignReq req;
    req.accumulate = true;
    req.ablate = ablate & 59;
    req.scale = scale.as<float>();
    req.sums = a.sums;
    req.counts = a.counts;
    req.cost_slab = (ablate & 4) ? nullptr : a.cost_slab;  // 4: the Lloyd pass without a cost
    req.fast1 = true;
    Buffer dr = ctx.alloc(5 * sizeof(u64));
    ctx.memset(dr.data(), 0, 5 * sizeof(u64), s);
    req.deferred_rows = dr.as<u64>();
    OAP_CHECK(lean_applies(x, k, g.kpad, req), "lean path not applicable");
    gpu_assign(ctx, x, g, req, s);  // warm
    e0.record(s);
    for (int i = 0; i < reps; ++i) gpu_assign(ctx, x, g, req, s);
    e1.record(s);
    e1.sync();
    u64 n_def = 0;
    ctx.copy_to_host(&n_def, dr.data(), sizeof(u64));
    Logger::instance().log(LogLevel::Info, "kmeans/timing_deferred",
                           "\"rows_per_pass\":" + std::to_string(double(n_def) / (reps + 1)));
    last_timing_deferred() = double(n_def) / (reps + 1);
    return Event::elapsed_ms(e0, e1) / std::max(reps, 1);
  }
  kern::kmeans_assign(a, ctx.info().cu_count, s);  // warm
  e0.record(s);
  for (int i = 0; i < reps; ++i) kern::kmeans_assign(a, ctx.info().cu_count, s);
  e1.record(s);
  e1.sync();
  return Event::elapsed_ms(e0, e1) / std::max(reps, 1);
}


// Steady-state image-pass timing (tools/kmeans_img_probe.py): a full lean pass at centers_a
// writes the operand image and the labels, then each rep restores those labels and statistics
// and times one delta image pass at centers_b (the moved rows of a Lloyd step): the lean pass
// alone (kernel: 0 kmeans_lloyd, 1 kmeans_lean_img with configuration cfg) and, separately, the
// pass plus the exact re-decision of its deferred rows.
ImageTiming kmeans_image_timing(Context& ctx, const DenseTable& x,
                                const std::vector<double>& centers_a,
                                const std::vector<double>& centers_b, int k, int reps, int kernel,
                                int cfg, bool fallback) {
  OAP_CHECK(ctx.is_gpu() && x.dtype == DType::F32, "kmeans_image_timing needs f32 rows on a GPU");
  check_gpu_table(x);
  ctx.activate();
  const int d = x.cols;
  hipStream_t s = ctx.compute();
  GpuCenters ga = upload_centers(ctx, centers_a, k, d);
  GpuCenters gb = upload_centers(ctx, centers_b, k, d);
  std::vector<double> absmax(d, 64.0);
  FixedPoint fp = fixed_point_scales(absmax, x.rows, x.rows);
  Buffer scale = ctx.alloc(sizeof(float) * (round_up(d, 4) + 4));
  ctx.memset(scale.data(), 0, sizeof(float) * (round_up(d, 4) + 4));
  ctx.copy_to_backend(scale.data(), fp.scale.data(), sizeof(float) * d);
  const size_t nst = size_t(k) * d + k;
  Buffer stats = ctx.alloc(sizeof(u64) * nst), stats0 = ctx.alloc(sizeof(u64) * nst);
  Buffer slab = ctx.alloc(sizeof(double) * kern::kmeans_cost_slab_size(ctx.info().cu_count));
  Buffer lab = ctx.alloc(sizeof(int32_t) * size_t(x.rows));
  Buffer lab0 = ctx.alloc(sizeof(int32_t) * size_t(x.rows));
  const size_t ib = kern::kmeans_lloyd_image_bytes(x.rows, d);
  OAP_CHECK(ib > 0, "kmeans_image_timing: no operand image at d=" << d);
  Buffer img = ctx.alloc(ib), beta = ctx.alloc(sizeof(float) * 4);
  Buffer dr = ctx.alloc(5 * sizeof(u64));
  ctx.memset(stats.data(), 0, sizeof(u64) * nst, s);
  ctx.memset(dr.data(), 0, 5 * sizeof(u64), s);
  AssignReq req;
  req.accumulate = true;
  req.sums_too = true;
  req.scale = scale.as<float>();
  req.sums = stats.as<u64>();
  req.counts = stats.as<u64>() + size_t(k) * d;
  req.labels = lab.as<int32_t>();
  req.cost_slab = slab.as<double>();
  req.fast1 = true;
  req.ximg = img.data();
  req.img_beta = beta.as<float>();
  req.img_mode = 1;
  req.deferred_rows = dr.as<u64>();
  OAP_CHECK(lean_applies(x, k, ga.kpad, req), "kmeans_image_timing: lean path not applicable");
  gpu_assign(ctx, x, ga, req, s);  // writes the image and every label
  OAP_HIP_CHECK(hipMemcpyAsync(lab0.data(), lab.data(), sizeof(int32_t) * size_t(x.rows),
                               hipMemcpyDeviceToDevice, s));
  OAP_HIP_CHECK(hipMemcpyAsync(stats0.data(), stats.data(), sizeof(u64) * nst,
                               hipMemcpyDeviceToDevice, s));
  req.cost_slab = nullptr;
  req.img_mode = 2;
  req.delta = true;
  req.labels_valid = true;
  req.img_kernel = kernel;
  req.img_cfg = cfg;
  req.img_fallback = fallback;
  ImageTiming out;
  Event e0, e1;
  for (int pass = 0; pass < 2; ++pass) {
    req.skip_exact = pass == 0;
    double tot = 0.0;
    for (int i = 0; i <= reps; ++i) {  // (rep 0 warms)
      OAP_HIP_CHECK(hipMemcpyAsync(lab.data(), lab0.data(), sizeof(int32_t) * size_t(x.rows),
                                   hipMemcpyDeviceToDevice, s));
      OAP_HIP_CHECK(hipMemcpyAsync(stats.data(), stats0.data(), sizeof(u64) * nst,
                                   hipMemcpyDeviceToDevice, s));
      ctx.memset(dr.data(), 0, 5 * sizeof(u64), s);
      e0.record(s);
      gpu_assign(ctx, x, gb, req, s);
      e1.record(s);
      e1.sync();
      if (i > 0) tot += Event::elapsed_ms(e0, e1);
    }
    (pass == 0 ? out.lean_ms : out.pass_ms) = tot / std::max(reps, 1);
  }
  u64 h[3] = {0, 0, 0};
  ctx.copy_to_host(h, dr.data(), 3 * sizeof(u64), s);
  out.deferred_rows = static_cast<int64_t>(h[0]);
  out.moved_rows = static_cast<int64_t>(h[1]);
  out.image_passes = static_cast<int64_t>(h[2]);
  // the last rep's result: labels and statistics (for A/B equality checks)
  out.labels.resize(size_t(x.rows));
  ctx.copy_to_host(out.labels.data(), lab.data(), sizeof(int32_t) * size_t(x.rows), s);
  out.stats.resize(nst);
  ctx.copy_to_host(out.stats.data(), stats.data(), sizeof(u64) * nst, s);
  out.path = t_assign_path;
  return out;
}

}  // namespace oap
