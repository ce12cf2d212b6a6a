#include "drivers/pca.h"

#include <algorithm>
#include <chrono>
#include <cmath>

#include "kernels/kernels.h"
#include "linalg/eigen.h"
#include "linalg/eigen_gpu.h"
#include "runtime/knobs.h"
#include "runtime/log.h"

namespace oap {

namespace {

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// A shift vector close to the global mean: the count-weighted mean of every rank's first rows.
// It only conditions the one-pass statistics (any value gives the same covariance in exact
// arithmetic), so a small sample suffices.  Rounded to fp32, the precision the kernel subtracts.
std::vector<double> global_shift(Context& ctx, Comm& comm, const DenseTable& x) {
  const int d = x.cols;
  const int64_t m = std::min<int64_t>(x.rows, 256);
  std::vector<double> acc(d + 1, 0.0);
  if (m > 0) {
    std::vector<double> rows = table_rows_f64(ctx, x, 0, m);
    for (int64_t r = 0; r < m; ++r)
      for (int c = 0; c < d; ++c) acc[c] += rows[size_t(r) * d + c];
  }
  acc[d] = double(m);
  comm_allreduce_host(ctx, comm, acc.data(), acc.size(), DType::F64, ReduceOp::Sum);
  std::vector<double> s(d, 0.0);
  if (acc[d] > 0)
    for (int c = 0; c < d; ++c) s[c] = double(float(acc[c] / acc[d]));
  return s;
}

// CPU engine: S = sum (x-s)(x-s)^T (upper triangle), c = sum (x-s), fp64, thread-blocked.
void cpu_stats(Context& ctx, const DenseTable& x, const std::vector<double>& shift,
               std::vector<double>& out) {
  const int d = x.cols;
  const int nt = ctx.pool().size();
  std::vector<std::vector<double>> part(nt);
  ctx.pool().parallel_for(x.rows, [&](int ci, int64_t b, int64_t e) {
    std::vector<double>& P = part[ci];
    P.assign(size_t(d) * d + d, 0.0);
    std::vector<double> v(d);
    for (int64_t r = b; r < e; ++r) {
      for (int c = 0; c < d; ++c) {
        const double xv = x.dtype == DType::F64 ? x.data.as<double>()[size_t(r) * x.ld + c]
                                                : x.data.as<float>()[size_t(r) * x.ld + c];
        v[c] = xv - shift[c];
      }
      for (int i = 0; i < d; ++i) {
        const double vi = v[i];
        double* row = &P[size_t(i) * d];
        for (int j = i; j < d; ++j) row[j] += vi * v[j];
        P[size_t(d) * d + i] += vi;
      }
    }
  });
  out.assign(size_t(d) * d + d, 0.0);
  for (auto& P : part) {
    if (P.empty()) continue;
    for (size_t i = 0; i < out.size(); ++i) out[i] += P[i];
  }
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < i; ++j) out[size_t(i) * d + j] = out[size_t(j) * d + i];
}

}  // namespace

// int8 exact engine: largest accepted err_bound relative to the largest variance
constexpr double kExactRelBound = 1e-10;

PcaCovariance pca_covariance(Context& ctx, Comm& comm, DenseTable& x, const PcaParams& p,
                             bool device_cov) {
  TraceRange tr(&ctx.metrics(), "pca/covariance");
  const int d = x.cols;
  OAP_CHECK(d > 0, "PCA needs at least one feature");
  if (x.global_rows < 0) assign_global_offsets(ctx, comm, x);
  PcaCovariance res;
  res.d = d;
  res.n = x.global_rows;
  OAP_CHECK(res.n > 1, "Cannot compute the covariance of a matrix with <= 1 row");
  const std::vector<double> shift = global_shift(ctx, comm, x);
  const size_t cnt = size_t(d) * d + d;
  std::vector<double> stats(cnt, 0.0);
  if (ctx.is_gpu()) {
    OAP_CHECK(x.dtype == DType::F32 || (p.exact && x.dtype == DType::F64),
              "GPU PCA expects an f32 table (f32 or f64 in exact mode)");
    ctx.activate();
    hipStream_t s = ctx.compute();
    // exact mode on f32 rows: the int8 digit products (kernels/pca_ozaki.hip); the fp64 MFMA
    // for f64 rows (their 53-bit inputs would need more digits) or when the knob says so
    bool digits = p.exact && x.dtype == DType::F32 &&
                  knob_str("OAP_PCA_EXACT_ENGINE") != "fp64";
    res.engine = !p.exact ? "bf16_split" : digits ? "int8_digits" : "fp64_mfma";
    // [S | c | bound]: the bound rides in the one allreduce (summed over the ranks)
    const size_t cnt_x = cnt + (digits ? 1 : 0);
    Buffer out = ctx.alloc(cnt_x * sizeof(double));
    Buffer part, cpart, shf, ws;
    kern::PcaPlan plan;
    kern::PcaOzakiPlan oplan;
    auto setup_mfma = [&]() {  // the fp64 (exact) or bf16-split (fast) SYRK's plan and slabs
      plan = p.exact ? kern::pca_syrk_plan_f64(x.rows, d, ctx.info().cu_count)
                     : kern::pca_syrk_plan(x.rows, d, ctx.info().cu_count);
      part = ctx.alloc(plan.part_elems * sizeof(double));
      cpart = ctx.alloc(plan.cpart_elems * sizeof(double));
      shf = ctx.alloc(plan.shift_elems * sizeof(double));
      if (p.exact) {  // the fp64 shift itself (no fp32 rounding: exact mode subtracts in fp64)
        std::vector<double> hs(plan.shift_elems, 0.0);
        for (int c = 0; c < d; ++c) hs[c] = shift[c];
        ctx.copy_to_backend(shf.data(), hs.data(), hs.size() * sizeof(double), s);
      } else {
        std::vector<float> hs(plan.shift_elems, 0.f);
        for (int c = 0; c < d; ++c) hs[c] = float(shift[c]);
        ctx.copy_to_backend(shf.data(), hs.data(), hs.size() * sizeof(float), s);
      }
    };
    if (digits) {
      size_t free_b = 0, total_b = 0;
      OAP_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
      // digit planes of one row chunk (7 bytes per padded element): at most 16 GiB (knob) and a
      // third of what is free (the 40 GB bench table takes 5 chunks)
      const size_t cap = std::min<size_t>(size_t(knob_int("OAP_PCA_DIGIT_CHUNK_BYTES")),
                                          free_b / 3);
      oplan = kern::pca_ozaki_plan(x.rows, d, ctx.info().cu_count, cap);
      ws = ctx.alloc(oplan.ws_bytes);
    } else {
      setup_mfma();
    }
    Event e0, e1, e2;
    double bound_s = 0.0;
    // one pass: statistics, the one allreduce, the host copy; with the int8 engine a negative
    // allreduced bound means some rank's sampled column scales were too small — every rank sees
    // it and redoes the pass with exact scales (the same decision everywhere)
    auto run = [&](bool exact_scales) {
      e0.record(s);
      {
        TraceRange k(&ctx.metrics(), "pca/syrk_launch");
        if (digits) {
          kern::pca_syrk_ozaki(x.data.as<float>(), x.ld, shift.data(), oplan, ws.data(),
                               out.as<double>(), out.as<double>() + size_t(d) * d,
                               out.as<double>() + cnt, exact_scales, s);
        } else {
          if (p.exact)
            kern::pca_syrk_f64(x.data.data(), x.dtype == DType::F64, x.rows, x.ld, d,
                               shf.as<double>(), plan, part.as<double>(), cpart.as<double>(), s);
          else
            kern::pca_syrk(x.data.as<float>(), x.rows, x.ld, d, shf.as<float>(), plan,
                           part.as<double>(), cpart.as<double>(), p.precise, p.flush_rows, s);
          kern::pca_reduce(plan, part.as<double>(), cpart.as<double>(), d, out.as<double>(),
                           out.as<double>() + size_t(d) * d, s);
        }
      }
      e1.record(s);
      comm_allreduce(ctx, comm, out.data(), digits ? cnt_x : cnt, DType::F64, ReduceOp::Sum, s);
      if (comm.on_device()) comm.wait(s);
      e2.record(s);
      if (device_cov) {  // the covariance stays on the device; only c comes back (the mean)
        if (!res.dev_cov.data()) res.dev_cov = ctx.alloc(sizeof(double) * size_t(d) * d);
        kern::pca_cov(out.as<double>(), d, res.n, res.dev_cov.as<double>(), s);
        std::vector<double> tail(size_t(d) + (digits ? 1 : 0));
        ctx.copy_to_host(tail.data(), out.as<double>() + size_t(d) * d,
                         tail.size() * sizeof(double));
        std::copy(tail.begin(), tail.begin() + d, stats.begin() + size_t(d) * d);
        if (digits) bound_s = tail[d];
      } else {
        std::vector<double> all(digits ? cnt_x : cnt);
        ctx.copy_to_host(all.data(), out.data(), all.size() * sizeof(double));
        std::copy(all.begin(), all.begin() + cnt, stats.begin());
        if (digits) bound_s = all[cnt];
      }
    };
    run(false);
    if (digits && bound_s < 0) {
      res.scales_redone = true;
      run(true);
    }
    res.err_bound = digits ? bound_s / double(res.n - 1) : 0.0;
    if (digits) {
      // The bound is relative to the column ranges (max |v_j| max |v_k|), not to each product: a
      // column whose range dwarfs its spread (a far outlier) can leave it above fp64 accuracy.
      // Then the pass is redone on the fp64 MFMA (same decision on every rank: S, c and the
      // bound are allreduced).
      std::vector<double> sdiag(d);
      OAP_HIP_CHECK(hipMemcpy2DAsync(sdiag.data(), sizeof(double), out.data(),
                                     size_t(d + 1) * sizeof(double), sizeof(double), d,
                                     hipMemcpyDeviceToHost, s));
      OAP_HIP_CHECK(hipStreamSynchronize(s));
      const double nn = double(res.n);
      double vmax = 0.0;
      for (int j = 0; j < d; ++j) {
        const double cj = stats[size_t(d) * d + j];
        vmax = std::max(vmax, (sdiag[j] - cj * cj / nn) / (nn - 1.0));
      }
      res.int8_rel_bound = vmax > 0 ? res.err_bound / vmax : 0.0;
      if (!(res.err_bound <= kExactRelBound * vmax)) {
        res.fallback_fp64 = true;
        digits = false;
        res.engine = "fp64_mfma";
        res.err_bound = 0.0;
        ws = Buffer();
        setup_mfma();
        run(false);
      }
    }
    res.stats_ms = Event::elapsed_ms(e0, e1);
    res.allreduce_ms = Event::elapsed_ms(e1, e2);
    ctx.metrics().add("pca/syrk_kernel", res.stats_ms * 1e3,
                      int64_t(x.rows) * x.ld * int64_t(sizeof(float)));
    ctx.metrics().add("pca/allreduce", res.allreduce_ms * 1e3, int64_t(cnt * sizeof(double)));
  } else {
    res.engine = "cpu";
    auto t0 = std::chrono::steady_clock::now();
    cpu_stats(ctx, x, shift, stats);
    res.stats_ms = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    comm_allreduce_host(ctx, comm, stats.data(), cnt, DType::F64, ReduceOp::Sum);
    res.allreduce_ms = ms_since(t0);
  }
  maybe_inject_fault(comm.rank(), "pca_stats", 0);
  // cov = (S - c c^T / n) / (n - 1), mean = s + c / n
  const double n = double(res.n);
  const double* S = stats.data();
  const double* c = stats.data() + size_t(d) * d;
  res.mean.resize(d);
  for (int i = 0; i < d; ++i) res.mean[i] = shift[i] + c[i] / n;
  if (res.dev_cov.data()) return res;
  res.cov.resize(size_t(d) * d);
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j)
      res.cov[size_t(i) * d + j] = (S[size_t(i) * d + j] - c[i] * c[j] / n) / (n - 1.0);
  return res;
}

PcaResult pca_fit(Context& ctx, Comm& comm, DenseTable& x, const PcaParams& p) {
  auto t0 = std::chrono::steady_clock::now();
  const int d = x.cols;
  OAP_CHECK(p.k >= 1 && p.k <= d, "PCA k must be in [1, numFeatures=" << d << "], got " << p.k);
  const bool gpu_eig = ctx.is_gpu() && p.gpu_eig && sym_eig_gpu_supported(ctx, d, p.k);
  PcaCovariance cv = pca_covariance(ctx, comm, x, p, gpu_eig);
  PcaResult r;
  r.d = d;
  r.k = p.k;
  r.n = cv.n;
  r.mean = cv.mean;
  r.stats_ms = cv.stats_ms;
  r.allreduce_ms = cv.allreduce_ms;
  r.engine = cv.engine;
  r.err_bound = cv.err_bound;
  auto t1 = std::chrono::steady_clock::now();
  SymEig eg;
  {
    TraceRange tr(&ctx.metrics(), "pca/eigensolver");
    if (gpu_eig) {
      hipStream_t s = ctx.compute();
      GpuEigTiming t;
      eg = sym_eig_topk_gpu(ctx, cv.dev_cov.as<double>(), d, p.k, s, &t);
      r.eig_on_gpu = true;
      r.eig_tridiag_ms = t.tridiag_ms;
      r.eig_host_ms = t.host_ms;
      r.eig_backtransform_ms = t.backtransform_ms;
    } else {
      eg = sym_eig_topk(cv.cov, d, p.k, &ctx.pool());
    }
  }
  r.eig_ms = ms_since(t1);
  r.eigenvalues = eg.values;
  double tot = 0.0;
  for (double v : eg.values) tot += std::fabs(v);
  r.explained.resize(p.k);
  for (int j = 0; j < p.k; ++j) r.explained[j] = tot > 0 ? std::fabs(eg.values[j]) / tot : 0.0;
  r.pc = std::move(eg.vectors);  // d x k
  r.total_ms = ms_since(t0);
  if (comm.rank() == 0 && Logger::instance().level() <= LogLevel::Info)
    Logger::instance().log(LogLevel::Info, "pca/fit",
                           "\"n\":" + std::to_string(r.n) + ",\"d\":" + std::to_string(d) +
                               ",\"k\":" + std::to_string(p.k) + ",\"stats_ms\":" +
                               std::to_string(r.stats_ms) + ",\"eig_ms\":" +
                               std::to_string(r.eig_ms));
  return r;
}

}  // namespace oap
