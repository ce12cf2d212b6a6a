#include "linalg/eigen_gpu.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <vector>

#include "kernels/kernels.h"
#include "runtime/common.h"
#include "runtime/knobs.h"

namespace oap {

bool sym_eig_gpu_supported(const Context& ctx, int n, int k) {
  return ctx.is_gpu() && 2 * k <= n && kern::eig_tridiag_supported(n, ctx.info().cu_count) &&
         size_t(n) * 8 + 64 <= 160 * 1024;
}

SymEig sym_eig_topk_gpu(Context& ctx, const double* a, int n, int k, hipStream_t s,
                        GpuEigTiming* timing) {
  OAP_CHECK(sym_eig_gpu_supported(ctx, n, k), "sym_eig_topk_gpu: unsupported n=" << n << " k="
                                                                                 << k);
  const int cus = ctx.info().cu_count;
  Buffer de = ctx.alloc(sizeof(double) * 4 * size_t(n));  // d, e, tau, eigenvalues
  Buffer vr = ctx.alloc(sizeof(double) * size_t(n) * n);
  Buffer scr = ctx.alloc(sizeof(double) * kern::eig_tridiag_scratch_doubles(n, cus));
  Buffer bar = ctx.alloc(sizeof(unsigned) * (size_t(cus) + 64));
  double* d = de.as<double>();
  double* e = d + n;
  double* tau = e + n;
  double* lam = tau + n;
  Event e0, e1, eb0, eb1, e2, e3;
  e0.record(s);
  OAP_HIP_CHECK(hipMemsetAsync(e, 0, sizeof(double) * n, s));
  kern::eig_tridiag(a, n, cus, d, e, vr.as<double>(), tau, scr.as<double>(),
                    reinterpret_cast<unsigned*>(bar.data()), s);
  e1.record(s);
  unsigned abort_word = 0;
  if (kern::eig_vectors_supported(n, k) && !knob_on("OAP_EIG_HOST_INVIT")) {
    // the rest on the device (kern::eig_top_vectors): bracket, bisection, selection, inverse
    // iteration, back-transform and signs — only the results come back
    Buffer zb = ctx.alloc(sizeof(double) * size_t(n) * k);
    Buffer sb = ctx.alloc(sizeof(double) * kern::eig_vectors_scratch_doubles(n, k));
    eb0.record(s);
    kern::eig_top_vectors(d, e, n, k, vr.as<double>(), tau, lam, zb.as<double>(), sb.as<double>(),
                          s);
    eb1.record(s);
    std::vector<double> vals(n);
    SymEig out;
    out.n = n;
    out.vectors.resize(size_t(n) * k);
    ctx.copy_to_host(vals.data(), lam, sizeof(double) * n, s);
    ctx.copy_to_host(out.vectors.data(), zb.data(), sizeof(double) * out.vectors.size(), s);
    ctx.copy_to_host(&abort_word, bar.data(), sizeof(unsigned), s);
    OAP_CHECK(abort_word == 0, "eig_tridiag: exchange timed out (workgroups not co-resident)");
    std::vector<int> perm(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    std::stable_sort(perm.begin(), perm.end(),
                     [&](int x, int y) { return std::fabs(vals[x]) > std::fabs(vals[y]); });
    out.values.resize(n);
    for (int j = 0; j < n; ++j) out.values[j] = vals[perm[j]];
    if (timing) {
      timing->tridiag_ms = Event::elapsed_ms(e0, e1);
      timing->bisect_ms = Event::elapsed_ms(eb0, eb1);  // (bisection .. signs, on the device)
      timing->backtransform_ms = 0.0;
      timing->host_ms = 0.0;
    }
    return out;
  }
  std::vector<double> hd(2 * size_t(n));
  ctx.copy_to_host(hd.data(), d, sizeof(double) * 2 * n, s);
  ctx.copy_to_host(&abort_word, bar.data(), sizeof(unsigned), s);
  OAP_CHECK(abort_word == 0, "eig_tridiag: exchange timed out (workgroups not co-resident)");
  std::vector<double> hdiag(hd.begin(), hd.begin() + n), hoff(hd.begin() + n, hd.end());
  hoff[n - 1] = 0.0;
  // Gershgorin bracket and the Sturm-count pivot floor (LAPACK dstebz conventions)
  double lo = hdiag[0], hi = hdiag[0], emax2 = 0.0, tnorm = 0.0;
  for (int i = 0; i < n; ++i) {
    const double r =
        (i > 0 ? std::fabs(hoff[i - 1]) : 0.0) + (i + 1 < n ? std::fabs(hoff[i]) : 0.0);
    lo = std::min(lo, hdiag[i] - r);
    hi = std::max(hi, hdiag[i] + r);
    tnorm = std::max(tnorm, std::fabs(hdiag[i]) + r);
    if (i + 1 < n) emax2 = std::max(emax2, hoff[i] * hoff[i]);
  }
  const double pivmin = std::numeric_limits<double>::min() * std::max(1.0, emax2);
  const double pad = 2.0 * std::numeric_limits<double>::epsilon() * tnorm + 4.0 * pivmin;
  lo -= pad;
  hi += pad;
  eb0.record(s);
  kern::eig_bisect(d, e, n, lo, hi, pivmin, lam, s);
  eb1.record(s);
  std::vector<double> vals(n);
  ctx.copy_to_host(vals.data(), lam, sizeof(double) * n, s);
  const auto th = std::chrono::steady_clock::now();
  double dev_ms = 0.0;
  Buffer zb;
  SymEig out = sym_eig_from_tridiag(
      hdiag, hoff, n, k,
      [&](std::vector<double>& z, int kk) {
        zb = ctx.alloc(sizeof(double) * size_t(n) * kk);
        ctx.copy_to_backend(zb.data(), z.data(), sizeof(double) * z.size(), s);
        e2.record(s);
        kern::eig_apply_q(vr.as<double>(), tau, n, kk, zb.as<double>(), s);
        e3.record(s);
        ctx.copy_to_host(z.data(), zb.data(), sizeof(double) * z.size(), s);
        dev_ms = Event::elapsed_ms(e2, e3);
      },
      &vals, &ctx.pool());
  if (timing) {
    timing->tridiag_ms = Event::elapsed_ms(e0, e1);
    timing->bisect_ms = Event::elapsed_ms(eb0, eb1);
    timing->backtransform_ms = dev_ms;
    timing->host_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th).count() -
        dev_ms;
  }
  return out;
}

}  // namespace oap
