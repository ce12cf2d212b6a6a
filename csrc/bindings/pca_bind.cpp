// PCA bindings: the role of the reference's JNI entry PCADALImpl.cPCATrainDAL
// (mllib-dal/src/main/native/javah/org_apache_spark_ml_feature_PCADALImpl.h:12-16), returning
// arrays instead of filling PCAResult fields with leaked native table handles.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "bindings/bindings.h"
#include "drivers/pca.h"
#include "linalg/eigen.h"
#include "linalg/eigen_gpu.h"

namespace py = pybind11;
using namespace oap;

namespace {

py::array_t<double> to_array(const std::vector<double>& v, int64_t rows, int64_t cols) {
  py::array_t<double> a({rows, cols});
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(double));
  return a;
}

}  // namespace

void register_pca(py::module_& m) {
  m.def(
      "pca_fit",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<Comm> comm, std::shared_ptr<DenseTable> t,
         int k, bool precise, bool gpu_eig, bool exact) {
        PcaParams p;
        p.k = k;
        p.precise = precise;
        p.gpu_eig = gpu_eig;
        p.exact = exact;
        PcaResult r;
        {
          py::gil_scoped_release rel;
          r = pca_fit(*ctx, *comm, *t, p);
        }
        py::dict out;
        out["pc"] = to_array(r.pc, r.d, r.k);
        out["explained_variance"] = r.explained;
        out["eigenvalues"] = r.eigenvalues;
        out["mean"] = r.mean;
        out["n"] = r.n;
        out["stats_ms"] = r.stats_ms;
        out["allreduce_ms"] = r.allreduce_ms;
        out["eig_ms"] = r.eig_ms;
        out["total_ms"] = r.total_ms;
        out["eig_on_gpu"] = r.eig_on_gpu;
        out["eig_tridiag_ms"] = r.eig_tridiag_ms;
        out["eig_host_ms"] = r.eig_host_ms;
        out["eig_backtransform_ms"] = r.eig_backtransform_ms;
        out["engine"] = r.engine;
        out["err_bound"] = r.err_bound;
        return out;
      },
      py::arg("ctx"), py::arg("comm"), py::arg("table"), py::arg("k"),
      py::arg("precise") = false, py::arg("gpu_eig") = true, py::arg("exact") = false);
  m.def(
      "pca_covariance",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<Comm> comm, std::shared_ptr<DenseTable> t,
         bool precise, bool exact) {
        PcaParams p;
        p.precise = precise;
        p.exact = exact;
        PcaCovariance c;
        {
          py::gil_scoped_release rel;
          c = pca_covariance(*ctx, *comm, *t, p);
        }
        py::dict out;
        out["cov"] = to_array(c.cov, c.d, c.d);
        out["mean"] = c.mean;
        out["n"] = c.n;
        out["stats_ms"] = c.stats_ms;
        out["allreduce_ms"] = c.allreduce_ms;
        out["engine"] = c.engine;
        out["err_bound"] = c.err_bound;
        out["scales_redone"] = c.scales_redone;
        out["fallback_fp64"] = c.fallback_fp64;
        out["int8_rel_bound"] = c.int8_rel_bound;
        return out;
      },
      py::arg("ctx"), py::arg("comm"), py::arg("table"), py::arg("precise") = false,
      py::arg("exact") = false);
  m.def(
      "sym_eig",
      [](py::array_t<double, py::array::c_style | py::array::forcecast> a, int k, int threads) {
        if (a.ndim() != 2 || a.shape(0) != a.shape(1))
          throw ConfigError("sym_eig expects a square matrix");
        const int n = static_cast<int>(a.shape(0));
        if (k <= 0 || k > n) k = n;
        std::vector<double> A(a.data(), a.data() + a.size());
        SymEig e;
        {
          py::gil_scoped_release rel;
          ThreadPool pool(threads > 0 ? threads : 1);
          e = sym_eig_topk(A, n, k, &pool);
        }
        return py::make_tuple(e.values, to_array(e.vectors, n, k));
      },
      py::arg("a"), py::arg("k") = 0, py::arg("threads") = 4,
      "Eigen-decomposition of a symmetric matrix: (values sorted by |.| desc, vectors n x k).");
  m.def(
      "sym_eig_gpu",
      [](std::shared_ptr<Context> ctx,
         py::array_t<double, py::array::c_style | py::array::forcecast> a, int k) {
        if (a.ndim() != 2 || a.shape(0) != a.shape(1))
          throw ConfigError("sym_eig_gpu expects a square matrix");
        const int n = static_cast<int>(a.shape(0));
        if (k <= 0 || k > n) k = n;
        SymEig e;
        GpuEigTiming t;
        {
          py::gil_scoped_release rel;
          hipStream_t s = ctx->compute();
          Buffer da = ctx->alloc(sizeof(double) * size_t(n) * n);
          ctx->copy_to_backend(da.data(), a.data(), sizeof(double) * size_t(n) * n, s);
          e = sym_eig_topk_gpu(*ctx, da.as<double>(), n, k, s, &t);
        }
        py::dict tm;
        tm["tridiag_ms"] = t.tridiag_ms;
        tm["bisect_ms"] = t.bisect_ms;
        tm["host_ms"] = t.host_ms;
        tm["backtransform_ms"] = t.backtransform_ms;
        return py::make_tuple(e.values, to_array(e.vectors, n, k), tm);
      },
      py::arg("ctx"), py::arg("a"), py::arg("k"),
      "Device eigensolver (tridiagonalisation + back-transform on the GPU): (values, vectors, "
      "timing).");
}
