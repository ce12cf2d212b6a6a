// Distributed PCA driver.
//
// MI355X-native counterpart of the reference's PCA path: Spark-side mean centring
// (mllib-dal/src/main/scala/org/apache/spark/ml/feature/PCADALImpl.scala:101-106), oneDAL
// step1Local on every rank + allgatherv of serialized partials + step2Master on rank 0
// (native/PCADALImpl.cpp:63-153), then top-k extraction and explained variance on the driver
// (PCADALImpl.scala:108-135).  Here: one fused shifted SYRK pass per rank (kernels/pca.hip),
// ONE allreduce of [S | column sums] (d^2 + d doubles), the fp64 covariance correction and the
// hand-written symmetric eigensolver (linalg/eigen.cpp) evaluated redundantly on every rank —
// no root and no broadcast.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "comm/comm.h"
#include "runtime/context.h"
#include "runtime/table.h"

namespace oap {

struct PcaParams {
  int k = 1;
  bool precise = false;  // 4-term bf16 split products (adds lo*lo); default 3-term
  // reference precision (oneDAL fp64, PCADALImpl.cpp:31): fp64 products and sums of f32 or f64
  // rows on the fp64 MFMA; the fast path (bf16 split products) otherwise
  bool exact = false;
  int flush_rows = 4096; // rows accumulated in fp32 before the fp64 flush (GPU)
  bool gpu_eig = true;   // device eigensolver (linalg/eigen_gpu.h) when the context is a GPU
};

struct PcaCovariance {
  int d = 0;
  int64_t n = 0;             // global rows
  std::vector<double> cov;   // d x d sample covariance (divided by n - 1), row-major
  std::vector<double> mean;  // d
  double stats_ms = 0.0;     // local SYRK + reduce (device time on GPU)
  double allreduce_ms = 0.0;
  // GPU engine with device_cov requested: `cov` stays empty and the covariance is here instead
  // ([d][d] doubles on the device; the GPU eigensolver reads it without a host round trip)
  Buffer dev_cov;
  // which kernel formed S: "int8_digits" (exact mode, f32 rows: kernels/pca_ozaki.hip),
  // "fp64_mfma" (exact mode, f64 rows or OAP_PCA_EXACT_ENGINE=fp64), "bf16_split" (fast), "cpu"
  std::string engine;
  // int8_digits: a bound on max_jk |cov_jk - cov_exact_jk| from the digit products (the
  // statistics' own error; the fp64 correction c c^T / n is the fp64 path's); else 0
  double err_bound = 0.0;
  // int8_digits: the column scales sampled from 65536 rows proved too small (a digit overflowed)
  // and the pass was redone with scales from every row
  bool scales_redone = false;
  // int8_digits gave a bound above 1e-10 of the largest variance: redone on the fp64 MFMA
  bool fallback_fp64 = false;
  double int8_rel_bound = 0.0;  // the int8 engine's err_bound / largest variance (diagnostic)
};

struct PcaResult {
  int d = 0, k = 0;
  int64_t n = 0;
  std::vector<double> pc;           // d x k row-major (column j = j-th principal component)
  std::vector<double> explained;    // k: |lambda_j| / sum_i |lambda_i|
  std::vector<double> eigenvalues;  // all d, |.|-descending
  std::vector<double> mean;
  double stats_ms = 0.0, allreduce_ms = 0.0, eig_ms = 0.0, total_ms = 0.0;
  bool eig_on_gpu = false;
  double eig_tridiag_ms = 0.0, eig_host_ms = 0.0, eig_backtransform_ms = 0.0;
  std::string engine;       // PcaCovariance::engine
  double err_bound = 0.0;   // PcaCovariance::err_bound
};

PcaCovariance pca_covariance(Context& ctx, Comm& comm, DenseTable& x, const PcaParams& p,
                             bool device_cov = false);
PcaResult pca_fit(Context& ctx, Comm& comm, DenseTable& x, const PcaParams& p);

}  // namespace oap
