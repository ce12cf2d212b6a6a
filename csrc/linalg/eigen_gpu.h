// GPU symmetric eigensolver for PCA (fp64): device tridiagonalisation (kernels/eig.hip), the
// O(n^2) tridiagonal stage on the host (QL eigenvalues + inverse iteration for the k wanted
// vectors, linalg/eigen.cpp), device back-transformation.  Replaces the reference's master-rank
// svdDense finalisation (mllib-dal/src/main/native/PCADALImpl.cpp:127-150).
#pragma once

#include <hip/hip_runtime.h>

#include "linalg/eigen.h"
#include "runtime/context.h"

namespace oap {

struct GpuEigTiming {
  double tridiag_ms = 0.0, bisect_ms = 0.0, host_ms = 0.0, backtransform_ms = 0.0;
};

// Whether the device path handles an n x n problem keeping k vectors on this context.
bool sym_eig_gpu_supported(const Context& ctx, int n, int k);

// a: device n x n symmetric (row-major).  Same contract as sym_eig_topk.
SymEig sym_eig_topk_gpu(Context& ctx, const double* a, int n, int k, hipStream_t s,
                        GpuEigTiming* timing = nullptr);

}  // namespace oap
