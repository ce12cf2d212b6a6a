// Dense symmetric eigensolver (fp64, host, thread-parallel) — the replacement for the reference's
// oneDAL `pca::Distributed<step2Master, svdDense>` finalisation (mllib-dal/src/main/native/
// PCADALImpl.cpp:127-153), which returned the full eigenvalue vector and eigenvector matrix.
//
// Algorithm: Householder tridiagonalisation (Q explicit), implicit-shift QL on the tridiagonal
// matrix with the Givens rotation sequence recorded, then the rotations applied to Q^T in
// column slices on the thread pool (rows of the eigenvector matrix are independent).
#pragma once

#include <cstdint>
#include <functional>
#include <vector>

#include "runtime/thread_pool.h"

namespace oap {

struct SymEig {
  int n = 0;
  std::vector<double> values;   // n eigenvalues, sorted by |lambda| descending (SVD order)
  std::vector<double> vectors;  // n x n row-major, column j = unit eigenvector of values[j]
};

// A: n x n symmetric, row-major (only read).  Eigenvector signs are normalised so that the
// largest-magnitude component of each vector is positive (deterministic across runs and ranks).
SymEig sym_eig(const std::vector<double>& A, int n, ThreadPool* pool);

// Same, only the first `k` eigenvectors are kept (values still hold all n eigenvalues).
SymEig sym_eig_topk(const std::vector<double>& A, int n, int k, ThreadPool* pool);

// From an already tridiagonalised A = Q T Q^T (d: n diagonal, e: n off-diagonal, e[n-1] = 0):
// all eigenvalues (QL, or the given `eigvals` in any order) and the first `keep` eigenvectors of
// T (inverse iteration), which apply_q(z, keep) maps to eigenvectors of A in place (z: n x keep
// row-major).  The GPU path (linalg/eigen_gpu.h) tridiagonalises, bisects and back-transforms on
// the device around this.
SymEig sym_eig_from_tridiag(const std::vector<double>& d, const std::vector<double>& e, int n,
                            int keep,
                            const std::function<void(std::vector<double>&, int)>& apply_q,
                            const std::vector<double>* eigvals = nullptr,
                            ThreadPool* pool = nullptr);

}  // namespace oap
