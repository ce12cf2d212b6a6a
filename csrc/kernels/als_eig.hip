// Eigendecomposition of the ALS source Gramian Y^T Y on the device, for the low-rank (Woodbury)
// solve of short rows (kernels/als_lowrank.hip): Y^T Y = Q diag(eig) Q^T.
//
// The reference solves every row against the full normal equations inside oneDAL's step4Local
// (mllib-dal/src/main/native/ALSDALImpl.cpp:301-316).  Here the eigenbasis is computed once per
// half-iteration, on the GPU, in the same stream as the Gramian allreduce that produced it: no
// device -> host copy, no host eigensolver, no host wait inside the ALS iteration.
//
// One 1024-thread workgroup runs a cyclic parallel Jacobi in fp64: the n (= r rounded up to
// even) indices play a round-robin tournament, so each round has n/2 disjoint (p, q) pairs whose
// rotations are independent; a round is one rotation-parameter phase, one row phase (J^T A) and
// one column phase (A J, and V J) with a barrier after each.  A lives in LDS (odd row stride:
// 2-way bank conflicts at most on the column phase); V lives in LDS too when both fit in the
// 160 KB (r <= 100), otherwise in global memory (L2-resident, 128 KB).  Sweeps stop when the
// off-diagonal mass is below tol^2 of the total.
#include <hip/hip_runtime.h>

#include "kernels/kernels.h"
#include "runtime/common.h"

namespace oap {
namespace kern {

namespace {

constexpr int kEigThreads = 1024;

// round-robin tournament seat of player m in round t (player 0 fixed, the others rotate)
__device__ inline int rr_pos(int m, int t, int n) {
  return m == 0 ? 0 : ((m - 1 + t) % (n - 1)) + 1;
}

template <bool VLDS>
__global__ __launch_bounds__(kEigThreads) void oap_als_jacobi_eig(const double* __restrict__ G,
                                                                   int r, int ld,
                                                                   double* __restrict__ vglob,
                                                                   float* __restrict__ Q,
                                                                   float* __restrict__ QT,
                                                                   float* __restrict__ eig,
                                                                   int max_sweeps, double tol,
                                                                   unsigned long long* status) {
  extern __shared__ double sm[];
  const int n = r + (r & 1), S = n + 1, np = n / 2;
  const int tid = threadIdx.x;
  double* A = sm;
  double* V = VLDS ? sm + n * S : vglob;
  double* rot = VLDS ? V + n * S : A + n * S;  // [np][2]: c, s
  double* red = rot + 2 * np;                  // [2 * 16] wave partials
  for (int idx = tid; idx < n * n; idx += kEigThreads) {
    const int i = idx / n, j = idx - i * n;
    A[i * S + j] = (i < r && j < r) ? G[i * r + j] : 0.0;
    V[i * S + j] = i == j ? 1.0 : 0.0;
  }
  __syncthreads();
  bool converged = false;
  for (int sweep = 0; sweep < max_sweeps; ++sweep) {
    // convergence: off-diagonal vs total Frobenius mass
    double off = 0.0, tot = 0.0;
    for (int idx = tid; idx < n * n; idx += kEigThreads) {
      const int i = idx / n, j = idx - i * n;
      const double v = A[i * S + j];
      tot += v * v;
      if (i != j) off += v * v;
    }
    for (int m = 32; m >= 1; m >>= 1) {
      off += __shfl_xor(off, m, 64);
      tot += __shfl_xor(tot, m, 64);
    }
    if ((tid & 63) == 0) {
      red[2 * (tid >> 6)] = off;
      red[2 * (tid >> 6) + 1] = tot;
    }
    __syncthreads();
    off = tot = 0.0;
    for (int w = 0; w < kEigThreads / 64; ++w) {
      off += red[2 * w];
      tot += red[2 * w + 1];
    }
    if (off <= tol * tol * tot) {  // (uniform: every thread read the same partials)
      converged = true;
      break;
    }
    __syncthreads();                     // red is rewritten next sweep
    for (int t = 0; t < n - 1; ++t) {
      if (tid < np) {  // rotation of pair tid: zeroes A[p][q] (sym.schur2)
        const int p = rr_pos(tid, t, n), q = rr_pos(n - 1 - tid, t, n);
        const double apq = A[p * S + q];
        double c = 1.0, s = 0.0;
        if (fabs(apq) > 1e-300) {
          const double tau = (A[q * S + q] - A[p * S + p]) / (2.0 * apq);
          const double tt = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
          c = 1.0 / sqrt(1.0 + tt * tt);
          s = tt * c;
        }
        rot[2 * tid] = c;
        rot[2 * tid + 1] = s;
      }
      __syncthreads();
      for (int task = tid; task < np * n; task += kEigThreads) {  // rows p, q: J^T A
        const int k = task / n, col = task - k * n;
        const int p = rr_pos(k, t, n), q = rr_pos(n - 1 - k, t, n);
        const double c = rot[2 * k], s = rot[2 * k + 1];
        const double ap = A[p * S + col], aq = A[q * S + col];
        A[p * S + col] = c * ap - s * aq;
        A[q * S + col] = s * ap + c * aq;
      }
      __syncthreads();
      for (int task = tid; task < np * n; task += kEigThreads) {  // cols p, q: A J and V J
        const int k = task / n, row = task - k * n;
        const int p = rr_pos(k, t, n), q = rr_pos(n - 1 - k, t, n);
        const double c = rot[2 * k], s = rot[2 * k + 1];
        const double ap = A[row * S + p], aq = A[row * S + q];
        A[row * S + p] = c * ap - s * aq;
        A[row * S + q] = s * ap + c * aq;
        const double vp = V[row * S + p], vq = V[row * S + q];
        V[row * S + p] = c * vp - s * vq;
        V[row * S + q] = s * vp + c * vq;
      }
      __syncthreads();
    }
  }
  // the low-rank solve's operands: Q (ld x ld, identity padding), Q^T, eigenvalues (padding 1)
  for (int idx = tid; idx < ld * ld; idx += kEigThreads) {
    const int k = idx / ld, j = idx - k * ld;
    const float v = (k < r && j < r) ? float(V[k * S + j]) : (k == j ? 1.f : 0.f);
    Q[k * ld + j] = v;
    QT[j * ld + k] = v;
  }
  for (int j = tid; j < ld; j += kEigThreads) eig[j] = j < r ? float(fmax(A[j * S + j], 0.0)) : 1.f;
  // solves whose basis missed the tolerance within max_sweeps (the host reads it at its
  // per-iteration sync and reports it)
  if (tid == 0 && status && !converged) atomicAdd(status, 1ull);
}

size_t eig_lds_bytes(int r, bool vlds) {
  const size_t n = size_t(r + (r & 1)), S = n + 1;
  return ((vlds ? 2 : 1) * n * S + n + 32) * sizeof(double);
}

}  // namespace

size_t als_gram_eig_scratch_bytes(int r) {
  const size_t n = size_t(r + (r & 1));
  return eig_lds_bytes(r, true) <= 160 * 1024 ? 16 : n * (n + 1) * sizeof(double);
}

void als_gram_eig(const double* gram, int r, int ld, double* scratch, float* Q, float* QT,
                  float* eig, hipStream_t s, int max_sweeps, double tol,
                  unsigned long long* status) {
  OAP_CHECK(r >= 1 && r <= 128 && ld >= r && ld <= 128, "als_gram_eig: r <= ld <= 128");
  const bool vlds = eig_lds_bytes(r, true) <= 160 * 1024;
  const size_t lds = eig_lds_bytes(r, vlds);
  if (vlds) {
    static bool attr = false;
    if (!attr) {
      OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_als_jacobi_eig<true>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(oap_als_jacobi_eig<true>, dim3(1), dim3(kEigThreads), lds, s, gram, r, ld,
                       nullptr, Q, QT, eig, max_sweeps, tol, status);
  } else {
    static bool attr = false;
    if (!attr) {
      OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_als_jacobi_eig<false>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(oap_als_jacobi_eig<false>, dim3(1), dim3(kEigThreads), lds, s, gram, r,
                       ld, scratch, Q, QT, eig, max_sweeps, tol, status);
  }
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
