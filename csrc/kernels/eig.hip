// GPU symmetric eigensolver pieces for PCA (fp64): the reference finalises PCA with oneDAL's
// step2Master svdDense on the master rank (mllib-dal/src/main/native/PCADALImpl.cpp:127-150);
// here every rank runs it on its own GPU.
//
// oap_eig_tridiag — Householder tridiagonalisation A = Q T Q^T as ONE persistent cooperative
// kernel with the matrix resident in LDS across the whole chip: workgroup g (of G, one per CU)
// keeps rows i = g, g + G, ... (full rows, fp64) in its LDS for the entire reduction, so the
// O(n^3) traffic never leaves the CUs.  Per reflector j the only global traffic is the column
// being reduced and the product y = tau A v (published by their row owners) and per-workgroup
// partial sums, exchanged ONCE per reflector as step-tagged values that readers poll directly
// (no barrier: see tstore).  The rank-2 update of reflector j-1 is applied lazily, fused into the
// pass that forms y for reflector j (one LDS sweep of the trailing rows per step).  Partial sums
// are reduced in workgroup order by every workgroup: all of them derive bitwise-identical
// scalars (beta, tau, v^T y) without a broadcast.
//
// oap_eig_apply_q — V = Q Z for the selected tridiagonal eigenvectors Z (n x k): one workgroup per
// column, reflectors applied last to first from the stored reflector rows.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "kernels/device_utils.h"
#include "kernels/kernels.h"
#include "runtime/knobs.h"

namespace oap {
namespace kern {

namespace {

constexpr int kEigThreads = 256;
constexpr int kEigMaxRows = 8;  // rows per workgroup (n <= 8 G)
constexpr int kEigLdsCap = 159 * 1024;  // dynamic LDS (the kernels' own static LDS fits beside)

struct EigArgs {
  const double* a;  // n x n symmetric (row-major, full)
  int n, G, R;      // size, workgroups, rows per workgroup (ceil(n / G))
  double* d;        // n      diagonal of T
  double* e;        // n - 1  off-diagonal of T
  double* vrows;    // n x n  row j = reflector j (indices j+1..n-1), unnormalised (v0 = x0 - beta)
  double* tau;      // n
  double* xcol;     // n      published column / product (step scratch)
  double* ycol;     // n
  unsigned* bar;    // bar[0]: abort word (zeroed by the launch)
};

__device__ inline double block_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double s = wave_sum_f64(v);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const double t = ((red[0] + red[1]) + red[2]) + red[3];
  __syncthreads();
  return t;
}

// Reflector from the column x = [x0, tail] (tail = sum of squares below x0), the host
// solver's convention (linalg/eigen.cpp make_reflector): H x = beta e0, v0 = x0 - beta.
__device__ inline void make_reflector(double x0, double tail, double& beta, double& tau,
                                      double& v0) {
  beta = x0;
  tau = 0.0;
  v0 = 1.0;
  if (tail > 0.0) {
    const double nx = sqrt(x0 * x0 + tail);
    beta = x0 >= 0.0 ? -nx : nx;
    v0 = x0 - beta;
    tau = 2.0 / (v0 * v0 + tail);
  }
}

// Tagged exchange: a published double carries its step in the 2 lowest mantissa bits (step mod
// 4; the buffers alternate by step parity, so a stale value is always two steps old and its tag
// differs).  Readers poll the values themselves — no flag, no store-completion wait — so one
// exchange costs one store propagation plus one read.  (The 2 bits perturb an exchanged value
// by at most 3 ulp; every workgroup reads the same bits, so the reduction stays consistent.)
__device__ inline void tstore(double* p, double v, unsigned t) {
  const unsigned long long b =
      (static_cast<unsigned long long>(__double_as_longlong(v)) & ~3ull) | t;
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), b, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long tload_bits(const double* p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double bits_value(unsigned long long b) {
  return __longlong_as_double(static_cast<long long>(b));
}

// Polls up to 32 slots (bit q of `mask` set: slot q of ptr) until each carries tag t; returns
// false (and raises the abort word) after ~0.5 s or when another workgroup aborted.
template <int M>
__device__ inline bool tpoll(const double* (&ptr)[M], unsigned mask, unsigned t, double (&out)[M],
                             unsigned* abort_word) {
  for (unsigned spin = 0;; ++spin) {
#pragma unroll
    for (int q = 0; q < M; ++q) {
      if (mask & (1u << q)) {
        const unsigned long long b = tload_bits(ptr[q]);
        if (unsigned(b & 3ull) == t) {
          out[q] = bits_value(b);
          mask &= ~(1u << q);
        }
      }
    }
    if (mask == 0) return true;
    if ((spin & 63u) == 63u &&
        (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
         spin > (1u << 20))) {
      __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Sum over the workgroup (one value per thread, fixed shuffle tree and wave order: identical
// bits in every workgroup for identical inputs).  red: 4 doubles, not reused before the next
// __syncthreads of the caller.
__device__ inline double block_reduce(double x, double* red) {
  const double s = wave_sum_f64(x);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// One exchange per reflector.  Step j: each wave owns rows of the workgroup; the fused LDS pass
// applies the pending update of reflector j-1 to them and forms y_i = tau (A v_j)_i and
// alpha_i = a_i - y_i v_{j+1} (a = column j+1 after the pending update).  Those two values per
// row are the ONLY data exchanged.  Every workgroup then holds the full y and alpha and derives,
// redundantly and bitwise-identically: v^T y, w_j = y - (tau/2)(v^T y) v (the next pending
// update), the next column c = alpha + beta_c v (beta_c = tau (v^T y) v_{j+1} - y_{j+1}), its
// exact tail norm and reflector j+1.
__global__ __launch_bounds__(kEigThreads) void oap_eig_tridiag(EigArgs a) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = a.n, G = a.G, R = a.R, g = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  double* rows = reinterpret_cast<double*>(smem);  // R x n
  double* pv = rows + size_t(R) * n;                // pending reflector (step j-1)
  double* pw = pv + n;                              // pending w (step j-1)
  double* v = pw + n;                               // current reflector
  double* redA = v + n;                             // block reductions (4 + 4)
  double* redB = redA + 4;
  unsigned* abort_word = a.bar;
  constexpr int kPer = 8;  // n <= 8 * kEigThreads: own columns l = base + tid + q * 256
  auto acol_b = [&](int j) { return a.xcol + (j & 1) * n; };  // alpha (column 0 at init)
  auto ycol_b = [&](int j) { return a.ycol + (j & 1) * n; };  // y

  for (int r = 0; r < R; ++r) {
    const int i = g + r * G;
    for (int l = tid; l < n; l += kEigThreads)
      rows[size_t(r) * n + l] = i < n ? a.a[size_t(i) * n + l] : 0.0;
  }
  for (int l = tid; l < n; l += kEigThreads) {
    pv[l] = 0.0;
    pw[l] = 0.0;
  }
  __syncthreads();

  // ---- reflector 0 from column 0 (the buffers and tag of "step -1")
  double tau = 0.0;
  {
    double* acol = acol_b(1);
    const unsigned t = 3u;
    if (tid < R) {
      const int i = g + tid * G;
      if (i == 0) a.d[0] = rows[0];
      else if (i < n) tstore(acol + i, rows[size_t(tid) * n], t);
    }
    const double* ptr[kPer + 1];
    double val[kPer + 1];
    unsigned mask = 1u << kPer;
    ptr[kPer] = acol + 1;  // x0 (every thread)
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int l = 2 + tid + q * kEigThreads;
      ptr[q] = acol + (l < n ? l : 1);
      if (l < n) mask |= 1u << q;
    }
#pragma unroll
    for (int q = 0; q <= kPer; ++q) val[q] = 0.0;
    const bool ok = tpoll(ptr, mask, t, val, abort_word);
    if (__syncthreads_or(!ok)) return;
    double tl = 0.0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) tl += val[q] * val[q];
    const double tail = block_reduce(tl, redA);
    double beta, v0;
    make_reflector(val[kPer], tail, beta, tau, v0);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int l = 2 + tid + q * kEigThreads;
      if (l < n) {
        v[l] = val[q];
        if (g == 0) a.vrows[l] = val[q];
      }
    }
    if (tid == 0) {
      v[1] = v0;
      if (g == 0) {
        a.vrows[1] = v0;
        a.e[0] = beta;
        a.tau[0] = tau;
      }
    }
    __syncthreads();
  }

  for (int j = 0; j + 2 < n; ++j) {
    double* acol = acol_b(j);
    double* ycol = ycol_b(j);
    const unsigned t = unsigned(j & 3);
    const double vj1 = v[j + 1];
    // ---- fused pass (wave w: own rows r = w, w + 4, ...): pending update on columns >= j+1,
    // y_i = tau (A v)_i, alpha_i; published by lane 0
    for (int r = wave; r < R; r += kEigThreads / 64) {
      const int i = g + r * G;
      if (i < j + 1 || i >= n) continue;  // (wave-uniform)
      double* row = rows + size_t(r) * n;
      const double pvi = pv[i], pwi = pw[i];
      double acc = 0.0;
      for (int l = j + 1 + lane; l < n; l += 64) {
        const double x = row[l] - (pvi * pw[l] + pwi * pv[l]);
        row[l] = x;
        acc += x * v[l];
      }
      const double y = tau * wave_sum_f64(acc);
      if (lane == 0) {
        tstore(ycol + i, y, t);
        tstore(acol + i, row[j + 1] - y * vj1, t);
      }
    }
    // ---- every workgroup: the full y and alpha of step j
    const double* ptr[2 * kPer + 3];
    double val[2 * kPer + 3];
    unsigned mask = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int l = j + 1 + tid + q * kEigThreads;
      const int lc = l < n ? l : j + 1;
      ptr[q] = ycol + lc;
      ptr[kPer + q] = acol + lc;
      if (l < n) mask |= (1u << q) | (1u << (kPer + q));
    }
    ptr[2 * kPer] = ycol + j + 1;      // y_{j+1}
    ptr[2 * kPer + 1] = acol + j + 1;  // alpha_{j+1}
    ptr[2 * kPer + 2] = acol + j + 2;  // alpha_{j+2}
    mask |= 7u << (2 * kPer);
#pragma unroll
    for (int q = 0; q < 2 * kPer + 3; ++q) val[q] = 0.0;
    const bool ok = tpoll(ptr, mask, t, val, abort_word);
    if (__syncthreads_or(!ok)) return;
    double vy = 0.0;
    double vl[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int l = j + 1 + tid + q * kEigThreads;
      vl[q] = l < n ? v[l] : 0.0;
      vy += vl[q] * val[q];
    }
    const double S4 = block_reduce(vy, redA);
    const double hts = 0.5 * tau * S4;
    const double bc = 2.0 * hts * vj1 - val[2 * kPer];
    const double cj1 = val[2 * kPer + 1] + bc * vj1;
    const double x0 = val[2 * kPer + 2] + bc * v[j + 2];
    double cv[kPer];
    double tl = 0.0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int l = j + 1 + tid + q * kEigThreads;
      cv[q] = val[kPer + q] + bc * vl[q];
      if (l >= j + 3 && l < n) tl += cv[q] * cv[q];
    }
    const double tail = block_reduce(tl, redB);  // (every thread has read v above)
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int l = j + 1 + tid + q * kEigThreads;
      if (l < n) {
        pv[l] = vl[q];
        pw[l] = val[q] - hts * vl[q];
      }
    }
    if (j + 3 >= n) {
      // last step: the trailing 2 x 2 block (c_{n-2} = cj1, c_{n-1} = x0)
      __syncthreads();
      if (g == 0 && tid == 0) {
        a.d[n - 2] = cj1;
        a.e[n - 2] = x0;
      }
      if (tid < R) {
        const int i = g + tid * G;
        if (i == n - 1)
          a.d[n - 1] = rows[size_t(tid) * n + n - 1] - (pv[i] * pw[i] + pw[i] * pv[i]);
      }
      break;
    }
    double beta, v0;
    make_reflector(x0, tail, beta, tau, v0);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int l = j + 1 + tid + q * kEigThreads;
      if (l >= j + 3 && l < n) {
        v[l] = cv[q];
        if (g == 0) a.vrows[size_t(j + 1) * n + l] = cv[q];
      }
    }
    if (tid == 1) {  // (thread 1 owns column j + 2)
      v[j + 2] = v0;
      if (g == 0) a.vrows[size_t(j + 1) * n + j + 2] = v0;
    }
    if (g == 0 && tid == 0) {
      a.d[j + 1] = cj1;
      a.e[j + 1] = beta;
      a.tau[j + 1] = tau;
    }
    __syncthreads();
  }
}

// Z (n x k row-major) <- Q Z, Q = H_0 H_1 ... H_{n-3}: one wave per column, the column in
// registers (lane holds rows lane + 64 u), the reflector rows streamed D ahead through a
// register ring so their load latency hides under the previous D reflectors' dot + axpy.
template <int KZ, int D>
__global__ __launch_bounds__(64) void oap_eig_apply_q(const double* vrows, const double* tau,
                                                      int n, int k, double* z) {
#pragma clang fp contract(off)
  const int c = blockIdx.x, lane = threadIdx.x;
  double zc[KZ];
#pragma unroll
  for (int u = 0; u < KZ; ++u) {
    const int l = lane + 64 * u;
    zc[u] = l < n ? z[size_t(l) * k + c] : 0.0;
  }
  double buf[D][KZ];
  double tb[D];
  auto load = [&](int j, double (&b)[KZ], double& t) {
    t = 0.0;
    if (j < 0) return;  // (uniform)
    t = tau[j];
    const double* vr = vrows + size_t(j) * n;
#pragma unroll
    for (int u = 0; u < KZ; ++u) {
      const int l = lane + 64 * u;
      b[u] = (l > j && l < n) ? vr[l] : 0.0;
    }
  };
#pragma unroll
  for (int s = 0; s < D; ++s) load(n - 3 - s, buf[s], tb[s]);
  for (int j = n - 3; j >= 0; j -= D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      if (j - s < 0) break;  // (uniform)
      double dot = 0.0;
#pragma unroll
      for (int u = 0; u < KZ; ++u) dot += buf[s][u] * zc[u];
      const double f = tb[s] * wave_sum_f64(dot);
#pragma unroll
      for (int u = 0; u < KZ; ++u) zc[u] -= f * buf[s][u];
      load(j - s - D, buf[s], tb[s]);
    }
  }
#pragma unroll
  for (int u = 0; u < KZ; ++u) {
    const int l = lane + 64 * u;
    if (l < n) z[size_t(l) * k + c] = zc[u];
  }
}

// All eigenvalues of the symmetric tridiagonal (d, e) by 64-way multisection on Sturm counts:
// wave w of the grid owns eigenvalue index i = w (ascending); each round its 64 lanes count the
// eigenvalues below 64 interior points of the current bracket (the LDL^T recurrence with the
// LAPACK pivmin guard), and the bracket shrinks 65x (about 10 rounds to full fp64 precision).
__global__ __launch_bounds__(kEigThreads) void oap_eig_bisect(const double* d, const double* e,
                                                              int n, double lo0, double hi0,
                                                              double pivmin, double* out) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sd = reinterpret_cast<double*>(smem);
  double* se2 = sd + n;
  for (int i = threadIdx.x; i < n; i += kEigThreads) {
    sd[i] = d[i];
    se2[i] = i + 1 < n ? e[i] * e[i] : 0.0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int idx = blockIdx.x * (kEigThreads / 64) + (threadIdx.x >> 6);  // eigenvalue index
  if (idx >= n) return;  // (wave-uniform; no barrier follows)
  double lo = lo0, hi = hi0;
  for (int round = 0; round < 16; ++round) {
    const double w = hi - lo;
    if (!(w > 2.0 * 2.2204460492503131e-16 * fmax(fabs(lo), fabs(hi)) + 2.0 * pivmin)) break;
    const double x = lo + w * (double(lane + 1) / 65.0);
    int cnt = 0;
    double q = sd[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
    for (int i = 1; i < n; ++i) {
      q = (sd[i] - x) - se2[i - 1] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    // lanes whose point has at most idx eigenvalues below it: a prefix of the wave
    const unsigned long long below = __ballot(cnt <= idx);
    const int L = __popcll(below);
    const double xl = __shfl(x, L > 0 ? L - 1 : 0, 64), xh = __shfl(x, L < 64 ? L : 63, 64);
    if (L > 0) lo = xl;
    if (L < 64) hi = xh;
  }
  if (lane == 0) out[idx] = 0.5 * (lo + hi);
}

// Gershgorin bracket of the tridiagonal and the Sturm-count pivot floor (LAPACK dstebz
// conventions), on the device: out = [lo - pad, hi + pad, pivmin, ||T||_inf].  One block.
__global__ __launch_bounds__(kEigThreads) void oap_eig_gersh(const double* d, const double* e,
                                                             int n, double* out) {
  __shared__ double red[4][4];
  double lo = INFINITY, hi = -INFINITY, tn = 0.0, em = 0.0;
  for (int i = threadIdx.x; i < n; i += kEigThreads) {
    const double r = (i > 0 ? fabs(e[i - 1]) : 0.0) + (i + 1 < n ? fabs(e[i]) : 0.0);
    lo = fmin(lo, d[i] - r);
    hi = fmax(hi, d[i] + r);
    tn = fmax(tn, fabs(d[i]) + r);
    if (i + 1 < n) em = fmax(em, e[i] * e[i]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
    tn = fmax(tn, __shfl_xor(tn, o, 64));
    em = fmax(em, __shfl_xor(em, o, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
    red[2][w] = tn;
    red[3][w] = em;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < kEigThreads / 64; ++q) {
      lo = fmin(lo, red[0][q]);
      hi = fmax(hi, red[1][q]);
      tn = fmax(tn, red[2][q]);
      em = fmax(em, red[3][q]);
    }
    lo = fmin(lo, red[0][0]);
    hi = fmax(hi, red[1][0]);
    tn = fmax(tn, red[2][0]);
    em = fmax(em, red[3][0]);
    const double pivmin = 2.2250738585072014e-308 * fmax(1.0, em);
    const double pad = 2.0 * 2.2204460492503131e-16 * tn + 4.0 * pivmin;
    out[0] = lo - pad;
    out[1] = hi + pad;
    out[2] = pivmin;
    out[3] = tn;
  }
}

// The `keep` eigenvalues of largest magnitude in stable order (ties: lower index — the host
// path's stable sort of the bisection's ascending output), the clusters of close ones (LAPACK
// dstein: |lambda_j - lambda_{j-1}| < 1e-3 ||T||, exact multiples separated by 10 eps ||T||):
// sel [keep], cstart [keep] (index of the cluster's first member).  One block.
__global__ __launch_bounds__(kEigThreads) void oap_eig_select(const double* lam, int n, int keep,
                                                              const double* bracket, double* sel,
                                                              int* cstart) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned char* used = reinterpret_cast<unsigned char*>(smem);
  __shared__ double bv[4];
  __shared__ int bi[4];
  __shared__ int pick;
  for (int i = threadIdx.x; i < n; i += kEigThreads) used[i] = 0;
  __syncthreads();
  for (int t = 0; t < keep; ++t) {
    double v = -1.0;
    int ix = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += kEigThreads) {
      const double a = fabs(lam[i]);
      if (!used[i] && (a > v || (a == v && i < ix))) {
        v = a;
        ix = i;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(ix, o, 64);
      if (ov > v || (ov == v && oi < ix)) {
        v = ov;
        ix = oi;
      }
    }
    if ((threadIdx.x & 63) == 0) {
      bv[threadIdx.x >> 6] = v;
      bi[threadIdx.x >> 6] = ix;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double b = bv[0];
      int j = bi[0];
      for (int q = 1; q < kEigThreads / 64; ++q)
        if (bv[q] > b || (bv[q] == b && bi[q] < j)) {
          b = bv[q];
          j = bi[q];
        }
      used[j] = 1;
      pick = j;
      sel[t] = lam[j];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double tn = bracket[3] == 0.0 ? 1.0 : bracket[3];
    const double ortol = 1e-3 * tn, pert = 10.0 * 2.2204460492503131e-16 * tn;
    for (int j = 0; j < keep; ++j) {
      if (j > 0 && fabs(sel[j] - sel[j - 1]) < ortol) {
        if (fabs(sel[j] - sel[j - 1]) < pert)
          sel[j] = sel[j - 1] + (sel[j] <= sel[j - 1] ? -pert : pert);
        cstart[j] = cstart[j - 1];
      } else {
        cstart[j] = j;
      }
    }
  }
}

// Eigenvectors of the tridiagonal for sel[] by inverse iteration (the host path's recipe,
// linalg/eigen.cpp tridiag_inverse_iteration): one block per cluster head; thread 0 factors
// T - lambda I (LU with partial pivoting, in LDS) and runs the 4 solves, the block does the
// Gram-Schmidt against the cluster's earlier vectors and the normalisation.  z: n x keep
// row-major (column j for sel[j]).
__global__ __launch_bounds__(kEigThreads) void oap_eig_invit(const double* d, const double* e,
                                                             int n, int keep, const double* sel,
                                                             const int* cstart,
                                                             const double* bracket, double* z) {
#pragma clang fp contract(off)
  const int j0 = blockIdx.x;
  if (cstart[j0] != j0) return;  // (block-uniform: only cluster heads work)
  int j1 = j0 + 1;
  while (j1 < keep && cstart[j1] != j1) ++j1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* dd = reinterpret_cast<double*>(smem);
  double* du = dd + n;
  double* du2 = du + n;
  double* dl = du2 + n;
  double* b = dl + n;
  unsigned char* swp = reinterpret_cast<unsigned char*>(b + n);
  __shared__ double red[4];
  const double tn = bracket[3] == 0.0 ? 1.0 : bracket[3];
  const double tiny = 2.2204460492503131e-16 * tn;
  const int tid = threadIdx.x;
  for (int j = j0; j < j1; ++j) {
    const double lambda = sel[j];
    if (tid == 0) {
      for (int i = 0; i < n; ++i) {
        dd[i] = d[i] - lambda;
        du[i] = i + 1 < n ? e[i] : 0.0;
        dl[i] = i + 1 < n ? e[i] : 0.0;
        du2[i] = 0.0;
        swp[i] = 0;
      }
      for (int i = 0; i + 1 < n; ++i) {
        if (fabs(dd[i]) >= fabs(dl[i])) {
          if (dd[i] == 0.0) dd[i] = tiny;
          const double f = dl[i] / dd[i];
          dl[i] = f;
          dd[i + 1] -= f * du[i];
        } else {
          const double f = dd[i] / dl[i];
          dd[i] = dl[i];
          dl[i] = f;
          const double t = du[i];
          du[i] = dd[i + 1];
          dd[i + 1] = t - f * dd[i + 1];
          if (i + 2 < n) {
            du2[i] = du[i + 1];
            du[i + 1] = -f * du[i + 1];
          }
          swp[i] = 1;
        }
      }
      if (dd[n - 1] == 0.0) dd[n - 1] = tiny;
      for (int i = 0; i < n; ++i)
        if (fabs(dd[i]) < tiny) dd[i] = copysign(tiny, dd[i] == 0.0 ? 1.0 : dd[i]);
      uint64_t st = 0x9e3779b97f4a7c15ull * uint64_t(j + 1);  // deterministic start vector
      for (int i = 0; i < n; ++i) {
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        b[i] = double(st >> 11) * (1.0 / 9007199254740992.0) - 0.5;
      }
    }
    __syncthreads();
    for (int it = 0; it < 4; ++it) {
      if (tid == 0) {
        for (int i = 0; i + 1 < n; ++i) {
          if (swp[i]) {
            const double t = b[i];
            b[i] = b[i + 1];
            b[i + 1] = t;
          }
          b[i + 1] -= dl[i] * b[i];
        }
        b[n - 1] /= dd[n - 1];
        if (n >= 2) b[n - 2] = (b[n - 2] - du[n - 2] * b[n - 1]) / dd[n - 2];
        for (int i = n - 3; i >= 0; --i)
          b[i] = (b[i] - du[i] * b[i + 1] - du2[i] * b[i + 2]) / dd[i];
      }
      __syncthreads();
      for (int q = j0; q < j; ++q) {  // MGS against the cluster's vectors
        double part = 0.0;
        for (int i = tid; i < n; i += kEigThreads) part += z[size_t(i) * keep + q] * b[i];
        const double dot = block_reduce(part, red);
        __syncthreads();
        for (int i = tid; i < n; i += kEigThreads) b[i] -= dot * z[size_t(i) * keep + q];
        __syncthreads();
      }
      double part = 0.0;
      for (int i = tid; i < n; i += kEigThreads) part += b[i] * b[i];
      const double nrm = sqrt(block_reduce(part, red));
      __syncthreads();
      if (nrm == 0.0) {
        for (int i = tid; i < n; i += kEigThreads) b[i] = i == j % n ? 1.0 : 0.0;
      } else {
        for (int i = tid; i < n; i += kEigThreads) b[i] /= nrm;
      }
      __syncthreads();
    }
    for (int i = tid; i < n; i += kEigThreads) z[size_t(i) * keep + j] = b[i];
    __threadfence_block();
    __syncthreads();
  }
}

// Sign convention: each column's largest-magnitude component (first among equals) positive.
// One block per column.
__global__ __launch_bounds__(kEigThreads) void oap_eig_signs(double* z, int n, int keep) {
  __shared__ double bv[4];
  __shared__ int bi[4];
  __shared__ double sgn;
  const int c = blockIdx.x;
  double v = -1.0;
  int ix = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += kEigThreads) {
    const double a = fabs(z[size_t(i) * keep + c]);
    if (a > v) {  // (ascending i per thread: the first of equals)
      v = a;
      ix = i;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(ix, o, 64);
    if (ov > v || (ov == v && oi < ix)) {
      v = ov;
      ix = oi;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    bv[threadIdx.x >> 6] = v;
    bi[threadIdx.x >> 6] = ix;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double b = bv[0];
    int j = bi[0];
    for (int q = 1; q < kEigThreads / 64; ++q)
      if (bv[q] > b || (bv[q] == b && bi[q] < j)) {
        b = bv[q];
        j = bi[q];
      }
    sgn = z[size_t(j) * keep + c] < 0.0 ? -1.0 : 1.0;
  }
  __syncthreads();
  if (sgn < 0.0)
    for (int i = threadIdx.x; i < n; i += kEigThreads)
      z[size_t(i) * keep + c] = -z[size_t(i) * keep + c];
}

// Bisection with the bracket on the device (oap_eig_gersh's output)
__global__ __launch_bounds__(kEigThreads) void oap_eig_bisect_dev(const double* d, const double* e,
                                                                  int n, const double* bracket,
                                                                  double* out) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sd = reinterpret_cast<double*>(smem);
  double* se2 = sd + n;
  for (int i = threadIdx.x; i < n; i += kEigThreads) {
    sd[i] = d[i];
    se2[i] = i + 1 < n ? e[i] * e[i] : 0.0;
  }
  __syncthreads();
  const double pivmin = bracket[2];
  const int lane = threadIdx.x & 63;
  const int idx = blockIdx.x * (kEigThreads / 64) + (threadIdx.x >> 6);
  if (idx >= n) return;  // (wave-uniform; no barrier follows)
  double lo = bracket[0], hi = bracket[1];
  for (int round = 0; round < 16; ++round) {
    const double w = hi - lo;
    if (!(w > 2.0 * 2.2204460492503131e-16 * fmax(fabs(lo), fabs(hi)) + 2.0 * pivmin)) break;
    const double x = lo + w * (double(lane + 1) / 65.0);
    int cnt = 0;
    double q = sd[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
    for (int i = 1; i < n; ++i) {
      q = (sd[i] - x) - se2[i - 1] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    const unsigned long long below = __ballot(cnt <= idx);
    const int L = __popcll(below);
    const double xl = __shfl(x, L > 0 ? L - 1 : 0, 64), xh = __shfl(x, L < 64 ? L : 63, 64);
    if (L > 0) lo = xl;
    if (L < 64) hi = xh;
  }
  if (lane == 0) out[idx] = 0.5 * (lo + hi);
}

}  // namespace

void eig_bisect(const double* d, const double* e, int n, double lo, double hi, double pivmin,
                double* out, hipStream_t s) {
  const size_t lds = sizeof(double) * 2 * size_t(n);
  OAP_CHECK(n >= 1 && lds <= size_t(kEigLdsCap), "eig_bisect: n=" << n);
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_eig_bisect),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kEigLdsCap));
    attr = true;
  }
  const int per = kEigThreads / 64;
  hipLaunchKernelGGL(oap_eig_bisect, dim3((n + per - 1) / per), dim3(kEigThreads), lds, s, d, e,
                     n, lo, hi, pivmin, out);
  OAP_HIP_CHECK(hipGetLastError());
}

size_t eig_vectors_scratch_doubles(int n, int keep) { return 4 + size_t(keep) + size_t(keep); }

bool eig_vectors_supported(int n, int keep) {
  return n >= 3 && n <= 8 * kEigThreads && keep >= 1 && keep <= n &&
         size_t(n) * 41 + 64 <= size_t(kEigLdsCap);
}

void eig_top_vectors(const double* d, const double* e, int n, int keep, const double* vrows,
                     const double* tau, double* lam, double* z, double* scratch, hipStream_t s) {
  OAP_CHECK(eig_vectors_supported(n, keep), "eig_top_vectors: n=" << n << " keep=" << keep);
  double* bracket = scratch;           // [4]
  double* sel = scratch + 4;           // [keep]
  int* cstart = reinterpret_cast<int*>(sel + keep);  // [keep] ints (in keep doubles)
  static bool attr = false;
  if (!attr) {
    for (const void* f : {reinterpret_cast<const void*>(&oap_eig_bisect_dev),
                          reinterpret_cast<const void*>(&oap_eig_invit),
                          reinterpret_cast<const void*>(&oap_eig_select)})
      OAP_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        kEigLdsCap));
    attr = true;
  }
  hipLaunchKernelGGL(oap_eig_gersh, dim3(1), dim3(kEigThreads), 0, s, d, e, n, bracket);
  const int per = kEigThreads / 64;
  hipLaunchKernelGGL(oap_eig_bisect_dev, dim3((n + per - 1) / per), dim3(kEigThreads),
                     sizeof(double) * 2 * size_t(n), s, d, e, n, bracket, lam);
  hipLaunchKernelGGL(oap_eig_select, dim3(1), dim3(kEigThreads), size_t(n) + 16, s, lam, n, keep,
                     bracket, sel, cstart);
  hipLaunchKernelGGL(oap_eig_invit, dim3(keep), dim3(kEigThreads), size_t(n) * 41 + 16, s, d, e,
                     n, keep, sel, cstart, bracket, z);
  eig_apply_q(vrows, tau, n, keep, z, s);
  hipLaunchKernelGGL(oap_eig_signs, dim3(keep), dim3(kEigThreads), 0, s, z, n, keep);
  OAP_HIP_CHECK(hipGetLastError());
}

size_t eig_tridiag_lds_bytes(int n, int G) {
  const int R = (n + G - 1) / G;
  // rows, pv / pw / v, two 4-double reduction slots
  return sizeof(double) * (size_t(R) * n + 3 * size_t(n) + 8);
}

int eig_tridiag_grid(int n, int num_cus) {
  // one workgroup per CU (cooperative: all co-resident), at most n of them; fewer workgroups
  // (OAP_EIG_GRID) trade fused-pass parallelism for barrier traffic
  const int cap = int(knob_int("OAP_EIG_GRID"));
  int g = n < num_cus ? n : num_cus;
  if (cap > 0 && cap < g) g = cap;
  while (g > 1 && (n + g - 1) / g > kEigMaxRows) ++g;  // (cannot exceed num_cus for n <= 2048)
  return g;
}

bool eig_tridiag_supported(int n, int num_cus) {
  if (n < 3 || n > 8 * kEigThreads) return false;
  const int G = eig_tridiag_grid(n, num_cus);
  const int R = (n + G - 1) / G;
  return R <= kEigMaxRows && eig_tridiag_lds_bytes(n, G) <= size_t(kEigLdsCap);
}

void eig_tridiag(const double* a, int n, int num_cus, double* d, double* e, double* vrows,
                 double* tau, double* scratch, unsigned* bar, hipStream_t s) {
  OAP_CHECK(eig_tridiag_supported(n, num_cus), "eig_tridiag: unsupported n=" << n);
  EigArgs args;
  args.a = a;
  args.n = n;
  args.G = eig_tridiag_grid(n, num_cus);
  args.R = (n + args.G - 1) / args.G;
  args.d = d;
  args.e = e;
  args.vrows = vrows;
  args.tau = tau;
  args.xcol = scratch;                   // [2][n]
  args.ycol = scratch + 2 * size_t(n);   // [2][n]
  args.bar = bar;
  const size_t lds = eig_tridiag_lds_bytes(n, args.G);
  static bool attr = false;
  if (!attr) {
    OAP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&oap_eig_tridiag),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kEigLdsCap));
    attr = true;
  }
  OAP_HIP_CHECK(hipMemsetAsync(bar, 0, sizeof(unsigned) * (args.G + 1), s));
  // exchange slots start with tag 2 in every word (0xFE bytes): never mistaken for a first write
  OAP_HIP_CHECK(hipMemsetAsync(scratch, 0xFE,
                               sizeof(double) * eig_tridiag_scratch_doubles(n, num_cus), s));
  void* params[] = {&args};
  OAP_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&oap_eig_tridiag),
                                           dim3(args.G), dim3(kEigThreads), params,
                                           static_cast<unsigned>(lds), s));
}

size_t eig_tridiag_scratch_doubles(int n, int num_cus) {
  (void)num_cus;
  return 4 * size_t(n);
}

void eig_apply_q(const double* vrows, const double* tau, int n, int k, double* z, hipStream_t s) {
  OAP_CHECK(n >= 1 && k >= 1 && n <= 2048, "eig_apply_q: bad shape n=" << n << " k=" << k);
  if (n <= 1024)
    hipLaunchKernelGGL((oap_eig_apply_q<16, 4>), dim3(k), dim3(64), 0, s, vrows, tau, n, k, z);
  else
    hipLaunchKernelGGL((oap_eig_apply_q<32, 2>), dim3(k), dim3(64), 0, s, vrows, tau, n, k, z);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
