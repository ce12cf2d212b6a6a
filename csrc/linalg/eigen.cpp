#include "linalg/eigen.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <functional>
#include <numeric>

#include "runtime/common.h"

namespace oap {

namespace {

struct Rot {
  int i;
  double c, s;
};

// Runs fn(chunk, b, e) over [0, n) on the pool when the work pays for the wake-up.
template <class F>
void par(ThreadPool* pool, int64_t n, int64_t work, F&& fn) {
  if (pool == nullptr || pool->size() == 1 || work < (1 << 16)) {
    fn(0, int64_t(0), n);
    return;
  }
  pool->parallel_for(n, [&](int ci, int64_t b, int64_t e) { fn(ci, b, e); });
}

struct Reflector {
  int o = 0;      // acts on indices [o, n)
  double tau = 0.0;
  std::vector<double> v;  // length n - o
};

// Householder reflector H = I - tau v v^T with H x = beta e_0.
Reflector make_reflector(const double* x, int m, int o, double& beta) {
  Reflector R;
  R.o = o;
  R.v.assign(x, x + m);
  double tail = 0.0;
  for (int i = 1; i < m; ++i) tail += x[i] * x[i];
  beta = x[0];
  if (tail > 0.0) {
    const double nx = std::sqrt(x[0] * x[0] + tail);
    beta = x[0] >= 0.0 ? -nx : nx;
    R.v[0] = x[0] - beta;
    R.tau = 2.0 / (R.v[0] * R.v[0] + tail);
  }
  return R;
}

// Householder tridiagonalisation A = Q T Q^T working on the LOWER triangle of `a` (row-major,
// destroyed).  Each step makes ONE pass over the trailing lower triangle that both applies the
// rank-2 update of this reflector and accumulates y = A' v' for the next one (the next reflector
// is formed first from the already-updated column), so the O(n^3) work streams the matrix once
// per step instead of three times.  Rows are split over the pool by triangle area; the
// transposed half of the symmetric product goes to per-thread accumulators reduced in thread
// order (deterministic for a fixed pool size).
void tridiagonalize(std::vector<double>& a, int n, std::vector<double>& diag,
                    std::vector<double>& off, std::vector<Reflector>& refl, ThreadPool* pool) {
  diag.assign(n, 0.0);
  off.assign(n, 0.0);
  refl.clear();
  const int nt = pool ? pool->size() : 1;
  std::vector<std::vector<double>> ypriv(nt, std::vector<double>(n, 0.0));
  std::vector<double> y(n, 0.0), w(n, 0.0), col(n);
  double* A = a.data();
  auto at = [&](int i, int j) -> double& { return A[size_t(i) * n + j]; };

  // symmetric product y[i - o] = sum_j A[i][j] v[j - o] over the lower triangle of rows
  // [o, n), optionally first applying A -= v w^T + w v^T with the PREVIOUS reflector (pv, pw
  // indexed from po).  Rows [o, n) are split into nt contiguous ranges of equal triangle area.
  auto fused_pass = [&](int o, const double* v, bool update, int po, const double* pv,
                        const double* pw) {
    const int m = n - o;
    std::vector<int> bounds(nt + 1, n);
    bounds[0] = o;
    {
      const double total = 0.5 * double(m) * double(m + 1);
      int t = 1;
      double accum = 0.0;
      for (int i = o; i < n && t < nt; ++i) {
        accum += double(i - o + 1);
        if (accum >= total * t / nt) bounds[t++] = i + 1;
      }
      for (; t < nt; ++t) bounds[t] = n;
    }
    auto body = [&](int ci, int64_t, int64_t) {
      double* __restrict yp = ypriv[ci].data();
      std::fill(yp + o, yp + n, 0.0);
      for (int i = bounds[ci]; i < bounds[ci + 1]; ++i) {
        double* __restrict row = A + size_t(i) * n;
        if (update) {
          const double vi = pv[i - po], wi = pw[i - po];
          const double* __restrict pvo = pv - po;
          const double* __restrict pwo = pw - po;
          for (int j = o; j <= i; ++j) row[j] -= vi * pwo[j] + wi * pvo[j];
        }
        if (v) {
          const double* __restrict vo = v - o;
          const double vi = vo[i];
          double s = 0.0;
#pragma omp simd reduction(+ : s)
          for (int j = o; j < i; ++j) {
            s += row[j] * vo[j];
            yp[j] += row[j] * vi;
          }
          yp[i] += s + row[i] * vi;
        }
      }
    };
    if (nt == 1 || int64_t(m) * m < (1 << 15)) {
      // serial: one chunk covering everything
      std::vector<int> b2 = {o, n};
      bounds.swap(b2);
      body(0, 0, 0);
      bounds.swap(b2);
      if (v)
        for (int i = o; i < n; ++i) y[i - o] = ypriv[0][i];
      return;
    }
    pool->parallel_for(nt, [&](int, int64_t b, int64_t e) {
      for (int64_t ci = b; ci < e; ++ci) body(int(ci), 0, 0);
    });
    if (v)
      for (int i = o; i < n; ++i) {
        double s = 0.0;
        for (int t = 0; t < nt; ++t) s += ypriv[t][i];
        y[i - o] = s;
      }
  };

  if (n == 1) {
    diag[0] = at(0, 0);
    return;
  }
  // first reflector from column 0
  for (int i = 1; i < n; ++i) col[i - 1] = at(i, 0);
  double beta = 0.0;
  if (n > 2) {
    refl.push_back(make_reflector(col.data(), n - 1, 1, beta));
    diag[0] = at(0, 0);
    off[0] = beta;
    fused_pass(1, refl.back().v.data(), false, 0, nullptr, nullptr);
  }
  for (int k = 0; k + 2 < n; ++k) {
    const int o = k + 1, m = n - o;
    const Reflector& R = refl[k];
    const double* v = R.v.data();
    const double tau = R.tau;
    // w = p - (tau/2)(v.p) v,  p = tau * y
    double vp = 0.0;
    for (int i = 0; i < m; ++i) vp += v[i] * (tau * y[i]);
    const double kk = 0.5 * tau * vp;
    for (int i = 0; i < m; ++i) w[i] = tau * y[i] - kk * v[i];
    // update column o (rows o..n-1) first, so the next reflector can be formed
    for (int i = o; i < n; ++i) at(i, o) -= v[i - o] * w[0] + w[i - o] * v[0];
    diag[o] = at(o, o);
    if (o + 2 < n) {
      for (int i = o + 1; i < n; ++i) col[i - o - 1] = at(i, o);
      refl.push_back(make_reflector(col.data(), n - o - 1, o + 1, beta));
      off[o] = beta;
      // remaining update of rows [o+1, n), columns [o+1, i], fused with y = A' v'
      fused_pass(o + 1, refl.back().v.data(), true, o, v, w.data());
    } else {
      // last step: plain update of the 1x1 trailing block
      fused_pass(o + 1, nullptr, true, o, v, w.data());
    }
  }
  diag[n - 2] = at(n - 2, n - 2);
  diag[n - 1] = at(n - 1, n - 1);
  off[n - 2] = at(n - 1, n - 2);
  off[n - 1] = 0.0;
}

// Eigenvalue-only / rotation-recording implicit-shift QL on the symmetric tridiagonal (d, e);
// e[i] couples i and i+1.  Eigenvalues overwrite d.
void tridiag_ql(std::vector<double>& d, std::vector<double>& e, int n, std::vector<Rot>* rots) {
  // absolute deflation floor eps*||T||: without it a cluster of (numerically) zero eigenvalues,
  // e.g. a rank-deficient covariance, never meets the relative test
  double tnorm = 0.0;
  for (int i = 0; i < n; ++i) tnorm = std::max(tnorm, std::fabs(d[i]) + std::fabs(e[i]));
  const double floor_tol = DBL_EPSILON * tnorm;
  for (int l = 0; l < n; ++l) {
    int iter = 0, m;
    while (true) {
      for (m = l; m < n - 1; ++m) {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= DBL_EPSILON * dd || std::fabs(e[m]) <= floor_tol) break;
      }
      if (m == l) break;
      OAP_CHECK(++iter <= 60, "symmetric eigensolver: QL did not converge");
      double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
      double r = std::hypot(g, 1.0);
      g = d[m] - d[l] + e[l] / (g + std::copysign(r, g));
      double s = 1.0, c = 1.0, p = 0.0;
      bool underflow = false;
      for (int i = m - 1; i >= l; --i) {
        const double f = s * e[i], b = c * e[i];
        r = std::hypot(f, g);
        e[i + 1] = r;
        if (r == 0.0) {  // deflation by underflow: restart on the split problem
          d[i + 1] -= p;
          e[m] = 0.0;
          underflow = true;
          break;
        }
        s = f / r;
        c = g / r;
        g = d[i + 1] - p;
        r = (d[i] - g) * s + 2.0 * c * b;
        p = s * r;
        d[i + 1] = g + p;
        g = c * r - b;
        if (rots) rots->push_back({i, c, s});
      }
      if (underflow) continue;
      d[l] -= p;
      e[l] = g;
      e[m] = 0.0;
    }
  }
}

// Q = H_0 H_1 ... (explicit, row-major) from the reflectors, accumulated backwards.
std::vector<double> form_q(const std::vector<Reflector>& refl, int n, ThreadPool* pool) {
  std::vector<double> q(size_t(n) * n, 0.0);
  for (int i = 0; i < n; ++i) q[size_t(i) * n + i] = 1.0;
  std::vector<double> u(n);
  for (int k = int(refl.size()) - 1; k >= 0; --k) {
    const Reflector& R = refl[k];
    if (R.tau == 0.0) continue;
    const int o = R.o, m = n - o;
    const double* __restrict v = R.v.data();
    par(pool, m, int64_t(m) * m, [&](int, int64_t b, int64_t e) {
      double* __restrict uu = u.data();
      for (int64_t j = b; j < e; ++j) uu[j] = 0.0;
      for (int i = 0; i < m; ++i) {
        const double vi = v[i];
        const double* __restrict row = &q[size_t(o + i) * n + o];
        for (int64_t j = b; j < e; ++j) uu[j] += vi * row[j];
      }
      for (int i = 0; i < m; ++i) {
        const double tv = R.tau * v[i];
        double* __restrict row = &q[size_t(o + i) * n + o];
        for (int64_t j = b; j < e; ++j) row[j] -= tv * uu[j];
      }
    });
  }
  return q;
}

// Tridiagonal (d, e) - lambda I: LU with partial pivoting (rows i, i+1 interchanged when the
// sub-diagonal dominates), then solves in place.  Pivots that vanish are replaced by `tiny`.
struct TriLU {
  std::vector<double> dd, du, du2, dl;
  std::vector<char> swp;
  void factor(const std::vector<double>& d, const std::vector<double>& e, int n, double lambda,
              double tiny) {
    dd.resize(n);
    du.assign(n, 0.0);
    du2.assign(n, 0.0);
    dl.assign(n, 0.0);
    swp.assign(n, 0);
    for (int i = 0; i < n; ++i) dd[i] = d[i] - lambda;
    for (int i = 0; i + 1 < n; ++i) {
      du[i] = e[i];
      dl[i] = e[i];
    }
    for (int i = 0; i + 1 < n; ++i) {
      if (std::fabs(dd[i]) >= std::fabs(dl[i])) {
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
      if (std::fabs(dd[i]) < tiny) dd[i] = std::copysign(tiny, dd[i] == 0.0 ? 1.0 : dd[i]);
  }
  void solve(std::vector<double>& b, int n) const {
    for (int i = 0; i + 1 < n; ++i) {
      if (swp[i]) std::swap(b[i], b[i + 1]);
      b[i + 1] -= dl[i] * b[i];
    }
    b[n - 1] /= dd[n - 1];
    if (n >= 2) b[n - 2] = (b[n - 2] - du[n - 2] * b[n - 1]) / dd[n - 2];
    for (int i = n - 3; i >= 0; --i)
      b[i] = (b[i] - du[i] * b[i + 1] - du2[i] * b[i + 2]) / dd[i];
  }
};

// Eigenvectors of the tridiagonal for the selected eigenvalues by inverse iteration, with
// modified Gram-Schmidt inside clusters of close eigenvalues (the LAPACK dstein recipe).
// sel: eigenvalues in the order wanted.  Returns z (n x kk, column j for sel[j]) row-major.
std::vector<double> tridiag_inverse_iteration(const std::vector<double>& d,
                                              const std::vector<double>& e, int n,
                                              const std::vector<double>& sel,
                                              ThreadPool* pool = nullptr) {
  const int kk = static_cast<int>(sel.size());
  double tnorm = 0.0;
  for (int i = 0; i < n; ++i)
    tnorm = std::max(tnorm, std::fabs(d[i]) + (i > 0 ? std::fabs(e[i - 1]) : 0.0) +
                                (i + 1 < n ? std::fabs(e[i]) : 0.0));
  if (tnorm == 0.0) tnorm = 1.0;
  const double ortol = 1e-3 * tnorm, pert = 10.0 * DBL_EPSILON * tnorm;
  const double tiny = DBL_EPSILON * tnorm;
  // clusters of close eigenvalues (exact multiples separated) first: the vectors of one cluster
  // are orthogonalised in order, different clusters are independent (thread pool)
  std::vector<double> lam(sel);
  std::vector<int> cstart(kk, 0);
  for (int j = 0; j < kk; ++j) {
    if (j > 0 && std::fabs(lam[j] - lam[j - 1]) < ortol) {
      if (std::fabs(lam[j] - lam[j - 1]) < pert)  // separate exact multiples
        lam[j] = lam[j - 1] + (lam[j] <= lam[j - 1] ? -pert : pert);
      cstart[j] = cstart[j - 1];
    } else {
      cstart[j] = j;
    }
  }
  std::vector<int> heads;
  for (int j = 0; j < kk; ++j)
    if (cstart[j] == j) heads.push_back(j);
  std::vector<std::vector<double>> zs(kk);
  auto run_cluster = [&](int h) {
    const int j0 = heads[h], j1 = h + 1 < int(heads.size()) ? heads[h + 1] : kk;
    TriLU lu;
    std::vector<double> b(n);
    for (int j = j0; j < j1; ++j) {
      lu.factor(d, e, n, lam[j], tiny);
      uint64_t st = 0x9e3779b97f4a7c15ull * uint64_t(j + 1);
      for (int i = 0; i < n; ++i) {  // deterministic start vector
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        b[i] = double(st >> 11) * (1.0 / 9007199254740992.0) - 0.5;
      }
      for (int it = 0; it < 4; ++it) {
        lu.solve(b, n);
        for (int q = j0; q < j; ++q) {  // MGS against the cluster's vectors
          const std::vector<double>& z = zs[q];
          double dot = 0.0;
          for (int i = 0; i < n; ++i) dot += z[i] * b[i];
          for (int i = 0; i < n; ++i) b[i] -= dot * z[i];
        }
        double nrm = 0.0;
        for (int i = 0; i < n; ++i) nrm += b[i] * b[i];
        nrm = std::sqrt(nrm);
        if (nrm == 0.0) {
          std::fill(b.begin(), b.end(), 0.0);
          b[j % n] = 1.0;
          continue;
        }
        for (int i = 0; i < n; ++i) b[i] /= nrm;
      }
      zs[j] = b;
    }
  };
  const int nh = static_cast<int>(heads.size());
  if (pool && pool->size() > 1 && nh > 1 && int64_t(n) * kk > 20000)
    pool->parallel_for(nh, [&](int, int64_t b, int64_t e2) {
      for (int64_t h = b; h < e2; ++h) run_cluster(int(h));
    });
  else
    for (int h = 0; h < nh; ++h) run_cluster(h);
  std::vector<double> z(size_t(n) * kk);
  for (int j = 0; j < kk; ++j)
    for (int i = 0; i < n; ++i) z[size_t(i) * kk + j] = zs[j][i];
  return z;
}

// V = Q Z for Z (n x kk row-major): reflectors applied last-to-first, columns split over the pool.
void apply_q(const std::vector<Reflector>& refl, int n, std::vector<double>& z, int kk,
             ThreadPool* pool) {
  for (int k = int(refl.size()) - 1; k >= 0; --k) {
    const Reflector& R = refl[k];
    if (R.tau == 0.0) continue;
    const int o = R.o, m = n - o;
    const double* __restrict v = R.v.data();
    par(pool, kk, int64_t(m) * kk, [&](int, int64_t b, int64_t e) {
      std::vector<double> u(e - b, 0.0);
      for (int i = 0; i < m; ++i) {
        const double* __restrict row = &z[size_t(o + i) * kk];
        for (int64_t c = b; c < e; ++c) u[c - b] += v[i] * row[c];
      }
      for (int i = 0; i < m; ++i) {
        double* __restrict row = &z[size_t(o + i) * kk];
        const double tv = R.tau * v[i];
        for (int64_t c = b; c < e; ++c) row[c] -= tv * u[c - b];
      }
    });
  }
}

// sign: largest-magnitude component positive
void normalize_signs(std::vector<double>& vecs, int n, int keep) {
  for (int j = 0; j < keep; ++j) {
    int big = 0;
    for (int i = 1; i < n; ++i)
      if (std::fabs(vecs[size_t(i) * keep + j]) > std::fabs(vecs[size_t(big) * keep + j])) big = i;
    if (vecs[size_t(big) * keep + j] < 0.0)
      for (int i = 0; i < n; ++i) vecs[size_t(i) * keep + j] = -vecs[size_t(i) * keep + j];
  }
}

// Eigenvalues (QL, |lambda| descending) and the first `keep` eigenvectors of the tridiagonal by
// inverse iteration, back-transformed by apply_q.
SymEig tridiag_topk(const std::vector<double>& td, const std::vector<double>& te, int n, int keep,
                    const std::function<void(std::vector<double>&, int)>& apply_q_fn,
                    const std::vector<double>* eigvals = nullptr, ThreadPool* pool = nullptr) {
  SymEig out;
  out.n = n;
  std::vector<double> diag = td, off = te;
  if (eigvals)
    diag = *eigvals;
  else
    tridiag_ql(diag, off, n, nullptr);
  std::vector<int> perm(n);
  std::iota(perm.begin(), perm.end(), 0);
  std::stable_sort(perm.begin(), perm.end(),
                   [&](int x, int y) { return std::fabs(diag[x]) > std::fabs(diag[y]); });
  out.values.resize(n);
  for (int j = 0; j < n; ++j) out.values[j] = diag[perm[j]];
  std::vector<double> sel(out.values.begin(), out.values.begin() + keep);
  std::vector<double> vecs = tridiag_inverse_iteration(td, te, n, sel, pool);
  apply_q_fn(vecs, keep);
  normalize_signs(vecs, n, keep);
  out.vectors = std::move(vecs);
  return out;
}

SymEig solve(const std::vector<double>& A, int n, int keep, ThreadPool* pool) {
  OAP_CHECK(n > 0 && A.size() == size_t(n) * n, "sym_eig: bad matrix size");
  keep = std::max(1, std::min(keep, n));
  SymEig out;
  out.n = n;
  std::vector<double> a = A, diag, off;
  std::vector<Reflector> refl;
  tridiagonalize(a, n, diag, off, refl, pool);
  a.clear();
  a.shrink_to_fit();
  const std::vector<double> td = diag, te = off;  // tridiagonal, kept for inverse iteration

  std::vector<double> vecs;  // n x keep, column j = eigenvector j (before sign normalisation)
  std::vector<double> vals(n);
  if (2 * keep <= n) {
    return tridiag_topk(
        td, te, n, keep,
        [&](std::vector<double>& z, int kk) { apply_q(refl, n, z, kk, pool); }, nullptr, pool);
  } else {
    // many vectors: QL with every rotation replayed on Q^T (rows i, i+1), column slices per
    // thread
    std::vector<Rot> rots;
    rots.reserve(size_t(n) * 4);
    tridiag_ql(diag, off, n, &rots);
    std::vector<double> q = form_q(refl, n, pool), vt(size_t(n) * n);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) vt[size_t(j) * n + i] = q[size_t(i) * n + j];
    q.clear();
    par(pool, n, int64_t(rots.size()) * n, [&](int, int64_t b, int64_t e) {
      for (const Rot& R : rots) {
        double* __restrict ri = &vt[size_t(R.i) * n];
        double* __restrict rj = ri + n;
        const double c = R.c, s = R.s;
        for (int64_t col = b; col < e; ++col) {
          const double f = rj[col], g = ri[col];
          rj[col] = s * g + c * f;
          ri[col] = c * g - s * f;
        }
      }
    });
    std::vector<int> perm(n);
    std::iota(perm.begin(), perm.end(), 0);
    std::stable_sort(perm.begin(), perm.end(),
                     [&](int x, int y) { return std::fabs(diag[x]) > std::fabs(diag[y]); });
    for (int j = 0; j < n; ++j) vals[j] = diag[perm[j]];
    vecs.assign(size_t(n) * keep, 0.0);
    for (int j = 0; j < keep; ++j)
      for (int i = 0; i < n; ++i) vecs[size_t(i) * keep + j] = vt[size_t(perm[j]) * n + i];
  }
  out.values = vals;
  normalize_signs(vecs, n, keep);
  out.vectors = std::move(vecs);
  return out;
}

}  // namespace

SymEig sym_eig_from_tridiag(const std::vector<double>& d, const std::vector<double>& e, int n,
                            int keep,
                            const std::function<void(std::vector<double>&, int)>& apply_q_fn,
                            const std::vector<double>* eigvals, ThreadPool* pool) {
  OAP_CHECK(n > 0 && int(d.size()) == n && int(e.size()) == n, "sym_eig_from_tridiag: sizes");
  OAP_CHECK(!eigvals || int(eigvals->size()) == n, "sym_eig_from_tridiag: eigenvalue count");
  keep = std::max(1, std::min(keep, n));
  return tridiag_topk(d, e, n, keep, apply_q_fn, eigvals, pool);
}

SymEig sym_eig(const std::vector<double>& A, int n, ThreadPool* pool) {
  return solve(A, n, n, pool);
}

SymEig sym_eig_topk(const std::vector<double>& A, int n, int k, ThreadPool* pool) {
  return solve(A, n, k, pool);
}

}  // namespace oap
