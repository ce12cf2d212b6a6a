#include "drivers/als.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <climits>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "kernels/als_setup.h"
#include "kernels/kernels.h"
#include "kernels/rng.h"
#include "linalg/eigen.h"
#include "runtime/log.h"
#include "runtime/knobs.h"

namespace oap {

namespace {

struct Rec {
  int32_t a, b;
  float r;
};
static_assert(sizeof(Rec) == 12, "Rec must be packed");

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int owner_of(int32_t id, int P) { return int(((int64_t(id) % P) + P) % P); }

// ---- host-memory collectives that work with any comm ------------------------------------
std::vector<int64_t> allgather_i64(Context& ctx, Comm& comm, const std::vector<int64_t>& mine) {
  const int P = comm.size();
  std::vector<int64_t> all(mine.size() * P);
  if (comm.trivial()) {
    std::copy(mine.begin(), mine.end(), all.begin());
    return all;
  }
  if (comm.on_device()) {
    Buffer s = ctx.alloc(mine.size() * 8), r = ctx.alloc(all.size() * 8);
    hipStream_t st = ctx.comm_stream();
    OAP_HIP_CHECK(
        hipMemcpyAsync(s.data(), mine.data(), mine.size() * 8, hipMemcpyHostToDevice, st));
    comm.allgather(s.data(), r.data(), mine.size(), DType::I64, st);
    OAP_HIP_CHECK(hipMemcpyAsync(all.data(), r.data(), all.size() * 8, hipMemcpyDeviceToHost, st));
    comm.wait(st);
  } else {
    comm.allgather(mine.data(), all.data(), mine.size(), DType::I64, nullptr);
  }
  return all;
}

// Ratings to their owners: out[p] goes to rank p; returns what this rank received, in source
// rank order.
std::vector<Rec> exchange(Context& ctx, Comm& comm, std::vector<std::vector<Rec>>& out) {
  const int P = comm.size(), me = comm.rank();
  if (comm.trivial()) return std::move(out[0]);
  std::vector<int64_t> mine(P);
  for (int p = 0; p < P; ++p) mine[p] = int64_t(out[p].size());
  const std::vector<int64_t> all = allgather_i64(ctx, comm, mine);
  std::vector<size_t> sc(P), rc(P);
  size_t stot = 0, rtot = 0;
  for (int p = 0; p < P; ++p) {
    sc[p] = out[p].size() * sizeof(Rec);
    rc[p] = size_t(all[size_t(p) * P + me]) * sizeof(Rec);
    stot += sc[p];
    rtot += rc[p];
  }
  std::vector<char> send(stot);
  size_t off = 0;
  for (int p = 0; p < P; ++p) {
    if (!out[p].empty()) std::memcpy(send.data() + off, out[p].data(), sc[p]);
    off += sc[p];
    std::vector<Rec>().swap(out[p]);
  }
  std::vector<Rec> recv(rtot / sizeof(Rec));
  if (comm.on_device()) {
    Buffer ds = ctx.alloc(std::max<size_t>(stot, 16)), dr = ctx.alloc(std::max<size_t>(rtot, 16));
    hipStream_t st = ctx.comm_stream();
    if (stot)
      OAP_HIP_CHECK(hipMemcpyAsync(ds.data(), send.data(), stot, hipMemcpyHostToDevice, st));
    comm.alltoallv(ds.data(), sc, dr.data(), rc, DType::U8, st);
    if (rtot)
      OAP_HIP_CHECK(hipMemcpyAsync(recv.data(), dr.data(), rtot, hipMemcpyDeviceToHost, st));
    comm.wait(st);
  } else {
    comm.alltoallv(send.data(), sc, recv.data(), rc, DType::U8, nullptr);
  }
  return recv;
}

// allgatherv of int32 ids (counts known on every rank), rank order.
std::vector<int32_t> allgatherv_i32(Context& ctx, Comm& comm, const std::vector<int32_t>& mine,
                                    const std::vector<int64_t>& counts) {
  const int P = comm.size();
  if (comm.trivial()) return mine;
  int64_t mx = 1;
  for (int64_t c : counts) mx = std::max(mx, c);
  std::vector<int64_t> pad(mx, 0);
  for (size_t i = 0; i < mine.size(); ++i) pad[i] = mine[i];
  const std::vector<int64_t> all = allgather_i64(ctx, comm, pad);
  std::vector<int32_t> out;
  for (int p = 0; p < P; ++p)
    for (int64_t i = 0; i < counts[p]; ++i) out.push_back(int32_t(all[size_t(p) * mx + i]));
  return out;
}

struct Csr {
  std::vector<int64_t> ptr;
  std::vector<int32_t> col;
  std::vector<float> val;
};

// CSR by counting sort (rows are a - row_base, dense in [0, nrows)): atomic row histogram,
// prefix sum, atomic scatter, then every row sorted by (col, value) — so the result does not
// depend on the scatter order or the thread count.  O(nnz) + per-row sorts, all on the pool.
Csr build_csr(ThreadPool& pool, std::vector<Rec>& recs, int64_t nrows, int64_t row_base) {
  const int64_t nnz = int64_t(recs.size());
  Csr c;
  std::vector<std::atomic<int64_t>> cnt(nrows + 1);
  pool.parallel_for(nrows + 1, [&](int, int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) cnt[i].store(0, std::memory_order_relaxed);
  });
  std::atomic<bool> bad{false};
  pool.parallel_for(nnz, [&](int, int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      const int64_t row = int64_t(recs[k].a) - row_base;
      if (row < 0 || row >= nrows) {
        bad = true;
        continue;
      }
      cnt[row + 1].fetch_add(1, std::memory_order_relaxed);
    }
  });
  OAP_CHECK(!bad, "ALS CSR: row out of range");
  c.ptr.assign(nrows + 1, 0);
  for (int64_t i = 0; i < nrows; ++i) c.ptr[i + 1] = c.ptr[i] + cnt[i + 1].load();
  pool.parallel_for(nrows, [&](int, int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) cnt[i].store(c.ptr[i], std::memory_order_relaxed);
  });
  c.col.resize(nnz);
  c.val.resize(nnz);
  pool.parallel_for(nnz, [&](int, int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      const int64_t pos =
          cnt[int64_t(recs[k].a) - row_base].fetch_add(1, std::memory_order_relaxed);
      c.col[pos] = recs[k].b;
      c.val[pos] = recs[k].r;
    }
  });
  pool.parallel_for(nrows, [&](int, int64_t b, int64_t e) {
    std::vector<std::pair<int32_t, float>> tmp;
    for (int64_t i = b; i < e; ++i) {
      const int64_t p0 = c.ptr[i], p1 = c.ptr[i + 1];
      if (p1 - p0 < 2) continue;
      tmp.resize(p1 - p0);
      for (int64_t q = p0; q < p1; ++q) tmp[q - p0] = {c.col[q], c.val[q]};
      std::sort(tmp.begin(), tmp.end());
      for (int64_t q = p0; q < p1; ++q) {
        c.col[q] = tmp[q - p0].first;
        c.val[q] = tmp[q - p0].second;
      }
    }
  });
  return c;
}

// Sorted distinct ids with O(1) id -> rank lookup: a bitmap over [min, max] with per-word
// popcount prefixes when the id range is moderate (the common case), else sort + binary search.
struct IdIndex {
  std::vector<int32_t> ids;  // sorted distinct
  int64_t lo = 0;
  std::vector<uint64_t> bits;
  std::vector<int64_t> prefix;  // rank of the first id in each word
  bool bitmap = false;

  void build(ThreadPool& pool, const std::vector<Rec>& recs, bool use_a) {
    const int64_t n = int64_t(recs.size());
    ids.clear();
    if (n == 0) return;
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (int64_t k = 0; k < n; ++k) {
      const int64_t v = use_a ? recs[k].a : recs[k].b;
      mn = std::min(mn, v);
      mx = std::max(mx, v);
    }
    lo = mn;
    const int64_t range = mx - mn + 1;
    if (range <= (int64_t(1) << 31) && range <= 64 * n + (1 << 20)) {
      bitmap = true;
      const int64_t nw = (range + 63) / 64;
      std::vector<std::atomic<uint64_t>> w(nw);
      pool.parallel_for(nw, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) w[i].store(0, std::memory_order_relaxed);
      });
      pool.parallel_for(n, [&](int, int64_t b, int64_t e) {
        for (int64_t k = b; k < e; ++k) {
          const int64_t v = (use_a ? recs[k].a : recs[k].b) - lo;
          w[v >> 6].fetch_or(uint64_t(1) << (v & 63), std::memory_order_relaxed);
        }
      });
      bits.resize(nw);
      prefix.resize(nw + 1);
      prefix[0] = 0;
      for (int64_t i = 0; i < nw; ++i) {
        bits[i] = w[i].load();
        prefix[i + 1] = prefix[i] + __builtin_popcountll(bits[i]);
      }
      ids.resize(prefix[nw]);
      pool.parallel_for(nw, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
          uint64_t x = bits[i];
          int64_t o = prefix[i];
          while (x) {
            const int t = __builtin_ctzll(x);
            ids[o++] = int32_t(lo + i * 64 + t);
            x &= x - 1;
          }
        }
      });
    } else {
      ids.resize(n);
      for (int64_t k = 0; k < n; ++k) ids[k] = use_a ? recs[k].a : recs[k].b;
      std::sort(ids.begin(), ids.end());
      ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    }
  }
  int64_t rank(int32_t id) const {
    if (bitmap) {
      const int64_t v = int64_t(id) - lo;
      const uint64_t word = bits[v >> 6];
      const uint64_t below = (v & 63) ? (word & ((uint64_t(1) << (v & 63)) - 1)) : 0;
      return prefix[v >> 6] + __builtin_popcountll(below);
    }
    return std::lower_bound(ids.begin(), ids.end(), id) - ids.begin();
  }
};

struct Side {  // one factor matrix and the CSR of this rank's owned rows of it
  int64_t n = 0;                 // global rows
  std::vector<int64_t> cnt, off;  // per-rank owned counts / global offsets
  std::vector<int32_t> ids;      // global index -> id
  Csr csr;                       // owned rows; cols index the OTHER side
};

void init_factor_row(uint64_t seed, int32_t id, int r, int ld, float* out) {
  double nrm = 0.0;
  for (int f = 0; f < r; ++f) {
    const double g = kern::als_init_gaussian(seed, id, f);
    nrm += g * g;
  }
  nrm = std::sqrt(nrm);
  for (int f = 0; f < ld; ++f)
    out[f] = f < r ? float(kern::als_init_gaussian(seed, id, f) / nrm) : 0.f;
}

// fp64 Cholesky solve of the r x r SPD system (lower triangle of A used); false if not SPD.
bool chol_solve(std::vector<double>& A, std::vector<double>& b, int r) {
  for (int j = 0; j < r; ++j) {
    double d = A[size_t(j) * r + j];
    for (int k = 0; k < j; ++k) d -= A[size_t(j) * r + k] * A[size_t(j) * r + k];
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    A[size_t(j) * r + j] = d;
    for (int i = j + 1; i < r; ++i) {
      double s = A[size_t(i) * r + j];
      for (int k = 0; k < j; ++k) s -= A[size_t(i) * r + k] * A[size_t(j) * r + k];
      A[size_t(i) * r + j] = s / d;
    }
  }
  for (int j = 0; j < r; ++j) {
    double s = b[j];
    for (int k = 0; k < j; ++k) s -= A[size_t(j) * r + k] * b[k];
    b[j] = s / A[size_t(j) * r + j];
  }
  for (int j = r - 1; j >= 0; --j) {
    double s = b[j];
    for (int k = j + 1; k < r; ++k) s -= A[size_t(k) * r + j] * b[k];
    b[j] = s / A[size_t(j) * r + j];
  }
  return true;
}

// Non-negative least squares on the normal equations: min 1/2 x^T A x - b^T x subject to x >= 0
// (A = lower triangle of an SPD r x r matrix, row-major), by the Lawson-Hanson active set: the
// strictly convex problem has one minimiser, the one Spark's projected-CG NNLS
// (mllib/optimization/NNLS.scala, ALS.scala:1718-1800 with nonnegative = true) converges to.
// Each passive-set solve is a Cholesky of the passive block.  x gets the solution.  Returns
// kNnlsOk, kNnlsCapped (the iteration cap: x holds the last feasible, nearly optimal iterate —
// usable, but reported) or kNnlsNotSpd (a passive block is not SPD: x is not usable).
enum NnlsStatus : int { kNnlsOk = 0, kNnlsCapped = 1, kNnlsNotSpd = 2 };
NnlsStatus nnls_solve(const std::vector<double>& A, const std::vector<double>& b, int r,
                      std::vector<double>& x) {
  auto a = [&](int i, int j) { return i >= j ? A[size_t(i) * r + j] : A[size_t(j) * r + i]; };
  x.assign(r, 0.0);
  std::vector<char> passive(r, 0);
  std::vector<int> idx;
  std::vector<double> sub, z(r), rhs;
  double amax = 0.0;
  for (int i = 0; i < r; ++i) amax = std::max(amax, std::fabs(a(i, i)));
  const double tol = 1e-12 * std::max(amax, 1e-300) * (1.0 + std::fabs(*std::max_element(
      b.begin(), b.end(), [](double u, double v) { return std::fabs(u) < std::fabs(v); })));
  auto solve_passive = [&]() -> bool {  // z_P = A_PP^-1 b_P, z elsewhere 0
    idx.clear();
    for (int i = 0; i < r; ++i)
      if (passive[i]) idx.push_back(i);
    const int m = int(idx.size());
    sub.assign(size_t(m) * m, 0.0);
    rhs.assign(m, 0.0);
    for (int i = 0; i < m; ++i) {
      rhs[i] = b[idx[i]];
      for (int j = 0; j <= i; ++j) sub[size_t(i) * m + j] = a(idx[i], idx[j]);
    }
    if (!chol_solve(sub, rhs, m)) return false;
    std::fill(z.begin(), z.end(), 0.0);
    for (int i = 0; i < m; ++i) z[idx[i]] = rhs[i];
    return true;
  };
  // (Lawson-Hanson safeguard: a coordinate whose entry was undone at once — its passive solve
  // gave z_j <= 0 from x_j = 0, so it left again in the first inner step — is not offered again
  // until the passive set changes otherwise; without that the same j would re-enter forever)
  std::vector<char> blocked(r, 0);
  for (int outer = 0; outer < 8 * r + 32; ++outer) {
    // gradient of the objective's negative: w = b - A x; the best free coordinate enters
    int jbest = -1;
    double wbest = tol;
    for (int j = 0; j < r; ++j) {
      if (passive[j] || blocked[j]) continue;
      double w = b[j];
      for (int i = 0; i < r; ++i) w -= a(j, i) * x[i];
      if (w > wbest) {
        wbest = w;
        jbest = j;
      }
    }
    if (jbest < 0) return kNnlsOk;
    passive[jbest] = 1;
    for (int inner = 0; inner < 3 * r + 10; ++inner) {
      if (!solve_passive()) return kNnlsNotSpd;
      double alpha = 1.0;
      bool feasible = true;
      for (int i = 0; i < r; ++i)
        if (passive[i] && z[i] <= 0.0) {
          feasible = false;
          const double den = x[i] - z[i];
          if (den > 0.0) alpha = std::min(alpha, x[i] / den);
        }
      if (feasible) {
        x = z;
        break;
      }
      for (int i = 0; i < r; ++i) {
        x[i] += alpha * (z[i] - x[i]);
        if (passive[i] && x[i] <= 0.0) {
          passive[i] = 0;
          x[i] = 0.0;
        }
      }
    }
    if (!passive[jbest]) {
      blocked[jbest] = 1;  // its entry was undone: skip it until the passive set moves
    } else {
      std::fill(blocked.begin(), blocked.end(), 0);
    }
  }
  return kNnlsCapped;  // (the caller keeps x and counts the row as failed)
}

// Rows of X (global user order, stride ld) whose id appears in the caller's initial factors
// (ids sorted ascending, rank columns) are overwritten with them — the resume path.
void overlay_init(const std::vector<int32_t>& ids, int r, int ld, const AlsParams& p,
                  float* X) {
  if (p.init_ids == nullptr || p.n_init == 0) return;
  for (size_t g = 0; g < ids.size(); ++g) {
    const int32_t* it = std::lower_bound(p.init_ids, p.init_ids + p.n_init, ids[g]);
    if (it == p.init_ids + p.n_init || *it != ids[g]) continue;
    const float* src = p.init_factors + size_t(it - p.init_ids) * r;
    for (int f = 0; f < r; ++f) X[g * size_t(ld) + f] = src[f];
  }
}

}  // namespace

AlsResult als_fit(Context& ctx, Comm& comm, const int32_t* users, const int32_t* items,
                  const float* ratings, int64_t n, const AlsParams& p) {
  TraceRange tr_all(&ctx.metrics(), "als/fit");
  OAP_CHECK(p.rank >= 1, "ALS rank must be >= 1");
  OAP_CHECK(p.max_iter >= 0, "ALS maxIter must be >= 0");
  const int P = comm.size(), me = comm.rank();
  // a trivial comm (world of one, no communicator) skips every exchange; any other comm — a
  // 1-rank RCCL communicator included — runs the multi-rank code path end to end
  const bool local = comm.trivial();
  // factor row pitch = the solves' padded width (multiple of 16 >= rank); OAP_ALS_LD overrides
  // it upward (timing experiments: whole 128-byte lines per gathered row)
  const int r = p.rank;
  int ld = int(round_up(size_t(r), 16));
  {
    const int v = int(knob_int("OAP_ALS_LD"));
    if (v >= ld && v % 16 == 0 && v <= 128) ld = v;
  }
  AlsResult res;
  res.rank = r;
  auto t_setup = std::chrono::steady_clock::now();

  Side U, I;
  // ---- on a GPU: re-indexing, the ratings shuffle and both CSRs on the device
  // (kernels/als_setup.hip); OAP_ALS_HOST_SETUP=1 forces the host setup below
  kern::AlsDeviceSetup dev_setup;
  kern::AlsDistSetup dist_setup;
  bool on_device = false;
  kern::AlsDeviceCsr *dev_ucsr = nullptr, *dev_icsr = nullptr;
  // (host_engine: the fp64 host solver on a GPU world, e.g. ranks beyond the GPU kernels; the
  // GPU context only stages the collectives)
  const bool gpu_engine = ctx.is_gpu() && !p.host_engine && !p.nonnegative;
  if (gpu_engine && !knob_on("OAP_ALS_HOST_SETUP")) {
    ctx.activate();
    if (local)
      on_device = kern::als_device_setup(ctx, users, items, ratings, n, ctx.compute(), &dev_setup);
    else
      on_device = kern::als_device_setup_dist(ctx, comm, users, items, ratings, n, ctx.compute(),
                                              &dist_setup);
  }
  if (on_device) {
    auto fill = [](Side& S, std::vector<int32_t>& ids, kern::AlsDeviceCsr& c,
                   std::vector<int64_t> cnt, std::vector<int64_t> off) {
      S.n = off.back();
      S.cnt = std::move(cnt);
      S.off = std::move(off);
      S.ids = std::move(ids);
      S.csr.ptr = c.ptr_h;  // (cols / values stay on the device)
    };
    if (local) {
      const int64_t nu = dev_setup.users.nrows, ni = dev_setup.items.nrows;
      fill(U, dev_setup.user_ids, dev_setup.users, {nu}, {0, nu});
      fill(I, dev_setup.item_ids, dev_setup.items, {ni}, {0, ni});
      dev_ucsr = &dev_setup.users;
      dev_icsr = &dev_setup.items;
      res.nnz = n;
    } else {
      fill(U, dist_setup.user_ids, dist_setup.users, dist_setup.ucnt, dist_setup.uoff);
      fill(I, dist_setup.item_ids, dist_setup.items, dist_setup.icnt, dist_setup.ioff);
      dev_ucsr = &dist_setup.users;
      dev_icsr = &dist_setup.items;
      res.nnz = dist_setup.nnz;
    }
    res.setup_ms = ms_since(t_setup);
    ctx.metrics().add("als/setup", res.setup_ms * 1e3, n * int64_t(sizeof(Rec)) * 3);
    if (Logger::instance().level() <= LogLevel::Info) {
      const std::string det =
          local ? "\"upload_ms\":" + std::to_string(dev_setup.upload_ms) +
                      ",\"index_ms\":" + std::to_string(dev_setup.index_ms) +
                      ",\"sort_ms\":" + std::to_string(dev_setup.sort_ms)
                : "\"upload_ms\":" + std::to_string(dist_setup.upload_ms) +
                      ",\"shuffle_ms\":" + std::to_string(dist_setup.shuffle_ms) +
                      ",\"index_ms\":" + std::to_string(dist_setup.index_ms);
      Logger::instance().log(LogLevel::Info, "als/device_setup", det);
    }
  } else {
    // ---- 1. ratings -> item owners; dense item indices --------------------------------------
    std::vector<Rec> recv1;
    if (local) {
      recv1.resize(n);
      ctx.pool().parallel_for(n, [&](int, int64_t b, int64_t e) {
        for (int64_t k = b; k < e; ++k) recv1[k] = {users[k], items[k], ratings[k]};
      });
    } else {
      std::vector<std::vector<Rec>> out(P);
      for (int64_t k = 0; k < n; ++k)
        out[owner_of(items[k], P)].push_back({users[k], items[k], ratings[k]});
      recv1 = exchange(ctx, comm, out);
    }
    IdIndex item_idx;
    item_idx.build(ctx.pool(), recv1, false);
    const std::vector<int32_t>& my_items = item_idx.ids;
    I.cnt = allgather_i64(ctx, comm, {int64_t(my_items.size())});
    I.off.assign(P + 1, 0);
    for (int q = 0; q < P; ++q) I.off[q + 1] = I.off[q] + I.cnt[q];
    I.n = I.off[P];
    // ---- 2. -> user owners; dense user indices, user CSR (cols = global item index) ---------
    std::vector<Rec> recv2;
    if (local) {
      ctx.pool().parallel_for(int64_t(recv1.size()), [&](int, int64_t b, int64_t e) {
        for (int64_t k = b; k < e; ++k) recv1[k].b = int32_t(item_idx.rank(recv1[k].b));
      });
      recv2.swap(recv1);
    } else {
      std::vector<std::vector<Rec>> out(P);
      for (const Rec& x : recv1)
        out[owner_of(x.a, P)].push_back({x.a, int32_t(I.off[me] + item_idx.rank(x.b)), x.r});
      std::vector<Rec>().swap(recv1);
      recv2 = exchange(ctx, comm, out);
    }
    IdIndex user_idx;
    user_idx.build(ctx.pool(), recv2, true);
    const std::vector<int32_t>& my_users = user_idx.ids;
    U.cnt = allgather_i64(ctx, comm, {int64_t(my_users.size())});
    U.off.assign(P + 1, 0);
    for (int q = 0; q < P; ++q) U.off[q + 1] = U.off[q] + U.cnt[q];
    U.n = U.off[P];
    ctx.pool().parallel_for(int64_t(recv2.size()), [&](int, int64_t b, int64_t e) {
      for (int64_t k = b; k < e; ++k) recv2[k].a = int32_t(U.off[me] + user_idx.rank(recv2[k].a));
    });
    // ---- 3. (global user, global item) -> item owners: item CSR (cols = global user index) --
    std::vector<Rec> recv3;
    if (local) {
      recv3.resize(recv2.size());
      ctx.pool().parallel_for(int64_t(recv2.size()), [&](int, int64_t b, int64_t e) {
        for (int64_t k = b; k < e; ++k) recv3[k] = {recv2[k].b, recv2[k].a, recv2[k].r};
      });
    } else {
      std::vector<std::vector<Rec>> out(P);
      for (const Rec& x : recv2) {
        const int q =
            int(std::upper_bound(I.off.begin(), I.off.end(), int64_t(x.b)) - I.off.begin()) - 1;
        out[q].push_back({x.b, x.a, x.r});
      }
      recv3 = exchange(ctx, comm, out);
    }
    U.csr = build_csr(ctx.pool(), recv2, U.cnt[me], U.off[me]);
    I.csr = build_csr(ctx.pool(), recv3, I.cnt[me], I.off[me]);
    std::vector<Rec>().swap(recv2);
    std::vector<Rec>().swap(recv3);
    U.ids = allgatherv_i32(ctx, comm, my_users, U.cnt);
    I.ids = allgatherv_i32(ctx, comm, my_items, I.cnt);
    {
      int64_t nn = int64_t(U.csr.col.size());
      res.nnz = int64_t(comm_allreduce_scalar(ctx, comm, double(nn), ReduceOp::Sum));
    }
    res.setup_ms = ms_since(t_setup);
    ctx.metrics().add("als/setup", res.setup_ms * 1e3, res.nnz * int64_t(sizeof(Rec)) * 3);
  }  // host setup

  std::vector<float> Xh, Yh;  // final factors (host, [n][ld])
  auto t_train = std::chrono::steady_clock::now();
  if (gpu_engine) {
    OAP_CHECK(r <= kern::als_max_rank(), "GPU ALS supports rank <= " << kern::als_max_rank()
                                                                      << " (use the CPU engine)");
    ctx.activate();
    hipStream_t s = ctx.compute();
    const int cus = ctx.info().cu_count;
    // Multi-rank: each half solves its owned rows in C row-range chunks; chunk c of every rank
    // is broadcast (root = owner, straight into the replicated factor slab) on the comm stream
    // while chunk c+1 solves on the compute stream.
    const int C = local ? 1 : 4;
    // implicit rows with <= 64 ratings: low-rank (Woodbury) solve in the eigenbasis of Y^T Y
    // (kernels/als_lowrank.hip); OAP_ALS_LOWRANK=0 sends every row to the direct r x r solve
    const bool lowrank = knob_int("OAP_ALS_LOWRANK") != 0;
    // long-row chunks: split-fp16 Gramian (kernels/als.hip); OAP_ALS_GRAM=fp32 keeps the
    // exact-fp32 MFMA products
    const bool x3_gram = knob_str("OAP_ALS_GRAM") != "fp32";
    struct Dev {
      Buffer f, ptr, col, val;
      Buffer short_rows, long_rows, long_chunk_ptr, chunk_begin, chunk_end, partials;
      // low-rank path: per chunk, lr offsets into the chunk's short rows (AlsSolveArgs::lr_off);
      // rot: this side's factors in the eigenbasis of their Gramian (when it is a source)
      std::vector<std::array<int64_t, 5>> lro;
      Buffer rot, lr_scratch;
      // split-fp16 long-row Gramian scale inputs: [max |rating| (fixed), max |source factor|]
      Buffer absmax;
      // per row-range chunk c: [sr_off[c], sr_off[c+1]) of short_rows, [lr_off[c], ...) of
      // long_rows (long_chunk_ptr segment at lr_off[c] + c), [cb_off[c], ...) of chunk_begin/end
      std::vector<int64_t> sr_off, lr_off, cb_off;
      // per chunk: leading short rows longer than x3_min (split-fp16 direct Gramian)
      std::vector<int64_t> x3n;
    } dU, dI;
    // direct rows at most this long keep the fp32 Gramian (OAP_ALS_X3_MIN_LEN)
    const int64_t x3_min = knob_int("OAP_ALS_X3_MIN_LEN");
    // rows longer than kLong ratings are split into kLong-sized chunks (partial Gramians)
    constexpr int64_t kLong = 4096;
    auto upload_side = [&](Side& S, Dev& D, kern::AlsDeviceCsr* dc) {
      D.f = ctx.alloc(std::max<size_t>(size_t(S.n) * ld * 4, 256));
      if (dc) {  // built on the device
        D.ptr = std::move(dc->ptr);
        D.col = std::move(dc->col);
        D.val = std::move(dc->val);
      } else {
        D.ptr = ctx.alloc(S.csr.ptr.size() * 8);
        D.col = ctx.alloc(std::max<size_t>(S.csr.col.size() * 4, 16));
        D.val = ctx.alloc(std::max<size_t>(S.csr.val.size() * 4, 16));
        ctx.copy_to_backend(D.ptr.data(), S.csr.ptr.data(), S.csr.ptr.size() * 8, s);
        if (!S.csr.col.empty()) {
          ctx.copy_to_backend(D.col.data(), S.csr.col.data(), S.csr.col.size() * 4, s);
          ctx.copy_to_backend(D.val.data(), S.csr.val.data(), S.csr.val.size() * 4, s);
        }
      }
      ctx.memset(D.f.data(), 0, size_t(S.n) * ld * 4);
      std::vector<int32_t> sr, lr;
      std::vector<int64_t> lcp, cb, ce;
      const int64_t nloc = int64_t(S.csr.ptr.size()) - 1;
      D.sr_off.assign(1, 0);
      D.lr_off.assign(1, 0);
      D.cb_off.assign(1, 0);
      for (int c = 0; c < C; ++c) {
        const int64_t lo = nloc * c / C, hi = nloc * (c + 1) / C;
        // longest rows first: they start early and the short ones fill in behind them (a
        // counting sort by length: O(rows), rows longer than kLong by a comparison sort)
        std::vector<std::pair<int64_t, int32_t>> order;
        order.reserve(hi - lo);
        {
          std::vector<int64_t> bucket(kLong + 2, 0);
          std::vector<std::pair<int64_t, int32_t>> longs;
          for (int64_t i = lo; i < hi; ++i) {
            const int64_t len = S.csr.ptr[i + 1] - S.csr.ptr[i];
            if (len > kLong) longs.push_back({len, int32_t(i)});
            else ++bucket[kLong - len + 1];
          }
          std::stable_sort(longs.begin(), longs.end(),
                           [](const auto& x, const auto& y) { return x.first > y.first; });
          order = longs;
          for (int64_t b = 1; b <= kLong + 1; ++b) bucket[b] += bucket[b - 1];
          const size_t base = order.size();
          order.resize(base + size_t(bucket[kLong + 1]));
          for (int64_t i = lo; i < hi; ++i) {  // stable within a length (ascending row)
            const int64_t len = S.csr.ptr[i + 1] - S.csr.ptr[i];
            if (len <= kLong) order[base + size_t(bucket[kLong - len]++)] = {len, int32_t(i)};
          }
        }
        const int64_t cb0 = int64_t(cb.size());
        lcp.push_back(0);
        // low-rank classes: the short rows come by decreasing length, so each class
        // (<= 64, 48, 32, 16 ratings) is a contiguous tail of the chunk's short rows
        std::array<int64_t, 5> lo5{};
        {
          int64_t nsh = 0;
          std::array<int64_t, 4> above{};  // short rows longer than 64, 48, 32, 16
          for (const auto& [len, i] : order) {
            if (len > kLong) continue;
            ++nsh;
            for (int j = 0; j < 4; ++j) above[j] += len > 16 * (4 - j) ? 1 : 0;
          }
          const bool use = lowrank && p.implicit;
          for (int j = 0; j < 4; ++j) lo5[j] = use ? above[j] : nsh;
          lo5[4] = nsh;
        }
        D.lro.push_back(lo5);
        {
          int64_t nx = 0;
          for (const auto& [len, i] : order) nx += (len <= kLong && len > x3_min) ? 1 : 0;
          D.x3n.push_back(nx);
        }
        for (const auto& [len, i] : order) {
          if (len > kLong) {
            lr.push_back(i);
            for (int64_t p0 = S.csr.ptr[i]; p0 < S.csr.ptr[i + 1]; p0 += kLong) {
              cb.push_back(p0);
              ce.push_back(std::min(p0 + kLong, S.csr.ptr[i + 1]));
            }
            lcp.push_back(int64_t(cb.size()) - cb0);
          } else {
            sr.push_back(i);
          }
        }
        D.sr_off.push_back(int64_t(sr.size()));
        D.lr_off.push_back(int64_t(lr.size()));
        D.cb_off.push_back(int64_t(cb.size()));
      }
      auto up = [&](Buffer& b, const void* h, size_t bytes) {
        b = ctx.alloc(std::max<size_t>(bytes, 16));
        if (bytes) ctx.copy_to_backend(b.data(), h, bytes, s);
      };
      up(D.short_rows, sr.data(), sr.size() * 4);
      up(D.long_rows, lr.data(), lr.size() * 4);
      up(D.long_chunk_ptr, lcp.data(), lcp.size() * 8);
      up(D.chunk_begin, cb.data(), cb.size() * 8);
      up(D.chunk_end, ce.data(), ce.size() * 8);
      int64_t max_chunks = 1;
      for (int c = 0; c < C; ++c)
        max_chunks = std::max(max_chunks, D.cb_off[c + 1] - D.cb_off[c]);
      D.partials =
          ctx.alloc(std::max<size_t>(size_t(max_chunks) * kern::als_partial_floats(r) * 4, 16));
      int64_t max_lr = 0;
      for (const auto& o : D.lro) max_lr = std::max(max_lr, o[4] - o[0]);
      if (max_lr > 0) D.lr_scratch = ctx.alloc(size_t(max_lr) * ld * 4);
      if ((!lr.empty() || !sr.empty()) && x3_gram) {
        D.absmax = ctx.alloc(16);
        ctx.memset(D.absmax.data(), 0, 16);
        kern::als_absmax(D.val.as<float>(), S.csr.ptr.empty() ? 0 : S.csr.ptr.back(),
                         D.absmax.as<unsigned>(), s);
      }
      OAP_HIP_CHECK(hipStreamSynchronize(s));
    };
    upload_side(U, dU, dev_ucsr);
    upload_side(I, dI, dev_icsr);
    {  // initial user factors from their ids (world-size independent), or the caller's
      Buffer ids = ctx.alloc(std::max<size_t>(U.ids.size() * 4, 16));
      if (!U.ids.empty()) ctx.copy_to_backend(ids.data(), U.ids.data(), U.ids.size() * 4, s);
      kern::als_init_factors(ids.as<int32_t>(), U.n, r, ld, p.seed, dU.f.as<float>(), s);
      OAP_HIP_CHECK(hipStreamSynchronize(s));
      if (p.init_ids && p.n_init && U.n) {
        std::vector<float> X0(size_t(U.n) * ld);
        ctx.copy_to_host(X0.data(), dU.f.data(), X0.size() * 4);
        overlay_init(U.ids, r, ld, p, X0.data());
        ctx.copy_to_backend(dU.f.data(), X0.data(), X0.size() * 4, s);
        OAP_HIP_CHECK(hipStreamSynchronize(s));
      }
    }
    // [0, 8): solve work queues (als.hip / als_lowrank.hip slots), [2] failed rows;
    // [12]: Gramian eigensolves that missed the tolerance
    Buffer ctr = ctx.alloc(128);
    ctx.memset(ctr.data(), 0, 128);
    // low-rank path state: eigenbasis of the source Gramian, computed on the device
    // (kernels/als_eig.hip) straight from the allreduced fp64 Gramian — no host round trip
    Buffer lrQ = ctx.alloc(size_t(ld) * ld * 4), lrQT = ctx.alloc(size_t(ld) * ld * 4),
           lrEig = ctx.alloc(size_t(ld) * 4);
    Buffer eig_scratch = ctx.alloc(kern::als_gram_eig_scratch_bytes(r));
    Buffer gram64 = ctx.alloc((size_t(r) * r + r) * 8), gram32 = ctx.alloc(size_t(r) * r * 4);
    Buffer zshift = ctx.alloc(size_t(ld + 128) * 4);
    ctx.memset(zshift.data(), 0, size_t(ld + 128) * 4);
    hipStream_t cs = ctx.comm_stream() ? ctx.comm_stream() : s;
    const bool dev_comm = !local && comm.on_device();
    struct HalfEvents {
      Event e0, e1, e2, e3;
      std::vector<Event> solved;  // per chunk (compute stream -> comm stream)
      std::vector<Event> bc0, bc1;  // per chunk: its broadcasts on the comm stream
      Event gram_in, gram_out, gathered;
    };
    std::vector<HalfEvents> hev(2);
    // one half-iteration: dst rows of side D from source side S
    auto half = [&](HalfEvents& E, Side& Dst, Dev& dD, Side& Src, Dev& dS) {
      E.e0.record(s);
      // Gramian of the source factors: owned slice -> allreduce (on the comm stream, after the
      // previous half's broadcasts: every collective of this communicator is issued in one order)
      if (p.implicit) {
        const int64_t cnt = Src.cnt[me];
        const kern::PcaPlan plan = kern::pca_syrk_plan(cnt, r, cus);
        Buffer part = ctx.alloc(plan.part_elems * 8), cpart = ctx.alloc(plan.cpart_elems * 8);
        kern::pca_syrk(dS.f.as<float>() + Src.off[me] * ld, cnt, ld, r, zshift.as<float>(), plan,
                       part.as<double>(), cpart.as<double>(), false, 4096, s);
        kern::pca_reduce(plan, part.as<double>(), cpart.as<double>(), r, gram64.as<double>(),
                         gram64.as<double>() + size_t(r) * r, s);
        if (dev_comm) {
          E.gram_in.record(s);
          E.gram_in.wait_on(cs);
          comm.allreduce(gram64.data(), size_t(r) * r, DType::F64, ReduceOp::Sum, cs);
          E.gram_out.record(cs);
          E.gram_out.wait_on(s);
        } else {
          comm_allreduce(ctx, comm, gram64.data(), size_t(r) * r, DType::F64, ReduceOp::Sum, s);
        }
        kern::f64_to_f32(gram64.as<double>(), gram32.as<float>(), int64_t(r) * r, s);
      }
      // low-rank path: Y^T Y = Q Lambda Q^T on the device (fp64 Jacobi, identical on every
      // rank: the same allreduced Gramian in, the same deterministic sweeps), the source
      // factors rotated once into that basis — all stream-ordered behind the allreduce
      bool lr_on = false;
      for (const auto& o : dD.lro) lr_on = lr_on || o[4] > o[0];
      if (lr_on) {
        kern::als_gram_eig(gram64.as<double>(), r, ld, eig_scratch.as<double>(), lrQ.as<float>(),
                           lrQT.as<float>(), lrEig.as<float>(), s, 30, 1e-14,
                           ctr.as<unsigned long long>() + 12);
        if (!dS.rot.data()) dS.rot = ctx.alloc(std::max<size_t>(size_t(Src.n) * ld * 4, 256));
        kern::als_rotate(dS.f.as<float>(), nullptr, dS.rot.as<float>(), nullptr, Src.n,
                         lrQ.as<float>(), ld, cus, s);
      }
      if (dD.absmax.data()) {  // this half's source factors bound the split-fp16 scale
        OAP_HIP_CHECK(hipMemsetAsync(dD.absmax.as<unsigned>() + 1, 0, 4, s));
        kern::als_absmax(dS.f.as<float>(), Src.n * ld, dD.absmax.as<unsigned>() + 1, s);
      }
      E.e1.record(s);
      kern::AlsSolveArgs a;
      a.rowptr = dD.ptr.as<int64_t>();
      a.cols = dD.col.as<int32_t>();
      a.vals = dD.val.as<float>();
      a.partials = dD.partials.as<float>();
      a.absmax = dD.absmax.data() ? dD.absmax.as<unsigned>() : nullptr;
      a.src = dS.f.as<float>();
      a.ld = ld;
      a.r = r;
      a.yty = p.implicit ? gram32.as<float>() : nullptr;
      a.alpha = float(p.alpha);
      a.lambda = float(p.reg);
      a.implicit = p.implicit;
      a.dst = dD.f.as<float>() + Dst.off[me] * ld;  // owned rows, in place in the slab
      a.queue = ctr.as<unsigned long long>();
      a.fail = ctr.as<unsigned long long>() + 2;
      if (int(E.solved.size()) != C) {
        E.solved = std::vector<Event>(C);
        E.bc0 = std::vector<Event>(C);
        E.bc1 = std::vector<Event>(C);
      }
      for (int c = 0; c < C; ++c) {
        a.short_rows = dD.short_rows.as<int32_t>() + dD.sr_off[c];
        a.n_short = dD.sr_off[c + 1] - dD.sr_off[c];
        a.long_rows = dD.long_rows.as<int32_t>() + dD.lr_off[c];
        a.n_long = dD.lr_off[c + 1] - dD.lr_off[c];
        a.long_chunk_ptr = dD.long_chunk_ptr.as<int64_t>() + dD.lr_off[c] + c;
        a.chunk_begin = dD.chunk_begin.as<int64_t>() + dD.cb_off[c];
        a.chunk_end = dD.chunk_end.as<int64_t>() + dD.cb_off[c];
        a.n_chunks = dD.cb_off[c + 1] - dD.cb_off[c];
        for (int j = 0; j < 5; ++j) a.lr_off[j] = dD.lro[c][j];
        a.n_direct_x3 = dD.x3n[c];
        if (lr_on) {
          a.lr_src = dS.rot.as<float>();
          a.lr_eig = lrEig.as<float>();
          a.lr_back = lrQT.as<float>();
          a.lr_scratch = dD.lr_scratch.as<float>();
        }
        kern::als_solve(a, cus, s);
        if (local) continue;
        // chunk c of every rank's rows -> every rank (root = owner; in place in the slab)
        auto bcast_chunk = [&](hipStream_t st) {
          if (comm.name() == std::string("rccl")) static_cast<RcclComm&>(comm).group_start();
          for (int q = 0; q < P; ++q) {
            const int64_t lo = Dst.cnt[q] * c / C, hi = Dst.cnt[q] * (c + 1) / C;
            if (hi > lo)
              comm_bcast(ctx, comm, dD.f.as<float>() + (Dst.off[q] + lo) * ld,
                         size_t(hi - lo) * ld, DType::F32, q, st);
          }
          if (comm.name() == std::string("rccl")) static_cast<RcclComm&>(comm).group_end();
        };
        if (dev_comm) {
          E.solved[c].record(s);
          E.solved[c].wait_on(cs);
          E.bc0[c].record(cs);
          bcast_chunk(cs);
          E.bc1[c].record(cs);
        } else {
          bcast_chunk(s);
        }
      }
      E.e2.record(s);
      if (dev_comm) {  // the next half reads every rank's rows
        E.gathered.record(cs);
        E.gathered.wait_on(s);
      }
      E.e3.record(s);
    };
    for (int it = 0; it < p.max_iter; ++it) {
      auto t0 = std::chrono::steady_clock::now();
      {
        TraceRange tr(&ctx.metrics(), "als/half_items");
        half(hev[0], I, dI, U, dU);
      }
      {
        TraceRange tr(&ctx.metrics(), "als/half_users");
        half(hev[1], U, dU, I, dI);
      }
      // one host wait per iteration (both halves queued back to back, nothing in between)
      if (dev_comm) comm.wait(s);
      hev[1].e3.sync();
      for (HalfEvents& E : hev) {
        if (dev_comm)
          for (int c = 0; c < C; ++c) res.bcast_ms += Event::elapsed_ms(E.bc0[c], E.bc1[c]);
        res.gram_ms += Event::elapsed_ms(E.e0, E.e1);
        res.solve_ms += Event::elapsed_ms(E.e1, E.e2);
        res.comm_ms += Event::elapsed_ms(E.e2, E.e3);  // exposed (not overlapped) gather time
      }
      res.iter_ms.push_back(ms_since(t0));
      if (!local)  // every rank's rows but its own, both halves
        res.bcast_recv_bytes += (U.n - U.cnt[me] + I.n - I.cnt[me]) * int64_t(ld) * 4;
      maybe_inject_fault(me, "als_iter", it);
    }
    unsigned long long fails = 0;
    ctx.copy_to_host(&fails, ctr.as<unsigned long long>() + 2, 8);
    unsigned long long eig_uncv = 0;
    ctx.copy_to_host(&eig_uncv, ctr.as<unsigned long long>() + 12, 8);
    res.eig_unconverged = int64_t(eig_uncv);
    if (eig_uncv && me == 0)
      Logger::instance().log(LogLevel::Warn, "als/eig_unconverged",
                             "\"solves\":" + std::to_string(eig_uncv) +
                                 ",\"note\":\"Jacobi sweeps hit max_sweeps (30) above tol 1e-14; "
                                 "low-rank solves used the last basis\"");
    res.failed_rows = int64_t(comm_allreduce_scalar(ctx, comm, double(fails), ReduceOp::Sum));
    // the result handoff (the reference copies each factor row into a Java array,
    // ALSDALImpl.cpp:500-576): pitched 2D copies drop the ld padding on the GPU side into pinned
    // staging, drained by the thread pool straight into the returned (uninitialised) arrays
    res.user_factors = HostArray<float>::alloc(size_t(U.n) * r);
    res.item_factors = HostArray<float>::alloc(size_t(I.n) * r);
    ctx.download_rows(res.user_factors.data(), size_t(r) * 4, dU.f.data(), size_t(ld) * 4,
                      size_t(r) * 4, U.n, s);
    ctx.download_rows(res.item_factors.data(), size_t(r) * 4, dI.f.data(), size_t(ld) * 4,
                      size_t(r) * 4, I.n, s);
  } else {
    Xh.assign(size_t(U.n) * ld, 0.f);
    Yh.assign(size_t(I.n) * ld, 0.f);
    ctx.pool().parallel_for(U.n, [&](int, int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) init_factor_row(p.seed, U.ids[i], r, ld, &Xh[size_t(i) * ld]);
    });
    overlay_init(U.ids, r, ld, p, Xh.data());
    int64_t fails = 0;
    auto half = [&](Side& Dst, std::vector<float>& Fd, Side& Src, std::vector<float>& Fs) {
      auto t0 = std::chrono::steady_clock::now();
      std::vector<double> yty(size_t(r) * r, 0.0);
      if (p.implicit) {
        const int nt = ctx.pool().size();
        std::vector<std::vector<double>> part(nt);
        ctx.pool().parallel_for(Src.cnt[me], [&](int ci, int64_t b, int64_t e) {
          std::vector<double>& G = part[ci];
          G.assign(size_t(r) * r, 0.0);
          for (int64_t k = b; k < e; ++k) {
            const float* y = &Fs[size_t(Src.off[me] + k) * ld];
            for (int i = 0; i < r; ++i)
              for (int j = 0; j <= i; ++j) G[size_t(i) * r + j] += double(y[i]) * double(y[j]);
          }
        });
        for (auto& G : part)
          if (!G.empty())
            for (size_t q = 0; q < yty.size(); ++q) yty[q] += G[q];
        comm_allreduce_host(ctx, comm, yty.data(), yty.size(), DType::F64, ReduceOp::Sum);
      }
      auto t1 = std::chrono::steady_clock::now();
      res.gram_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
      const int64_t nloc = Dst.cnt[me];
      std::vector<float> mine(size_t(std::max<int64_t>(nloc, 1)) * ld, 0.f);
      std::vector<int64_t> fail_part(ctx.pool().size(), 0);
      ctx.pool().parallel_for(nloc, [&](int ci, int64_t b, int64_t e) {
        std::vector<double> A(size_t(r) * r), bv(r), y(r);
        for (int64_t row = b; row < e; ++row) {
          if (p.implicit)
            A = yty;
          else
            std::fill(A.begin(), A.end(), 0.0);
          std::fill(bv.begin(), bv.end(), 0.0);
          int64_t nexp = 0;
          for (int64_t q = Dst.csr.ptr[row]; q < Dst.csr.ptr[row + 1]; ++q) {
            const float* ys = &Fs[size_t(Dst.csr.col[q]) * ld];
            for (int f = 0; f < r; ++f) y[f] = ys[f];
            const double rv = Dst.csr.val[q];
            double ca, cb;
            if (p.implicit) {
              const double c1 = p.alpha * std::fabs(rv);
              ca = c1;
              cb = rv > 0.0 ? 1.0 + c1 : 0.0;
              if (rv > 0.0) ++nexp;
            } else {
              ca = 1.0;
              cb = rv;
              ++nexp;
            }
            for (int i = 0; i < r; ++i) {
              const double yi = ca * y[i];
              for (int j = 0; j <= i; ++j) A[size_t(i) * r + j] += yi * y[j];
              bv[i] += cb * y[i];
            }
          }
          const double lam = p.reg * double(nexp);
          for (int i = 0; i < r; ++i) A[size_t(i) * r + i] += lam;
          float* out = &mine[size_t(row) * ld];
          if (p.nonnegative) {
            const NnlsStatus st = nnls_solve(A, bv, r, y);
            if (st != kNnlsNotSpd)  // (capped: the feasible iterate, still counted below)
              for (int f = 0; f < r; ++f) out[f] = float(y[f]);
            if (st != kNnlsOk) ++fail_part[ci];
          } else if (chol_solve(A, bv, r)) {
            for (int f = 0; f < r; ++f) out[f] = float(bv[f]);
          } else {
            ++fail_part[ci];
          }
        }
      });
      for (int64_t f : fail_part) fails += f;
      auto t2 = std::chrono::steady_clock::now();
      res.solve_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
      if (local) {
        std::copy(mine.begin(), mine.begin() + size_t(nloc) * ld, Fd.begin());
      } else {
        int64_t mx = 1;
        for (int q = 0; q < P; ++q) mx = std::max(mx, Dst.cnt[q]);
        mine.resize(size_t(mx) * ld, 0.f);
        std::vector<float> all(size_t(mx) * ld * P);
        comm_allgather_host(ctx, comm, mine.data(), all.data(), size_t(mx) * ld, DType::F32);
        for (int q = 0; q < P; ++q)
          std::copy(all.begin() + size_t(q) * mx * ld,
                    all.begin() + size_t(q) * mx * ld + size_t(Dst.cnt[q]) * ld,
                    Fd.begin() + size_t(Dst.off[q]) * ld);
      }
      res.comm_ms += ms_since(t2);
    };
    for (int it = 0; it < p.max_iter; ++it) {
      auto t0 = std::chrono::steady_clock::now();
      half(I, Yh, U, Xh);
      half(U, Xh, I, Yh);
      res.iter_ms.push_back(ms_since(t0));
      maybe_inject_fault(me, "als_iter", it);
    }
    res.failed_rows = int64_t(comm_allreduce_scalar(ctx, comm, double(fails), ReduceOp::Sum));
  }
  res.train_ms = ms_since(t_train);
  res.user_ids = U.ids;
  res.item_ids = I.ids;
  if (!Xh.empty() || !Yh.empty()) {  // (host engine: repack [n][ld] -> [n][r] on the pool)
    res.user_factors = HostArray<float>::alloc(size_t(U.n) * r);
    res.item_factors = HostArray<float>::alloc(size_t(I.n) * r);
    auto repack = [&](float* dst, const std::vector<float>& src, int64_t rows) {
      ctx.pool().parallel_for(rows, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i)
          std::memcpy(dst + size_t(i) * r, src.data() + size_t(i) * ld, size_t(r) * 4);
      });
    };
    repack(res.user_factors.data(), Xh, U.n);
    repack(res.item_factors.data(), Yh, I.n);
  }
  if (me == 0 && Logger::instance().level() <= LogLevel::Info)
    Logger::instance().log(LogLevel::Info, "als/fit",
                           "\"nnz\":" + std::to_string(res.nnz) + ",\"users\":" +
                               std::to_string(U.n) + ",\"items\":" + std::to_string(I.n) +
                               ",\"rank\":" + std::to_string(r) + ",\"train_ms\":" +
                               std::to_string(res.train_ms));
  return res;
}

}  // namespace oap
