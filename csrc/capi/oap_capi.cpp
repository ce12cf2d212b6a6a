// C ABI over the native drivers (see oap_capi.h).  Exceptions never cross the boundary: every
// entry point catches, stores the message in a thread-local buffer and returns a negative code.
#include "capi/oap_capi.h"
#include "comm/tcp_comm.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "comm/comm.h"
#include "drivers/als.h"
#include "drivers/kmeans.h"
#include "drivers/pca.h"
#include "kernels/kernels.h"
#include "runtime/context.h"
#include "runtime/table.h"

struct oap_ctx {
  std::unique_ptr<oap::Context> ctx;
  std::shared_ptr<oap::Comm> comm;
};

struct oap_als_result {
  oap::AlsResult r;
};

namespace {

thread_local std::string g_last_error;

template <typename F>
int guarded(F&& f) {
  try {
    g_last_error.clear();
    f();
    return 0;
  } catch (const oap::CommError& e) {
    g_last_error = std::string("CommError: ") + e.what();
    return -3;
  } catch (const oap::ConfigError& e) {
    g_last_error = std::string("ConfigError: ") + e.what();
    return -2;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return -1;
  } catch (...) {
    g_last_error = "unknown native error";
    return -1;
  }
}

// Rank-local rows -> the backend's K-Means / PCA table layout.
oap::DenseTable upload(oap_ctx* c, const double* x, int64_t rows, int cols, bool kmeans_layout,
                       bool bf16) {
  OAP_CHECK(c && c->ctx, "null context");
  OAP_CHECK(rows >= 0 && cols > 0, "bad shape " << rows << "x" << cols);
  OAP_CHECK(x || rows == 0, "null row buffer");
  oap::Context& ctx = *c->ctx;
  if (!ctx.is_gpu())
    return oap::upload_dense(ctx, x, oap::DType::F64, rows, cols, cols, oap::DType::F64, cols);
  const oap::DType st = bf16 ? oap::DType::BF16 : oap::DType::F32;
  const int64_t ld = kmeans_layout ? oap::kern::kmeans_ld(cols, bf16) : cols;
  return oap::upload_dense(ctx, x, oap::DType::F64, rows, cols, cols,
                           kmeans_layout ? st : oap::DType::F32, ld);
}

}  // namespace

extern "C" {

int oap_capi_version(void) { return OAP_CAPI_VERSION; }

const char* oap_last_error(void) { return g_last_error.c_str(); }

int oap_device_count(void) { return oap::visible_device_count(); }

int oap_check_platform(int device) {
  int ok = 0;
  const int rc = guarded([&] {
    if (device < 0 || device >= oap::visible_device_count()) return;
    const oap::DeviceInfo d = oap::query_device(device);
    ok = d.arch.rfind("gfx950", 0) == 0 ? 1 : 0;
  });
  return rc < 0 ? rc : ok;
}

oap_ctx* oap_ctx_create(int device, double hbm_fraction, int cpu_threads) {
  oap_ctx* out = nullptr;
  guarded([&] {
    auto c = std::make_unique<oap_ctx>();
    c->ctx = std::make_unique<oap::Context>(device, hbm_fraction, cpu_threads);
    c->comm = std::make_shared<oap::LocalComm>(device >= 0);
    out = c.release();
  });
  return out;
}

void oap_ctx_destroy(oap_ctx* ctx) {
  guarded([&] {
    if (!ctx) return;
    ctx->comm.reset();
    delete ctx;
  });
}

int oap_rccl_unique_id(unsigned char out[OAP_UNIQUE_ID_BYTES]) {
  return guarded([&] {
    const std::string id = oap::rccl_unique_id();
    OAP_CHECK(id.size() <= OAP_UNIQUE_ID_BYTES, "unique id of " << id.size() << " bytes");
    std::memset(out, 0, OAP_UNIQUE_ID_BYTES);
    std::memcpy(out, id.data(), id.size());
  });
}

int oap_ctx_join(oap_ctx* c, const unsigned char id[OAP_UNIQUE_ID_BYTES], int world, int rank,
                 double timeout_s) {
  return guarded([&] {
    OAP_CHECK(c && c->ctx, "null context");
    OAP_CHECK(c->ctx->is_gpu(), "RCCL communicators need a GPU context");
    OAP_CHECK(world >= 1 && rank >= 0 && rank < world, "bad world/rank " << world << "/" << rank);
    if (world == 1) {
      c->comm = std::make_shared<oap::LocalComm>(true);
      return;
    }
    std::string uid(reinterpret_cast<const char*>(id), OAP_UNIQUE_ID_BYTES);
    c->comm = std::make_shared<oap::RcclComm>(uid, world, rank, c->ctx->device(), timeout_s);
  });
}

int oap_ctx_join_kvs(oap_ctx* c, const char* ip_port, int world, int rank, double timeout_s) {
  return guarded([&] {
    OAP_CHECK(c && c->ctx, "null context");
    OAP_CHECK(world >= 1 && rank >= 0 && rank < world, "bad world/rank " << world << "/" << rank);
    std::string ip;
    int port = 0;
    OAP_CHECK(ip_port && oap::parse_kvs_address(ip_port, &ip, &port),
              "expected an \"ip_port\" rendezvous address, got '" << (ip_port ? ip_port : "")
                                                                     << "'");
    if (world == 1) {
      c->comm = std::make_shared<oap::LocalComm>(c->ctx->is_gpu());
      return;
    }
    auto store = std::make_shared<oap::TcpStore>(ip, port, world, rank, timeout_s);
    if (c->ctx->is_gpu()) {
      std::string uid = rank == 0 ? oap::rccl_unique_id() : std::string(OAP_UNIQUE_ID_BYTES, '\0');
      store->broadcast(uid.data(), uid.size());
      c->comm = std::make_shared<oap::RcclComm>(uid, world, rank, c->ctx->device(), timeout_s);
    } else {
      c->comm = std::make_shared<oap::TcpComm>(store);
    }
  });
}

int oap_ctx_world_size(const oap_ctx* c) { return c && c->comm ? c->comm->size() : -1; }
int oap_ctx_rank(const oap_ctx* c) { return c && c->comm ? c->comm->rank() : -1; }

int oap_kmeans_fit(oap_ctx* c, const double* x, int64_t rows, int cols,
                   const double* init_centers, int k, int max_iter, double tol, int storage_bf16,
                   double* out_centers, double* out_cost, int* out_iters) {
  return guarded([&] {
    OAP_CHECK(init_centers && k >= 1, "initial centers required (k >= 1)");
    oap::DenseTable t = upload(c, x, rows, cols, true, storage_bf16 != 0);
    oap::KMeansParams p;
    p.k = k;
    p.max_iter = max_iter;
    p.tol = tol;
    p.init = oap::KMeansInit::Given;
    std::vector<double> init(init_centers, init_centers + size_t(k) * cols);
    oap::KMeansResult r = oap::kmeans_fit(*c->ctx, *c->comm, t, init, p);
    if (out_centers) std::memcpy(out_centers, r.centers.data(), r.centers.size() * sizeof(double));
    if (out_cost) *out_cost = r.cost;
    if (out_iters) *out_iters = r.num_iter;
  });
}

int oap_kmeans_init(oap_ctx* c, const double* x, int64_t rows, int cols, int k, const char* mode,
                    int init_steps, uint64_t seed, double* out_centers, int* out_k) {
  return guarded([&] {
    oap::DenseTable t = upload(c, x, rows, cols, true, false);
    oap::KMeansParams p;
    p.k = k;
    p.init_steps = init_steps;
    p.seed = seed;
    const std::string m = mode ? mode : "k-means||";
    OAP_CHECK(m == "random" || m == "k-means||", "unknown init mode '" << m << "'");
    p.init = m == "random" ? oap::KMeansInit::Random : oap::KMeansInit::Parallel;
    int keff = 0;
    std::vector<double> cs = oap::kmeans_init_centers(*c->ctx, *c->comm, t, p, &keff);
    if (out_centers) std::memcpy(out_centers, cs.data(), cs.size() * sizeof(double));
    if (out_k) *out_k = keff;
  });
}

int oap_kmeans_predict(oap_ctx* c, const double* x, int64_t rows, int cols, const double* centers,
                       int k, int32_t* labels, double* dist2) {
  return guarded([&] {
    OAP_CHECK(centers && k >= 1, "centers required");
    oap::DenseTable t = upload(c, x, rows, cols, true, false);
    std::vector<double> cs(centers, centers + size_t(k) * cols);
    std::vector<int32_t> lab(rows);
    std::vector<double> d2(rows);
    oap::kmeans_predict(*c->ctx, t, cs, k, lab.data(), d2.data());
    if (labels) std::memcpy(labels, lab.data(), lab.size() * sizeof(int32_t));
    if (dist2) std::memcpy(dist2, d2.data(), d2.size() * sizeof(double));
  });
}

int oap_pca_fit(oap_ctx* c, const double* x, int64_t rows, int cols, int k, double* out_pc,
                double* out_explained) {
  return guarded([&] {
    OAP_CHECK(k >= 1 && k <= cols, "k must be in [1, cols]");
    oap::DenseTable t = upload(c, x, rows, cols, false, false);
    oap::PcaParams p;
    p.k = k;
    oap::PcaResult r = oap::pca_fit(*c->ctx, *c->comm, t, p);
    if (out_pc) std::memcpy(out_pc, r.pc.data(), r.pc.size() * sizeof(double));
    if (out_explained)
      std::memcpy(out_explained, r.explained.data(), r.explained.size() * sizeof(double));
  });
}

int oap_als_fit(oap_ctx* c, const int32_t* users, const int32_t* items, const float* ratings,
                int64_t n, int rank, int max_iter, double reg, double alpha, int implicit,
                uint64_t seed, oap_als_result** out) {
  return guarded([&] {
    OAP_CHECK(c && c->ctx && out, "null argument");
    OAP_CHECK(n == 0 || (users && items && ratings), "null rating buffers");
    oap::AlsParams p;
    p.rank = rank;
    p.max_iter = max_iter;
    p.reg = reg;
    p.alpha = alpha;
    p.implicit = implicit != 0;
    p.seed = seed;
    auto res = std::make_unique<oap_als_result>();
    res->r = oap::als_fit(*c->ctx, *c->comm, users, items, ratings, n, p);
    *out = res.release();
  });
}

int64_t oap_als_result_count(const oap_als_result* res, int which) {
  if (!res) return -1;
  return static_cast<int64_t>(which == 0 ? res->r.user_ids.size() : res->r.item_ids.size());
}

int oap_als_result_rank(const oap_als_result* res) { return res ? res->r.rank : -1; }

const int32_t* oap_als_result_ids(const oap_als_result* res, int which) {
  if (!res) return nullptr;
  return which == 0 ? res->r.user_ids.data() : res->r.item_ids.data();
}

const float* oap_als_result_factors(const oap_als_result* res, int which) {
  if (!res) return nullptr;
  return which == 0 ? res->r.user_factors.data() : res->r.item_factors.data();
}

void oap_als_result_free(oap_als_result* res) { delete res; }

int oap_shuffle_ratings(oap_ctx* c, const void* records, int64_t n, int64_t n_total_keys,
                        int n_blocks, void** out, int64_t* out_n, int64_t* out_distinct) {
  return guarded([&] {
    OAP_CHECK(c && c->ctx && c->comm && out && out_n && out_distinct, "null argument");
    OAP_CHECK(n == 0 || records, "null record buffer");
    const int P = c->comm->size();
    OAP_CHECK(n_blocks == P, "n_blocks " << n_blocks << " != world size " << P);
    constexpr size_t kRec = 20;
    const int64_t per = std::max<int64_t>(n_total_keys / n_blocks, 1);
    const auto* rec = static_cast<const unsigned char*>(records);
    auto key_of = [&](const unsigned char* r) {
      int64_t k;
      std::memcpy(&k, r, 8);
      return k;
    };
    std::vector<size_t> send_cnt(P, 0), recv_cnt(P, 0);
    std::vector<int> dest(size_t(std::max<int64_t>(n, 0)));
    for (int64_t i = 0; i < n; ++i) {
      const int64_t k = key_of(rec + kRec * i);
      OAP_CHECK(k >= 0, "negative rating key " << k);
      dest[i] = int(std::min<int64_t>(k / per, P - 1));
      ++send_cnt[dest[i]];
    }
    std::vector<size_t> off(P + 1, 0);
    for (int q = 0; q < P; ++q) off[q + 1] = off[q] + send_cnt[q];
    std::vector<unsigned char> sendbuf(size_t(n) * kRec);
    {
      std::vector<size_t> pos(off.begin(), off.end() - 1);
      for (int64_t i = 0; i < n; ++i)
        std::memcpy(&sendbuf[kRec * pos[dest[i]]++], rec + kRec * i, kRec);
    }
    // counts: one int64 per peer
    std::vector<int64_t> sc(P), rc(P);
    for (int q = 0; q < P; ++q) sc[q] = int64_t(send_cnt[q]);
    oap::comm_alltoallv_host(*c->ctx, *c->comm, sc.data(), std::vector<size_t>(P, 1), rc.data(),
                             std::vector<size_t>(P, 1), oap::DType::I64);
    size_t rn = 0;
    for (int q = 0; q < P; ++q) {
      recv_cnt[q] = size_t(rc[q]);
      rn += recv_cnt[q];
    }
    std::vector<size_t> sb(P), rb(P);
    for (int q = 0; q < P; ++q) {
      sb[q] = send_cnt[q] * kRec;
      rb[q] = recv_cnt[q] * kRec;
    }
    auto* buf = static_cast<unsigned char*>(std::malloc(std::max<size_t>(rn * kRec, 1)));
    OAP_CHECK(buf, "out of host memory");
    oap::comm_alltoallv_host(*c->ctx, *c->comm, sendbuf.data(), sb, buf, rb, oap::DType::U8);
    // sort by (key, other), then count distinct keys (ALSShuffle.cpp:111,121)
    std::vector<std::pair<std::pair<int64_t, int64_t>, size_t>> order(rn);
    for (size_t i = 0; i < rn; ++i) {
      int64_t k, o;
      std::memcpy(&k, buf + kRec * i, 8);
      std::memcpy(&o, buf + kRec * i + 8, 8);
      order[i] = {{k, o}, i};
    }
    std::sort(order.begin(), order.end());
    auto* sorted = static_cast<unsigned char*>(std::malloc(std::max<size_t>(rn * kRec, 1)));
    if (!sorted) {
      std::free(buf);
      OAP_THROW(oap::Error, "out of host memory");
    }
    int64_t distinct = 0;
    for (size_t i = 0; i < rn; ++i) {
      std::memcpy(sorted + kRec * i, buf + kRec * order[i].second, kRec);
      if (i == 0 || order[i].first.first != order[i - 1].first.first) ++distinct;
    }
    std::free(buf);
    *out = sorted;
    *out_n = int64_t(rn);
    *out_distinct = distinct;
  });
}

int oap_allreduce_i64(oap_ctx* c, int64_t* vals, int count, int op) {
  return guarded([&] {
    OAP_CHECK(c && c->ctx && c->comm && (vals || count == 0), "null argument");
    const oap::ReduceOp o =
        op == 1 ? oap::ReduceOp::Max : op == 2 ? oap::ReduceOp::Min : oap::ReduceOp::Sum;
    oap::comm_allreduce_host(*c->ctx, *c->comm, vals, size_t(count), oap::DType::I64, o);
  });
}

void oap_free(void* p) { std::free(p); }

}  // extern "C"
