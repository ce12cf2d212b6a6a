// ALS bindings: the role of the reference's JNI entries ALSDALImpl.cShuffleData and
// cDALImplictALS (mllib-dal/src/main/native/javah/org_apache_spark_ml_recommendation_
// ALSDALImpl.h:12-24) — one call takes this rank's ratings (any partition) and returns the full
// id-indexed factor matrices instead of per-rank native tables plus offsets.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "bindings/bindings.h"
#include "drivers/als.h"
#include "drivers/recommend.h"
#include "kernels/kernels.h"

namespace py = pybind11;
using namespace oap;

void register_als(py::module_& m) {
  // the device Jacobi of kernels/als_eig.hip on a given symmetric matrix (tests)
  m.def(
      "als_gram_eig",
      [](std::shared_ptr<Context> ctx,
         py::array_t<double, py::array::c_style | py::array::forcecast> g, int ld) {
        if (g.ndim() != 2 || g.shape(0) != g.shape(1)) throw ConfigError("square matrix needed");
        if (!ctx->is_gpu()) throw ConfigError("als_gram_eig needs a GPU context");
        const int r = int(g.shape(0));
        if (ld <= 0) ld = int(round_up(size_t(r), 16));
        py::array_t<float> q({ld, ld}), qt({ld, ld}), e(ld);
        {
          py::gil_scoped_release rel;
          ctx->activate();
          hipStream_t s = ctx->compute();
          Buffer dg = ctx->alloc(size_t(r) * r * 8), dq = ctx->alloc(size_t(ld) * ld * 4),
                 dqt = ctx->alloc(size_t(ld) * ld * 4), de = ctx->alloc(size_t(ld) * 4),
                 sc = ctx->alloc(kern::als_gram_eig_scratch_bytes(r));
          ctx->copy_to_backend(dg.data(), g.data(), size_t(r) * r * 8, s);
          kern::als_gram_eig(dg.as<double>(), r, ld, sc.as<double>(), dq.as<float>(),
                             dqt.as<float>(), de.as<float>(), s);
          ctx->copy_to_host(q.mutable_data(), dq.data(), size_t(ld) * ld * 4, s);
          ctx->copy_to_host(qt.mutable_data(), dqt.data(), size_t(ld) * ld * 4, s);
          ctx->copy_to_host(e.mutable_data(), de.data(), size_t(ld) * 4, s);
        }
        return py::make_tuple(q, qt, e);
      },
      py::arg("ctx"), py::arg("gram"), py::arg("ld") = 0);
  m.def(
      "als_fit",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<Comm> comm,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> users,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> items,
         py::array_t<float, py::array::c_style | py::array::forcecast> ratings, int rank,
         int max_iter, double reg, double alpha, bool implicit, uint64_t seed,
         py::object init_ids, py::object init_factors, bool host_engine, bool nonnegative) {
        const int64_t n = users.size();
        if (items.size() != n || ratings.size() != n)
          throw ConfigError("users, items and ratings must have the same length");
        AlsParams p;
        p.rank = rank;
        p.max_iter = max_iter;
        p.reg = reg;
        p.alpha = alpha;
        p.implicit = implicit;
        p.seed = seed;
        p.host_engine = host_engine;
        p.nonnegative = nonnegative;
        py::array_t<int32_t, py::array::c_style | py::array::forcecast> iid;
        py::array_t<float, py::array::c_style | py::array::forcecast> ifac;
        if (!init_ids.is_none()) {
          iid = init_ids;
          ifac = init_factors;
          if (ifac.ndim() != 2 || ifac.shape(0) != iid.size() || ifac.shape(1) != rank)
            throw ConfigError("init_factors must be len(init_ids) x rank");
          for (int64_t q = 1; q < iid.size(); ++q)
            if (iid.data()[q - 1] >= iid.data()[q])
              throw ConfigError("init_ids must be strictly ascending");
          p.init_ids = iid.data();
          p.init_factors = ifac.data();
          p.n_init = iid.size();
        }
        AlsResult r;
        {
          py::gil_scoped_release rel;
          r = als_fit(*ctx, *comm, users.data(), items.data(), ratings.data(), n, p);
        }
        auto ids = [](const std::vector<int32_t>& v) {
          py::array_t<int32_t> a(int64_t(v.size()));
          if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * 4);
          return a;
        };
        auto fac = [&](const HostArray<float>& v, size_t rows) {
          if (v.empty() || rows == 0) return py::array_t<float>({int64_t(rows), int64_t(r.rank)});
          // zero-copy: the array keeps the native buffer alive
          auto* keep = new std::shared_ptr<float>(v.owner());
          py::capsule owner(keep, [](void* q) { delete static_cast<std::shared_ptr<float>*>(q); });
          return py::array_t<float>({int64_t(rows), int64_t(r.rank)},
                                    {int64_t(r.rank) * 4, int64_t(4)}, v.data(), owner);
        };
        py::dict out;
        out["user_ids"] = ids(r.user_ids);
        out["item_ids"] = ids(r.item_ids);
        out["user_factors"] = fac(r.user_factors, r.user_ids.size());
        out["item_factors"] = fac(r.item_factors, r.item_ids.size());
        out["nnz"] = r.nnz;
        out["setup_ms"] = r.setup_ms;
        out["train_ms"] = r.train_ms;
        out["iter_ms"] = r.iter_ms;
        out["gram_ms"] = r.gram_ms;
        out["solve_ms"] = r.solve_ms;
        out["comm_ms"] = r.comm_ms;
        out["bcast_ms"] = r.bcast_ms;
        out["bcast_recv_bytes"] = r.bcast_recv_bytes;
        out["failed_rows"] = r.failed_rows;
        out["eig_unconverged"] = r.eig_unconverged;
        return out;
      },
      py::arg("ctx"), py::arg("comm"), py::arg("users"), py::arg("items"), py::arg("ratings"),
      py::arg("rank") = 10, py::arg("max_iter") = 10, py::arg("reg") = 0.1,
      py::arg("alpha") = 1.0, py::arg("implicit") = true, py::arg("seed") = 0,
      py::arg("init_ids") = py::none(), py::arg("init_factors") = py::none(),
      py::arg("host_engine") = false, py::arg("nonnegative") = false);
  m.def("als_max_rank", &kern::als_max_rank);
  // recommendForAll*: fused score + top-k (kernels/als_recommend.hip); no score matrix stored
  m.def("als_recommend_max_num", &als_recommend_max_num);
  m.def(
      "als_recommend",
      [](std::shared_ptr<Context> ctx,
         py::array_t<float, py::array::c_style | py::array::forcecast> src,
         py::array_t<float, py::array::c_style | py::array::forcecast> dst, int num,
         int64_t slab_rows) {
        if (src.ndim() != 2 || dst.ndim() != 2 || src.shape(1) != dst.shape(1))
          throw ConfigError("als_recommend: src [n, rank] and dst [m, rank] needed");
        const int64_t n = src.shape(0), m = dst.shape(0);
        const int rank = int(src.shape(1));
        py::array_t<int32_t> idx({n, int64_t(num)});
        py::array_t<float> val({n, int64_t(num)});
        RecTiming t;
        {
          py::gil_scoped_release rel;
          als_recommend(*ctx, src.data(), n, dst.data(), m, rank, num, idx.mutable_data(),
                        val.mutable_data(), slab_rows, &t);
        }
        py::dict info;
        info["pack_dst_s"] = t.pack_dst_s;
        info["upload_s"] = t.upload_s;
        info["topk_s"] = t.topk_s;
        info["download_s"] = t.download_s;
        info["wall_s"] = t.wall_s;
        info["slabs"] = t.slabs;
        info["slab_rows"] = t.slab_rows;
        return py::make_tuple(idx, val, info);
      },
      py::arg("ctx"), py::arg("src"), py::arg("dst"), py::arg("num"), py::arg("slab_rows") = 0);
}
