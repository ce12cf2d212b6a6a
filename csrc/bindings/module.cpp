// Python bindings for the MI355X-native MLlib engine (pybind11).
//
// Plays the role of the reference's JNI surface (mllib-dal/src/main/native/javah/*.h; SURVEY.md
// §2.8) for the Python API layer: native handles are RAII objects owned by Python (no leaked
// `new SharedPtr<...>` as in KMeansDALImpl.cpp:245), arrays cross as numpy buffers, and native
// exceptions become oap_mllib_amd.errors.* Python exceptions instead of exit().
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "bindings/bindings.h"
#include "comm/comm.h"
#include "comm/tcp_comm.h"
#include "drivers/kmeans.h"
#include "kernels/kernels.h"
#include "runtime/context.h"
#include "runtime/knobs.h"
#include "runtime/table.h"

namespace py = pybind11;
using namespace oap;

namespace oap {
namespace py_bind {

py::dtype np_dtype(DType t) {
  switch (t) {
    case DType::F32: return py::dtype::of<float>();
    case DType::F64: return py::dtype::of<double>();
    case DType::BF16: return py::dtype("uint16");
    case DType::I32: return py::dtype::of<int32_t>();
    case DType::I64: return py::dtype::of<int64_t>();
    case DType::U8: return py::dtype::of<uint8_t>();
  }
  return py::dtype::of<uint8_t>();
}

const char* op_name(ReduceOp op) {
  switch (op) {
    case ReduceOp::Sum: return "sum";
    case ReduceOp::Max: return "max";
    case ReduceOp::Min: return "min";
  }
  return "sum";
}

// Non-owning numpy view over a host pointer.
py::array host_view(void* p, size_t count, DType t) {
  py::capsule nothing(p, [](void*) {});
  return py::array(np_dtype(t), {static_cast<py::ssize_t>(count)}, {}, p, nothing);
}

// Comm implemented by a Python object (torch.distributed / gloo on CPU, or anything exposing
// allreduce/allgather/alltoallv/bcast/barrier over numpy arrays).
class HostComm final : public Comm {
 public:
  HostComm(py::object impl, int rank, int world)
      : impl_(std::move(impl)), rank_(rank), world_(world) {}
  ~HostComm() override {
    py::gil_scoped_acquire g;
    impl_ = py::object();
  }
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  bool on_device() const override { return false; }
  const char* name() const override { return "host"; }
  void allreduce(void* buf, size_t count, DType dt, ReduceOp op, hipStream_t) override {
    py::gil_scoped_acquire g;
    call("allreduce", host_view(buf, count, dt), op_name(op));
  }
  void allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t) override {
    py::gil_scoped_acquire g;
    call("allgather", host_view(const_cast<void*>(send), count, dt),
         host_view(recv, count * world_, dt));
  }
  void alltoallv(const void* send, const std::vector<size_t>& sc, void* recv,
                 const std::vector<size_t>& rc, DType dt, hipStream_t) override {
    py::gil_scoped_acquire g;
    size_t sn = 0, rn = 0;
    for (auto c : sc) sn += c;
    for (auto c : rc) rn += c;
    call("alltoallv", host_view(const_cast<void*>(send), sn, dt), py::cast(sc),
         host_view(recv, rn, dt), py::cast(rc));
  }
  void bcast(void* buf, size_t count, DType dt, int root, hipStream_t) override {
    py::gil_scoped_acquire g;
    call("bcast", host_view(buf, count, dt), root);
  }
  void barrier() override {
    py::gil_scoped_acquire g;
    call("barrier");
  }

 private:
  template <typename... A>
  void call(const char* m, A&&... args) {
    try {
      impl_.attr(m)(std::forward<A>(args)...);
    } catch (py::error_already_set& e) {
      throw CommError(std::string("host comm ") + m + " failed: " + e.what());
    }
  }
  py::object impl_;
  int rank_, world_;
};

DType parse_dtype(const std::string& s) {
  if (s == "f32" || s == "float32") return DType::F32;
  if (s == "f64" || s == "float64") return DType::F64;
  if (s == "bf16" || s == "bfloat16") return DType::BF16;
  if (s == "i32" || s == "int32") return DType::I32;
  if (s == "i64" || s == "int64") return DType::I64;
  throw ConfigError("unknown dtype '" + s + "'");
}

py::dict metrics_dict(Context& ctx) {
  py::dict phases;
  for (auto& kv : ctx.metrics().phases()) {
    py::dict e;
    e["count"] = kv.second.count;
    e["total_us"] = kv.second.total_us;
    e["max_us"] = kv.second.max_us;
    e["bytes"] = kv.second.bytes;
    phases[py::str(kv.first)] = e;
  }
  py::dict vals;
  for (auto& kv : ctx.metrics().values()) vals[py::str(kv.first)] = kv.second;
  py::dict out;
  out["phases"] = phases;
  out["values"] = vals;
  if (ctx.is_gpu()) {
    py::dict arena;
    arena["used"] = ctx.arena()->used();
    arena["peak"] = ctx.arena()->peak();
    arena["reserved"] = ctx.arena()->reserved();
    arena["budget"] = ctx.arena()->budget();
    out["arena"] = arena;
  }
  return out;
}

}  // namespace py_bind
}  // namespace oap

using namespace oap::py_bind;

PYBIND11_MODULE(_native, m) {
  m.doc() = "MI355X-native (gfx950) K-Means / PCA / ALS engine";

  // ---------------------------------------------------------------- exceptions
  static py::exception<Error> exc_base(m, "OapError");
  static py::exception<DeviceError> exc_dev(m, "DeviceError", exc_base.ptr());
  static py::exception<CommError> exc_comm(m, "CommError", exc_base.ptr());
  static py::exception<ConfigError> exc_cfg(m, "ConfigError", exc_base.ptr());
  static py::exception<OutOfMemoryError> exc_oom(m, "OutOfMemoryError", exc_base.ptr());
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const OutOfMemoryError& e) {
      py::set_error(exc_oom, e.what());
    } catch (const ConfigError& e) {
      py::set_error(exc_cfg, e.what());
    } catch (const CommError& e) {
      py::set_error(exc_comm, e.what());
    } catch (const DeviceError& e) {
      py::set_error(exc_dev, e.what());
    } catch (const Error& e) {
      py::set_error(exc_base, e.what());
    }
  });

  // ---------------------------------------------------------------- runtime
  m.def("visible_device_count", &visible_device_count);
  m.def("rccl_available", &rccl_available);
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def(
      "configure_logging",
      [](int rank, int device, const std::string& level, const std::string& path) {
        LogLevel l = LogLevel::Warn;
        if (level == "debug") l = LogLevel::Debug;
        else if (level == "info") l = LogLevel::Info;
        else if (level == "warn") l = LogLevel::Warn;
        else if (level == "error") l = LogLevel::Error;
        else if (level == "off") l = LogLevel::Off;
        Logger::instance().configure(rank, device, l, path);
      },
      py::arg("rank"), py::arg("device"), py::arg("level") = "warn", py::arg("path") = "");
  // the native knob registry (runtime/knobs.h): Config.native_knobs installs overrides
  m.def("set_knob", &set_knob, py::arg("name"), py::arg("value"),
        "install (value non-empty) or remove (empty) a native knob override");
  m.def("clear_knobs", &clear_knobs);
  m.def("knob_value", [](const std::string& name) { return knob_str(name.c_str()); },
        py::arg("name"));
  m.def("knob_table", []() {
    py::list out;
    for (const KnobInfo& k : knob_table()) {
      py::dict d;
      d["name"] = k.name;
      d["default"] = k.def;
      d["doc"] = k.doc;
      out.append(d);
    }
    return out;
  });
  m.def("log", [](const std::string& level, const std::string& phase, const std::string& fields) {
    LogLevel l = level == "error" ? LogLevel::Error
                 : level == "warn" ? LogLevel::Warn
                 : level == "debug" ? LogLevel::Debug
                                    : LogLevel::Info;
    Logger::instance().log(l, phase, fields);
  });
  m.def("roctx_push", [](const std::string& s) { roctx_push(s.c_str()); });
  m.def("roctx_pop", []() { roctx_pop(); });

  py::class_<Context, std::shared_ptr<Context>>(m, "Context")
      .def(py::init<int, double, int>(), py::arg("device") = -1, py::arg("hbm_fraction") = 0.9,
           py::arg("cpu_threads") = 0)
      .def_property_readonly("is_gpu", &Context::is_gpu)
      .def_property_readonly("device", &Context::device)
      .def_property_readonly("info",
                             [](Context& c) {
                               py::dict d;
                               auto& i = c.info();
                               d["id"] = i.id;
                               d["name"] = i.name;
                               d["arch"] = i.arch;
                               d["cu_count"] = i.cu_count;
                               d["total_mem"] = i.total_mem;
                               d["free_mem"] = i.free_mem;
                               d["lds_per_block"] = i.lds_per_block;
                               d["warp_size"] = i.warp_size;
                               return d;
                             })
      .def("metrics", [](Context& c) { return metrics_dict(c); })
      .def("reset_metrics", [](Context& c) { c.metrics().reset(); })
      .def("sync", [](Context& c) {
        py::gil_scoped_release r;
        c.sync_all();
      })
      .def("trim", [](Context& c) {
        if (c.is_gpu()) c.arena()->trim();
      });

  // ---------------------------------------------------------------- comms
  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("on_device", &Comm::on_device)
      .def_property_readonly("name", [](Comm& c) { return std::string(c.name()); })
      .def("barrier",
           [](Comm& c) {
             py::gil_scoped_release r;
             c.barrier();
           })
      .def("abort", &Comm::abort)
      .def(
          "allreduce_f64",
          [](Comm& c, std::shared_ptr<Context> ctx, py::array_t<double> a, const std::string& op) {
            auto buf = a.request(true);
            ReduceOp o = op == "max" ? ReduceOp::Max : op == "min" ? ReduceOp::Min : ReduceOp::Sum;
            double* p = static_cast<double*>(buf.ptr);
            size_t n = static_cast<size_t>(buf.size);
            py::gil_scoped_release r;
            if (!c.on_device()) {
              c.allreduce(p, n, DType::F64, o, nullptr);
            } else {
              Buffer d = ctx->alloc(n * 8);
              hipStream_t s = ctx->comm_stream();
              OAP_HIP_CHECK(hipMemcpyAsync(d.data(), p, n * 8, hipMemcpyHostToDevice, s));
              c.allreduce(d.data(), n, DType::F64, o, s);
              OAP_HIP_CHECK(hipMemcpyAsync(p, d.data(), n * 8, hipMemcpyDeviceToHost, s));
              c.wait(s);
            }
          },
          py::arg("ctx"), py::arg("array"), py::arg("op") = "sum")
      .def_property_readonly("trivial", &Comm::trivial)
      // ---- collectives on backend buffers (device memory for a GPU context), numpy in / out:
      // they drive the same comm_* helpers the drivers use, so a 1-rank RCCL communicator runs
      // its real device code (send/recv to self, grouped launches, watchdog waits) in tests
      .def(
          "exchange_f64",
          [](Comm& c, std::shared_ptr<Context> ctx, const std::string& op,
             py::array_t<double, py::array::c_style | py::array::forcecast> a,
             std::vector<size_t> send_counts, std::vector<size_t> recv_counts, int root,
             bool grouped) {
            const size_t n = size_t(a.size());
            const int P = c.size();
            size_t out_n = n;
            if (op == "allgather") out_n = n * P;
            if (op == "alltoallv") {
              OAP_CHECK(int(send_counts.size()) == P && int(recv_counts.size()) == P,
                        "exchange_f64: counts need one entry per rank");
              out_n = 0;
              for (size_t v : recv_counts) out_n += v;
            }
            std::vector<double> hin(a.data(), a.data() + n), hout(std::max<size_t>(out_n, 1));
            {
              py::gil_scoped_release r;
              ctx->activate();
              hipStream_t s = ctx->is_gpu() ? ctx->compute() : nullptr;
              Buffer din = ctx->alloc(std::max<size_t>(n, 1) * 8);
              Buffer dout = ctx->alloc(std::max<size_t>(out_n, 1) * 8);
              ctx->copy_to_backend(din.data(), hin.data(), n * 8, s);
              RcclComm* rc = dynamic_cast<RcclComm*>(&c);
              if (grouped && rc) rc->group_start();
              if (op == "allreduce") {
                comm_allreduce(*ctx, c, din.data(), n, DType::F64, ReduceOp::Sum, s);
              } else if (op == "allreduce_max") {
                comm_allreduce(*ctx, c, din.data(), n, DType::F64, ReduceOp::Max, s);
              } else if (op == "allgather") {
                comm_allgather(*ctx, c, din.data(), dout.data(), n, DType::F64, s);
              } else if (op == "bcast") {
                comm_bcast(*ctx, c, din.data(), n, DType::F64, root, s);
              } else if (op == "alltoallv") {
                comm_alltoallv(*ctx, c, din.data(), send_counts, dout.data(), recv_counts,
                               DType::F64, s);
              } else {
                OAP_THROW(ConfigError, "exchange_f64: unknown op " << op);
              }
              if (grouped && rc) rc->group_end();
              if (ctx->is_gpu()) c.wait(s);  // watchdog wait (RcclComm) / stream sync
              const bool in_place = op == "allreduce" || op == "allreduce_max" || op == "bcast";
              ctx->copy_to_host(hout.data(), (in_place ? din : dout).data(), out_n * 8, s);
            }
            hout.resize(out_n);
            return py::array_t<double>(py::ssize_t(out_n), hout.data());
          },
          py::arg("ctx"), py::arg("op"), py::arg("array"),
          py::arg("send_counts") = std::vector<size_t>{},
          py::arg("recv_counts") = std::vector<size_t>{}, py::arg("root") = 0,
          py::arg("grouped") = false);
  py::class_<LocalComm, Comm, std::shared_ptr<LocalComm>>(m, "LocalComm")
      .def(py::init<bool>(), py::arg("device") = false);
  py::class_<RcclComm, Comm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int world, int rank, int device, double timeout) {
             std::string id = uid;
             py::gil_scoped_release r;
             return std::make_shared<RcclComm>(id, world, rank, device, timeout);
           }),
           py::arg("unique_id"), py::arg("world"), py::arg("rank"), py::arg("device"),
           py::arg("timeout_s") = 600.0);
  // the KVS-rendezvous host comm (JNI / C ABI worlds), for tests of its collectives
  py::class_<TcpComm, Comm, std::shared_ptr<TcpComm>>(m, "TcpComm")
      .def(py::init([](const std::string& address, int world, int rank, double timeout) {
             std::string ip;
             int port = 0;
             OAP_CHECK(parse_kvs_address(address, &ip, &port),
                       "TcpComm: address must be ip_port or ip:port");
             py::gil_scoped_release r;
             return std::make_shared<TcpComm>(
                 std::make_shared<TcpStore>(ip, port, world, rank, timeout));
           }),
           py::arg("address"), py::arg("world"), py::arg("rank"), py::arg("timeout_s") = 60.0);
  py::class_<HostComm, Comm, std::shared_ptr<HostComm>>(m, "HostComm")
      .def(py::init<py::object, int, int>(), py::arg("impl"), py::arg("rank"), py::arg("world"));

  // ---------------------------------------------------------------- tables
  py::class_<DenseTable, std::shared_ptr<DenseTable>>(m, "DenseTable")
      .def_readonly("rows", &DenseTable::rows)
      .def_readonly("cols", &DenseTable::cols)
      .def_readonly("ld", &DenseTable::ld)
      .def_readonly("global_offset", &DenseTable::global_offset)
      .def_readonly("global_rows", &DenseTable::global_rows)
      .def_property_readonly("dtype",
                             [](DenseTable& t) { return std::string(dtype_name(t.dtype)); })
      .def_property_readonly("nbytes", &DenseTable::bytes)
      .def_property_readonly("on_gpu", [](DenseTable& t) { return t.backend == Backend::GPU; })
      .def("to_numpy",
           [](DenseTable& t, std::shared_ptr<Context> ctx, int64_t r0, int64_t n) {
             if (n < 0) n = t.rows - r0;
             std::vector<double> v;
             {
               py::gil_scoped_release r;
               v = table_rows_f64(*ctx, t, r0, n);
             }
             py::array_t<double> out({n, int64_t(t.cols)});
             if (!v.empty()) std::memcpy(out.mutable_data(), v.data(), v.size() * 8);
             return out;
           },
           py::arg("ctx"), py::arg("start") = 0, py::arg("count") = -1)
      .def("download_f32",
           [](DenseTable& t, std::shared_ptr<Context> ctx) {
             // an f32 table's rows as a dense (rows, cols) float32 array (one pitched copy)
             OAP_CHECK(t.dtype == DType::F32, "download_f32 needs an f32 table");
             py::array_t<float> out({t.rows, int64_t(t.cols)});
             float* dst = out.mutable_data();
             {
               py::gil_scoped_release r;
               if (t.rows > 0 && ctx->is_gpu()) {
                 ctx->activate();
                 OAP_HIP_CHECK(hipMemcpy2D(dst, size_t(t.cols) * 4, t.data.data(), size_t(t.ld) * 4,
                                           size_t(t.cols) * 4, size_t(t.rows),
                                           hipMemcpyDeviceToHost));
               } else {
                 for (int64_t i = 0; i < t.rows; ++i)
                   std::memcpy(dst + size_t(i) * t.cols, t.data.as<float>() + size_t(i) * t.ld,
                               size_t(t.cols) * 4);
               }
             }
             return out;
           },
           py::arg("ctx"))
      .def("set_global", [](DenseTable& t, int64_t off, int64_t tot) {
        t.global_offset = off;
        t.global_rows = tot;
      });

  m.def(
      "table_view",
      [](std::shared_ptr<Context> ctx, uintptr_t ptr, int64_t rows, int cols, int64_t ld,
         const std::string& dtype) {
        // Zero-copy view of memory owned elsewhere (a torch tensor's storage, ptr =
        // tensor.data_ptr()); the caller keeps the owner alive while the view is used.
        const DType dt = parse_dtype(dtype);
        OAP_CHECK(rows >= 0 && cols > 0 && ld >= cols, "bad view shape");
        OAP_CHECK(ptr != 0 || rows == 0, "null view pointer");
        OAP_CHECK(ptr % 16 == 0, "view rows must be 16-byte aligned");
        auto t = std::make_shared<DenseTable>();
        t->rows = rows;
        t->cols = cols;
        t->ld = ld;
        t->dtype = dt;
        t->backend = ctx->backend();
        t->data = Buffer::view(reinterpret_cast<void*>(ptr), size_t(rows) * ld * dtype_size(dt));
        return t;
      },
      py::arg("ctx"), py::arg("ptr"), py::arg("rows"), py::arg("cols"), py::arg("ld"),
      py::arg("dtype") = "f32");
  m.def(
      "kmeans_predict_device",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<DenseTable> t, py::array_t<double> centers,
         uintptr_t labels_ptr, uintptr_t dist_ptr) {
        auto c = py::array_t<double, py::array::c_style | py::array::forcecast>(centers);
        if (c.ndim() != 2 || c.shape(1) != t->cols)
          throw ConfigError("centers must be k x d with d == table cols");
        std::vector<double> cv(c.data(), c.data() + c.size());
        const int k = static_cast<int>(c.shape(0));
        py::gil_scoped_release rel;
        kmeans_predict_device(*ctx, *t, cv, k, reinterpret_cast<int32_t*>(labels_ptr),
                              reinterpret_cast<float*>(dist_ptr));
      },
      py::arg("ctx"), py::arg("table"), py::arg("centers"), py::arg("labels_ptr"),
      py::arg("dist_ptr"));
  m.def(
      "upload_dense",
      [](std::shared_ptr<Context> ctx, py::array arr, const std::string& storage, int64_t ld) {
        py::buffer_info bi = arr.request();
        if (bi.ndim != 2) throw ConfigError("upload_dense expects a 2-D array");
        DType src;
        if (bi.format == py::format_descriptor<double>::format()) src = DType::F64;
        else if (bi.format == py::format_descriptor<float>::format()) src = DType::F32;
        else throw ConfigError("upload_dense: array must be float32 or float64");
        int64_t rows = bi.shape[0], cols = bi.shape[1];
        size_t es = static_cast<size_t>(bi.itemsize);
        if (bi.strides[1] != static_cast<py::ssize_t>(es) ||
            bi.strides[0] % static_cast<py::ssize_t>(es) != 0)
          throw ConfigError("upload_dense: array must be row-major (C-contiguous rows)");
        int64_t src_ld = bi.strides[0] / static_cast<int64_t>(es);
        if (ld <= 0) ld = cols;
        DType st = parse_dtype(storage);
        auto t = std::make_shared<DenseTable>();
        {
          py::gil_scoped_release r;
          *t = upload_dense(*ctx, bi.ptr, src, rows, static_cast<int>(cols), src_ld, st, ld);
        }
        return t;
      },
      py::arg("ctx"), py::arg("array"), py::arg("storage") = "f32", py::arg("ld") = 0);
  m.def(
      "synth_blobs",
      [](std::shared_ptr<Context> ctx, int64_t rows, int cols, int64_t ld, int64_t row0,
         int ncenters, double box, double sigma, uint64_t seed, const std::string& storage) {
        auto t = std::make_shared<DenseTable>();
        const DType st = parse_dtype(storage);
        py::gil_scoped_release r;
        *t = synth_blobs_table(*ctx, rows, cols, ld <= 0 ? cols : ld, row0, ncenters, box, sigma,
                               seed, st);
        return t;
      },
      py::arg("ctx"), py::arg("rows"), py::arg("cols"), py::arg("ld") = 0, py::arg("row0") = 0,
      py::arg("ncenters") = 8, py::arg("box") = 10.0, py::arg("sigma") = 1.0,
      py::arg("seed") = 42, py::arg("storage") = "f32");
  m.def("assign_global_offsets",
        [](std::shared_ptr<Context> ctx, std::shared_ptr<Comm> comm,
           std::shared_ptr<DenseTable> t) {
          py::gil_scoped_release r;
          assign_global_offsets(*ctx, *comm, *t);
        });

  // ---------------------------------------------------------------- K-Means
  m.def(
      "kmeans_ld",
      [](int d, const std::string& dtype) { return kern::kmeans_ld(d, dtype == "bf16"); },
      py::arg("d"), py::arg("dtype") = "f32");
  m.def(
      "kmeans_lds_kmax", [](int d, bool precise) { return kern::kmeans_lds_kmax(d, precise); },
      py::arg("d"), py::arg("precise") = false,
      "largest k whose centroid plane one LDS plan holds (larger k: chunked passes)");
  m.def(
      "kmeans_fit",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<Comm> comm, std::shared_ptr<DenseTable> t,
         py::object init_centers, int k, int max_iter, double tol, const std::string& init_mode,
         int init_steps, uint64_t seed, bool precise, bool prune, bool delta,
         bool phase_events, double scan_min_prune) {
        KMeansParams p;
        p.scan_min_prune = scan_min_prune;
        p.precise = precise;
        p.prune = prune;
        p.delta = delta;
        p.phase_events = phase_events;
        p.k = k;
        p.max_iter = max_iter;
        p.tol = tol;
        p.init_steps = init_steps;
        p.seed = seed;
        std::vector<double> init;
        if (!init_centers.is_none()) {
          auto a = py::array_t<double, py::array::c_style | py::array::forcecast>(init_centers);
          init.assign(a.data(), a.data() + a.size());
          p.init = KMeansInit::Given;
        } else if (init_mode == "random") {
          p.init = KMeansInit::Random;
        } else if (init_mode == "k-means||") {
          p.init = KMeansInit::Parallel;
        } else {
          throw ConfigError("unknown initMode '" + init_mode + "'");
        }
        KMeansResult r;
        {
          py::gil_scoped_release rel;
          r = kmeans_fit(*ctx, *comm, *t, init, p);
        }
        py::dict out;
        py::array_t<double> c({int64_t(r.k), int64_t(r.d)});
        if (!r.centers.empty())
          std::memcpy(c.mutable_data(), r.centers.data(), r.centers.size() * 8);
        out["centers"] = c;
        out["cost"] = r.cost;
        out["num_iter"] = r.num_iter;
        out["converged"] = r.converged;
        out["cost_history"] = r.cost_history;
        out["shift_history"] = r.shift_history;
        out["last_counts"] = r.last_counts;
        out["init_seconds"] = r.init_seconds;
        out["iter_seconds"] = r.iter_seconds;
        out["global_rows"] = r.global_rows;
        out["refine_tiles"] = r.refine_tiles;
        out["tier3_tiles"] = r.tier3_tiles;
        out["pruned_tiles"] = r.pruned_tiles;
        out["assign_path"] = r.assign_path;
        out["deferred_rows"] = r.deferred_rows;
        out["moved_rows"] = r.moved_rows;
        out["image_passes"] = r.image_passes;
        out["pruned_rows"] = r.pruned_rows;
        out["image_bytes"] = r.image_bytes;
        out["final_cost_path"] = r.final_cost_path;
        out["scale_source"] = r.scale_source;
        return out;
      },
      py::arg("ctx"), py::arg("comm"), py::arg("table"), py::arg("init_centers") = py::none(),
      py::arg("k") = 2, py::arg("max_iter") = 20, py::arg("tol") = 1e-4,
      py::arg("init_mode") = "k-means||", py::arg("init_steps") = 2, py::arg("seed") = 1,
      py::arg("precise") = false, py::arg("prune") = true, py::arg("delta") = true,
      py::arg("phase_events") = false, py::arg("scan_min_prune") = 0.2);
  m.def(
      "kmeans_fit_streamed",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<Comm> comm,
         py::array_t<float, py::array::c_style | py::array::forcecast> x, py::object init_centers,
         int max_iter, double tol, int64_t chunk_rows, bool precise) {
        if (x.ndim() != 2) throw ConfigError("kmeans_fit_streamed expects a 2-D array");
        auto a = py::array_t<double, py::array::c_style | py::array::forcecast>(init_centers);
        std::vector<double> init(a.data(), a.data() + a.size());
        KMeansParams p;
        p.precise = precise;
        p.max_iter = max_iter;
        p.tol = tol;
        p.init = KMeansInit::Given;
        p.k = static_cast<int>(init.size() / std::max<int64_t>(x.shape(1), 1));
        KMeansResult r;
        {
          py::gil_scoped_release rel;
          r = kmeans_fit_streamed(*ctx, *comm, x.data(), x.shape(0), static_cast<int>(x.shape(1)),
                                  init, p, chunk_rows);
        }
        py::dict out;
        py::array_t<double> c({int64_t(r.k), int64_t(r.d)});
        if (!r.centers.empty())
          std::memcpy(c.mutable_data(), r.centers.data(), r.centers.size() * 8);
        out["centers"] = c;
        out["cost"] = r.cost;
        out["num_iter"] = r.num_iter;
        out["converged"] = r.converged;
        out["cost_history"] = r.cost_history;
        out["shift_history"] = r.shift_history;
        out["last_counts"] = r.last_counts;
        out["iter_seconds"] = r.iter_seconds;
        out["global_rows"] = r.global_rows;
        return out;
      },
      py::arg("ctx"), py::arg("comm"), py::arg("x"), py::arg("init_centers"),
      py::arg("max_iter") = 20, py::arg("tol") = 1e-4, py::arg("chunk_rows") = 1 << 22,
      py::arg("precise") = false,
      "Out-of-core K-Means: host rows streamed through HBM chunk buffers every iteration.");
  m.def(
      "kmeans_init",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<Comm> comm, std::shared_ptr<DenseTable> t,
         int k, const std::string& init_mode, int init_steps, uint64_t seed) {
        KMeansParams p;
        p.k = k;
        p.init_steps = init_steps;
        p.seed = seed;
        p.init = init_mode == "random" ? KMeansInit::Random : KMeansInit::Parallel;
        int keff = 0;
        std::vector<double> c;
        {
          py::gil_scoped_release rel;
          c = kmeans_init_centers(*ctx, *comm, *t, p, &keff);
        }
        py::array_t<double> out({int64_t(keff), int64_t(t->cols)});
        if (!c.empty()) std::memcpy(out.mutable_data(), c.data(), c.size() * 8);
        return out;
      },
      py::arg("ctx"), py::arg("comm"), py::arg("table"), py::arg("k"),
      py::arg("init_mode") = "k-means||", py::arg("init_steps") = 2, py::arg("seed") = 1);
  m.def(
      "kmeans_predict",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<DenseTable> t, py::array_t<double> centers) {
        auto c = py::array_t<double, py::array::c_style | py::array::forcecast>(centers);
        if (c.ndim() != 2 || c.shape(1) != t->cols)
          throw ConfigError("centers must be k x d with d == table cols");
        int k = static_cast<int>(c.shape(0));
        std::vector<double> cv(c.data(), c.data() + c.size());
        py::array_t<int32_t> labels(t->rows);
        py::array_t<double> dist(t->rows);
        int32_t* lp = labels.mutable_data();
        double* dp = dist.mutable_data();
        {
          py::gil_scoped_release rel;
          kmeans_predict(*ctx, *t, cv, k, lp, dp);
        }
        return py::make_tuple(labels, dist);
      });
  // The estimator's summary pass (KMeans.scala:359-368, model.transform + clusterSizes): labels
  // of the rows of an already-resident table (no re-upload, no per-row distances copied back)
  // and the per-cluster counts, counted on the host pool.
  m.def(
      "kmeans_labels",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<DenseTable> t, py::array_t<double> centers) {
        auto c = py::array_t<double, py::array::c_style | py::array::forcecast>(centers);
        if (c.ndim() != 2 || c.shape(1) != t->cols)
          throw ConfigError("centers must be k x d with d == table cols");
        const int k = static_cast<int>(c.shape(0));
        std::vector<double> cv(c.data(), c.data() + c.size());
        py::array_t<int32_t> labels(t->rows);
        py::array_t<int64_t> counts(k);
        int32_t* lp = labels.mutable_data();
        int64_t* cp = counts.mutable_data();
        {
          py::gil_scoped_release rel;
          kmeans_predict(*ctx, *t, cv, k, lp, nullptr);
          const int nt = ctx->pool().size();
          std::vector<std::vector<int64_t>> part(nt);
          ctx->pool().parallel_for(t->rows, [&](int ci, int64_t b, int64_t e) {
            std::vector<int64_t>& h = part[ci];
            h.assign(size_t(k), 0);
            for (int64_t i = b; i < e; ++i)
              if (lp[i] >= 0 && lp[i] < k) ++h[size_t(lp[i])];
          });
          std::fill(cp, cp + k, int64_t(0));
          for (const auto& h : part)
            for (size_t j = 0; j < h.size(); ++j) cp[j] += h[j];
        }
        return py::make_tuple(labels, counts);
      },
      py::arg("ctx"), py::arg("table"), py::arg("centers"));
  m.def("kmeans_set_lean_variant", &kmeans_set_lean_variant);
  m.def("kmeans_last_timing_deferred", []() { return last_timing_deferred(); });
  m.def(
      "kmeans_image_timing",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<DenseTable> t, py::array_t<double> ca,
         py::array_t<double> cb, int reps, int kernel, int cfg, bool fallback) {
        auto a = py::array_t<double, py::array::c_style | py::array::forcecast>(ca);
        auto b = py::array_t<double, py::array::c_style | py::array::forcecast>(cb);
        OAP_CHECK(a.ndim() == 2 && b.ndim() == 2 && a.shape(0) == b.shape(0) &&
                      a.shape(1) == b.shape(1) && a.shape(1) == t->cols,
                  "kmeans_image_timing: centers must both be [k][d]");
        std::vector<double> av(a.data(), a.data() + a.size()), bv(b.data(), b.data() + b.size());
        const int k = static_cast<int>(a.shape(0));
        ImageTiming r;
        {
          py::gil_scoped_release rel;
          r = kmeans_image_timing(*ctx, *t, av, bv, k, reps, kernel, cfg, fallback);
        }
        py::dict out;
        out["lean_ms"] = r.lean_ms;
        out["pass_ms"] = r.pass_ms;
        out["deferred_rows"] = r.deferred_rows;
        out["moved_rows"] = r.moved_rows;
        out["image_passes"] = r.image_passes;
        out["path"] = r.path;
        py::array_t<int32_t> lab(static_cast<py::ssize_t>(r.labels.size()));
        std::memcpy(lab.mutable_data(), r.labels.data(), r.labels.size() * 4);
        py::array_t<uint64_t> st(static_cast<py::ssize_t>(r.stats.size()));
        std::memcpy(st.mutable_data(), r.stats.data(), r.stats.size() * 8);
        out["labels"] = lab;
        out["stats"] = st;
        return out;
      },
      py::arg("ctx"), py::arg("table"), py::arg("centers_a"), py::arg("centers_b"),
      py::arg("reps") = 5, py::arg("kernel") = 1, py::arg("cfg") = -1, py::arg("fallback") = true);
  m.def(
      "kmeans_assign_timing",
      [](std::shared_ptr<Context> ctx, std::shared_ptr<DenseTable> t, py::array_t<double> centers,
         int reps, bool precise, int ablate) {
        auto c = py::array_t<double, py::array::c_style | py::array::forcecast>(centers);
        std::vector<double> cv(c.data(), c.data() + c.size());
        int k = static_cast<int>(c.shape(0));
        py::gil_scoped_release rel;
        return kmeans_assign_timing(*ctx, *t, cv, k, reps, precise, ablate);
      },
      py::arg("ctx"), py::arg("table"), py::arg("centers"), py::arg("reps") = 10,
      py::arg("precise") = false, py::arg("ablate") = 0);
  m.def("local_kmeans_pp",
        [](py::array_t<double> pts, py::array_t<double> w, int k, int max_iter, uint64_t seed) {
          auto p = py::array_t<double, py::array::c_style | py::array::forcecast>(pts);
          std::vector<double> pv(p.data(), p.data() + p.size()), wv(w.data(), w.data() + w.size());
          int d = static_cast<int>(p.shape(1));
          auto c = local_kmeans_pp(pv, wv, d, k, max_iter, seed);
          py::array_t<double> out({int64_t(k), int64_t(d)});
          std::memcpy(out.mutable_data(), c.data(), c.size() * 8);
          return out;
        });

  register_pca(m);
  register_als(m);
  register_io(m);
}
