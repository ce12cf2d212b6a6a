#include "runtime/table.h"

#include <cmath>
#include <cstring>
#include <limits>

#include "kernels/kernels.h"

namespace oap {

namespace {
// CPU helpers ---------------------------------------------------------------------------
double read_elem(const void* p, DType t, size_t i) {
  switch (t) {
    case DType::F32: return static_cast<const float*>(p)[i];
    case DType::F64: return static_cast<const double*>(p)[i];
    default: OAP_THROW(ConfigError, "unsupported element type " << dtype_name(t));
  }
}
uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
float u01(uint64_t h) { return static_cast<float>(h >> 40) * (1.0f / 16777216.0f); }
// float -> nearest-even bf16 -> float (the device's __bf16 conversion for finite values)
float bf16_round(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  u &= 0xffff0000u;
  float o;
  std::memcpy(&o, &u, 4);
  return o;
}
}  // namespace

DenseTable upload_dense(Context& ctx, const void* host, DType src_t, int64_t rows, int cols,
                        int64_t src_ld, DType storage, int64_t ld, int64_t chunk_rows) {
  OAP_CHECK(src_t == DType::F32 || src_t == DType::F64, "source must be f32 or f64");
  OAP_CHECK(ld >= cols, "ld (" << ld << ") < cols (" << cols << ")");
  OAP_CHECK(rows >= 0 && cols > 0, "bad shape " << rows << "x" << cols);
  DenseTable t;
  t.rows = rows;
  t.cols = cols;
  t.ld = ld;
  t.dtype = storage;
  t.backend = ctx.backend();
  TraceRange tr(&ctx.metrics(), "ingest/upload_dense", int64_t(rows) * cols * dtype_size(src_t));
  if (!ctx.is_gpu()) {
    OAP_CHECK(storage == DType::F64 || storage == DType::F32,
              "CPU tables are f32 or f64, got " << dtype_name(storage));
    t.data = Buffer::host(t.bytes());
    ctx.pool().parallel_for(rows, [&](int, int64_t b, int64_t e) {
      for (int64_t r = b; r < e; ++r)
        for (int c = 0; c < ld; ++c) {
          double v = c < cols ? read_elem(host, src_t, size_t(r) * src_ld + c) : 0.0;
          if (storage == DType::F64)
            t.data.as<double>()[size_t(r) * ld + c] = v;
          else
            t.data.as<float>()[size_t(r) * ld + c] = static_cast<float>(v);
        }
    });
    return t;
  }
  // f64 device tables serve the exact (reference-precision) PCA statistics only; K-Means reads
  // f32 / bf16 rows (check_gpu_table)
  OAP_CHECK(storage == DType::F32 || storage == DType::BF16 || storage == DType::F64,
            "GPU tables are f32, bf16 or f64, got " << dtype_name(storage));
  ctx.activate();
  t.data = ctx.alloc(t.bytes() == 0 ? 256 : t.bytes());
  if (rows == 0) return t;
  // Double-buffered pipeline: host memcpy into pinned[i%2] -> H2D into staging[i%2] -> device
  // convert/pad into the final layout; the event on each slot protects it from being refilled
  // while its copy is still in flight.  The staging copy is split over the context's thread pool
  // (one host thread copies ~10-15 GB/s, a PCIe Gen5 x16 DMA runs ~50+ GB/s): the copy into slot
  // i ^ 1 runs while slot i's DMA is in flight, so the upload runs at the slower of the two.
  const size_t es = dtype_size(src_t);
  if (chunk_rows > rows) chunk_rows = rows;
  const size_t chunk_bytes = size_t(chunk_rows) * cols * es;
  Buffer pinned[2] = {ctx.alloc_pinned(chunk_bytes), ctx.alloc_pinned(chunk_bytes)};
  Buffer stage[2] = {ctx.alloc(chunk_bytes), ctx.alloc(chunk_bytes)};
  Event done[2];
  bool used[2] = {false, false};
  hipStream_t s = ctx.h2d();
  int slot = 0;
  for (int64_t r0 = 0; r0 < rows; r0 += chunk_rows, slot ^= 1) {
    int64_t n = std::min<int64_t>(chunk_rows, rows - r0);
    if (used[slot]) done[slot].sync();
    const char* src = static_cast<const char*>(host) + size_t(r0) * src_ld * es;
    char* dst = pinned[slot].as<char>();
    const size_t row_bytes = size_t(cols) * es;
    if (size_t(n) * row_bytes < (size_t(4) << 20)) {  // (small: one thread)
      if (src_ld == cols)
        std::memcpy(dst, src, size_t(n) * row_bytes);
      else
        for (int64_t r = 0; r < n; ++r)
          std::memcpy(dst + size_t(r) * row_bytes, src + size_t(r) * src_ld * es, row_bytes);
    } else {
      ctx.pool().parallel_for(n, [&](int, int64_t b, int64_t e) {
        if (src_ld == cols)
          std::memcpy(dst + size_t(b) * row_bytes, src + size_t(b) * row_bytes,
                      size_t(e - b) * row_bytes);
        else
          for (int64_t r = b; r < e; ++r)
            std::memcpy(dst + size_t(r) * row_bytes, src + size_t(r) * src_ld * es, row_bytes);
      });
    }
    OAP_HIP_CHECK(hipMemcpyAsync(stage[slot].data(), dst, size_t(n) * cols * es,
                                 hipMemcpyHostToDevice, s));
    char* out = t.data.as<char>() + size_t(r0) * ld * dtype_size(storage);
    kern::convert_pad(stage[slot].data(), src_t, n, cols, cols, out, storage, ld, s);
    done[slot].record(s);
    used[slot] = true;
  }
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  return t;
}

DenseTable synth_blobs_table(Context& ctx, int64_t rows, int cols, int64_t ld, int64_t row0,
                             int ncenters, double box, double sigma, uint64_t seed,
                             DType storage) {
  OAP_CHECK(storage == DType::F32 || storage == DType::BF16,
            "synth_blobs: storage must be f32 or bf16");
  DenseTable t;
  t.rows = rows;
  t.cols = cols;
  t.ld = ld;
  t.backend = ctx.backend();
  TraceRange tr(&ctx.metrics(), "ingest/synth_blobs", int64_t(rows) * ld * dtype_size(storage));
  if (ctx.is_gpu()) {
    t.dtype = storage;
    ctx.activate();
    t.data = ctx.alloc(t.bytes() == 0 ? 256 : t.bytes());
    kern::synth_blobs(t.data.data(), storage, rows, cols, ld, row0, ncenters, float(box),
                      float(sigma), seed, ctx.compute());
    OAP_HIP_CHECK(hipStreamSynchronize(ctx.compute()));
    return t;
  }
  // Same generator on the CPU, in float32 arithmetic, cast to f64 storage.
  t.dtype = DType::F64;
  t.data = Buffer::host(t.bytes());
  double* x = t.data.as<double>();
  ctx.pool().parallel_for(rows, [&](int, int64_t b, int64_t e) {
    for (int64_t r = b; r < e; ++r) {
      int64_t grow = row0 + r;
      uint64_t lab = splitmix64(seed ^ (uint64_t(grow) * 0x2545F4914F6CDD1Dull)) %
                     uint64_t(ncenters);
      for (int c = 0; c < ld; ++c) {
        if (c >= cols) {
          x[size_t(r) * ld + c] = 0.0;
          continue;
        }
        uint64_t hc = splitmix64(seed * 31ull + lab * 1315423911ull + uint64_t(c) * 2654435761ull);
        float center = (u01(hc) * 2.f - 1.f) * float(box);
        uint64_t h1 = splitmix64(seed ^ 0xABCDEFull ^ (uint64_t(grow) << 20) ^ uint64_t(c));
        uint64_t h2 = splitmix64(h1);
        float u1 = std::fmax(u01(h1), 1e-7f), u2 = u01(h2);
        float g = std::sqrt(-2.f * std::log(u1)) * std::cos(6.2831853f * u2);
        const float v = center + float(sigma) * g;
        x[size_t(r) * ld + c] = storage == DType::BF16 ? double(bf16_round(v)) : double(v);
      }
    }
  });
  return t;
}

void assign_global_offsets(Context& ctx, Comm& comm, DenseTable& t) {
  auto counts = comm_allgather_i64(ctx, comm, t.rows);
  int64_t off = 0, tot = 0;
  for (int r = 0; r < comm.size(); ++r) {
    if (r < comm.rank()) off += counts[r];
    tot += counts[r];
  }
  t.global_offset = off;
  t.global_rows = tot;
}

std::vector<double> global_column_absmax(Context& ctx, Comm& comm, DenseTable& t) {
  std::vector<double> mx(t.cols, 0.0);
  if (ctx.is_gpu()) {
    Buffer d = ctx.alloc(sizeof(float) * t.cols);
    ctx.memset(d.data(), 0, sizeof(float) * t.cols);
    kern::column_absmax(t.data.data(), t.dtype, t.rows, t.cols, t.ld, d.as<float>(),
                        ctx.compute());
    std::vector<float> h(t.cols);
    ctx.copy_to_host(h.data(), d.data(), sizeof(float) * t.cols);
    for (int c = 0; c < t.cols; ++c) mx[c] = h[c];
  } else {
    std::vector<std::vector<double>> part(ctx.pool().size(), std::vector<double>(t.cols, 0.0));
    ctx.pool().parallel_for(t.rows, [&](int ci, int64_t b, int64_t e) {
      auto& p = part[ci];
      for (int64_t r = b; r < e; ++r)
        for (int c = 0; c < t.cols; ++c) {
          double v = t.dtype == DType::F64 ? t.data.as<double>()[size_t(r) * t.ld + c]
                                           : t.data.as<float>()[size_t(r) * t.ld + c];
          p[c] = std::max(p[c], std::fabs(v));
        }
    });
    for (auto& p : part)
      for (int c = 0; c < t.cols; ++c) mx[c] = std::max(mx[c], p[c]);
  }
  if (!comm.trivial()) {
    if (comm.on_device() && ctx.is_gpu()) {
      Buffer d = ctx.alloc(sizeof(double) * t.cols);
      ctx.copy_to_backend(d.data(), mx.data(), sizeof(double) * t.cols, ctx.comm_stream());
      comm.allreduce(d.data(), t.cols, DType::F64, ReduceOp::Max, ctx.comm_stream());
      OAP_HIP_CHECK(hipMemcpyAsync(mx.data(), d.data(), sizeof(double) * t.cols,
                                   hipMemcpyDeviceToHost, ctx.comm_stream()));
      comm.wait(ctx.comm_stream());
    } else {
      comm.allreduce(mx.data(), t.cols, DType::F64, ReduceOp::Max, nullptr);
    }
  }
  return mx;
}

double local_row_sqnorm(Context& ctx, DenseTable& t, double* rel_err) {
  *rel_err = 0.0;
  if (t.rows == 0) return 0.0;
  if (!ctx.is_gpu() || t.dtype != DType::F32) return std::numeric_limits<double>::quiet_NaN();
  Buffer part = ctx.alloc(sizeof(double) * kern::kSqnormBlocks);
  const int nb = kern::row_sqnorm_partials(t.data.as<float>(), t.rows, t.cols, t.ld,
                                           part.as<double>(), ctx.compute());
  if (nb < 0) return std::numeric_limits<double>::quiet_NaN();
  std::vector<double> h(nb);
  ctx.copy_to_host(h.data(), part.data(), sizeof(double) * nb);
  double sum = 0.0;
  for (double v : h) sum += v;
  // longest addition chain of any square: its thread's loop (one add per row group, 3 inside
  // the 4-term expression), 6 shuffle levels, 2 in the block, nb on the host; each add of
  // non-negative terms errs by at most u of the running (<= final) sum
  const int64_t per_block = (256 / (t.ld / 4)) * (t.ld / 4);
  const int64_t rstride = int64_t(nb) * (per_block / (t.ld / 4));
  const double chain = double((t.rows + rstride - 1) / rstride + 3 + 6 + 2 + nb);
  *rel_err = chain * 1.12e-16;
  return sum;
}

std::vector<double> table_rows_f64(Context& ctx, const DenseTable& t, int64_t r0, int64_t n) {
  OAP_CHECK(r0 >= 0 && r0 + n <= t.rows, "row range out of bounds");
  std::vector<double> out(size_t(n) * t.cols);
  size_t es = dtype_size(t.dtype);
  std::vector<char> raw(size_t(n) * t.ld * es);
  if (n == 0) return out;
  ctx.copy_to_host(raw.data(), t.data.as<char>() + size_t(r0) * t.ld * es, raw.size());
  for (int64_t r = 0; r < n; ++r)
    for (int c = 0; c < t.cols; ++c) {
      size_t i = size_t(r) * t.ld + c;
      double v;
      if (t.dtype == DType::F64)
        v = reinterpret_cast<double*>(raw.data())[i];
      else if (t.dtype == DType::F32)
        v = reinterpret_cast<float*>(raw.data())[i];
      else {
        uint16_t b = reinterpret_cast<uint16_t*>(raw.data())[i];
        uint32_t u = uint32_t(b) << 16;
        float f;
        std::memcpy(&f, &u, 4);
        v = f;
      }
      out[size_t(r) * t.cols + c] = v;
    }
  return out;
}

}  // namespace oap
