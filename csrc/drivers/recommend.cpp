// recommendForAll* driver (see recommend.h).
#include "drivers/recommend.h"

#include <algorithm>
#include <chrono>

#include "kernels/als_recommend.h"
#include "runtime/common.h"

namespace oap {

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

int als_recommend_max_num(int rank) {
  return std::max(kern::rec_max_num(rank), kern::rec_big_max_num(rank));
}

void als_recommend(Context& ctx, const float* src, int64_t n_src, const float* dst,
                   int64_t n_dst, int rank, int num, int32_t* out_idx, float* out_val,
                   int64_t slab_rows, RecTiming* timing) {
  OAP_CHECK(ctx.is_gpu(), "als_recommend needs a GPU context");
  OAP_CHECK(rank >= 1 && num >= 1 && num <= als_recommend_max_num(rank) && n_dst >= 1,
            "als_recommend: rank 1..256, num 1.." << als_recommend_max_num(rank));
  const bool big = num > kern::rec_max_num(rank);  // (lists in HBM: rec_topk_big)
  RecTiming t;
  const double w0 = now_s();
  ctx.activate();
  hipStream_t s = ctx.compute();
  const size_t rs = size_t(kern::rec_row_slots(rank)) * 16;  // packed row bytes
  // destinations: fp32 upload, max |x|, packed image (rows padded to the 64-row block)
  Buffer amax = ctx.alloc(2 * sizeof(unsigned));
  ctx.memset(amax.data(), 0, 2 * sizeof(unsigned), s);
  const int64_t dpad = (n_dst + 63) / 64 * 64;
  Buffer dimg = ctx.alloc(size_t(dpad) * rs);
  {
    Buffer d32 = ctx.alloc(size_t(n_dst) * rank * 4);
    ctx.copy_to_backend(d32.data(), dst, size_t(n_dst) * rank * 4, s);
    kern::rec_absmax(d32.as<float>(), n_dst, rank, rank, amax.as<unsigned>() + 1, s);
    kern::rec_pack(d32.as<float>(), n_dst, rank, rank, amax.as<unsigned>() + 1, nullptr,
                   dimg.data(), dpad, s);
    OAP_HIP_CHECK(hipStreamSynchronize(s));
  }
  t.pack_dst_s = now_s() - w0;
  // source slabs: fp32 rows + packed image + outputs per slab, sized to a quarter of the
  // arena's remaining budget (whole launches: multiples of the kernel's row granule)
  const int64_t gran = int64_t(kern::rec_src_granule(rank, num));
  const size_t per_row = size_t(rank) * 4 + rs + size_t(num) * 8 + 4;
  if (slab_rows <= 0) {
    DeviceArena* ar = ctx.arena();
    const size_t room =
        ar ? (ar->budget() - std::min(ar->budget(), ar->used())) / 4 : size_t(1) << 30;
    slab_rows = int64_t(std::max<size_t>(room / per_row, size_t(gran)));
  }
  slab_rows =
      std::max<int64_t>(gran, std::min<int64_t>(slab_rows, (n_src + gran - 1) / gran * gran));
  slab_rows = slab_rows / gran * gran;
  t.slab_rows = slab_rows;
  Buffer s32 = ctx.alloc(size_t(slab_rows) * rank * 4);
  Buffer simg = ctx.alloc(size_t(slab_rows) * rs);
  Buffer oidx = ctx.alloc(size_t(slab_rows) * num * 4);
  Buffer oval = ctx.alloc(size_t(slab_rows) * num * 4);
  Buffer sexp = ctx.alloc(size_t(slab_rows) * 4);
  // big num: candidate buffers for 512 workgroups per launch (the kernel chunks the grid; at
  // most 2 of its workgroups fit a CU's LDS, so 512 fill the chip), at most the slab's own
  // (4 MiB per workgroup at the largest cap: 2 GiB)
  Buffer cand;
  size_t cand_bytes = 0;
  if (big) {
    const int64_t wgs = std::min<int64_t>(512, (slab_rows + gran - 1) / gran);
    cand_bytes = size_t(wgs) * kern::rec_big_scratch_per_wg(num);
    cand = ctx.alloc(cand_bytes);
  }
  for (int64_t r0 = 0; r0 < n_src; r0 += slab_rows) {
    const int64_t rows = std::min(slab_rows, n_src - r0);
    const int64_t rpad = (rows + gran - 1) / gran * gran;
    double a0 = now_s();
    ctx.copy_to_backend(s32.data(), src + r0 * rank, size_t(rows) * rank * 4, s);
    kern::rec_row_exp(s32.as<float>(), rows, rank, rank, sexp.as<int32_t>(), s);
    kern::rec_pack(s32.as<float>(), rows, rank, rank, nullptr, sexp.as<int32_t>(), simg.data(),
                   rpad, s);
    OAP_HIP_CHECK(hipStreamSynchronize(s));
    double a1 = now_s();
    if (big)
      kern::rec_topk_big(simg.data(), sexp.as<int32_t>(), rows, dimg.data(),
                         amax.as<unsigned>() + 1, n_dst, rank, num, oidx.as<int32_t>(),
                         oval.as<float>(), cand.data(), cand_bytes, s);
    else
      kern::rec_topk(simg.data(), sexp.as<int32_t>(), rows, dimg.data(), amax.as<unsigned>() + 1,
                     n_dst, rank, num, oidx.as<int32_t>(), oval.as<float>(), s);
    OAP_HIP_CHECK(hipStreamSynchronize(s));
    double a2 = now_s();
    ctx.copy_to_host(out_idx + r0 * num, oidx.data(), size_t(rows) * num * 4, s);
    ctx.copy_to_host(out_val + r0 * num, oval.data(), size_t(rows) * num * 4, s);
    double a3 = now_s();
    t.upload_s += a1 - a0;
    t.topk_s += a2 - a1;
    t.download_s += a3 - a2;
    ++t.slabs;
  }
  t.wall_s = now_s() - w0;
  if (timing) *timing = t;
}

}  // namespace oap
