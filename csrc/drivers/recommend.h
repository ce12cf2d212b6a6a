// recommendForAll* driver: fused score + top-k (kernels/als_recommend.hip) over slabs of the
// source factor rows, the destination factors packed once and resident in HBM.  The role of
// Spark's blocked recommendForAll (spark-3.1.1/mllib/src/main/scala/org/apache/spark/ml/
// recommendation/ALS.scala:365-505); no score matrix is ever stored, on the device or the host.
#pragma once

#include <cstdint>

#include "runtime/context.h"

namespace oap {

struct RecTiming {
  double pack_dst_s = 0, upload_s = 0, topk_s = 0, download_s = 0, wall_s = 0;
  int slabs = 0;
  int64_t slab_rows = 0;
};

// Top-`num` destination rows (index into dst, score) of every source row: out_idx / out_val
// [n_src][num].  src [n_src][rank], dst [n_dst][rank] fp32 host rows.  slab_rows <= 0: sized
// from the device's free memory.
void als_recommend(Context& ctx, const float* src, int64_t n_src, const float* dst,
                   int64_t n_dst, int rank, int num, int32_t* out_idx, float* out_val,
                   int64_t slab_rows, RecTiming* timing);
int als_recommend_max_num(int rank);

}  // namespace oap
