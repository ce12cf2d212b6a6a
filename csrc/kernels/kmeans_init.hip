// k-means|| over candidate sets beyond one LDS plan (config 5: ~2000 candidates per round and
// ~4000 counted): the driver runs the centroid-chunked lean pass on super-chunks of at most 1024
// candidates (its keys carry 10-bit indices) and merges the per-row exact answers here — the
// nearer exact fp32 distance wins, the earlier super-chunk on ties, i.e. the single pass's
// lowest-index argmin.
#include "kernels/kmeans_init.h"

#include "runtime/common.h"

namespace oap {
namespace kern {

namespace {

__global__ void oap_kmeans_merge_argmin(float* __restrict__ best_dist,
                                        int32_t* __restrict__ best_lab,
                                        const float* __restrict__ dist,
                                        const int32_t* __restrict__ lab, int base, int64_t n,
                                        int first) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float d = dist[i];
    if (first || d < best_dist[i]) {
      best_dist[i] = d;
      best_lab[i] = lab[i] + base;
    }
  }
}

}  // namespace

void kmeans_merge_argmin(float* best_dist, int32_t* best_lab, const float* dist,
                         const int32_t* lab, int base, int64_t n, bool first, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(oap_kmeans_merge_argmin, dim3(unsigned(blocks < 8192 ? blocks : 8192)),
                     dim3(256), 0, s, best_dist, best_lab, dist, lab, base, n, first ? 1 : 0);
  OAP_HIP_CHECK(hipGetLastError());
}

}  // namespace kern
}  // namespace oap
