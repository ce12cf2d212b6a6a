// k-means|| helpers for candidate sets beyond one LDS plan (kernels/kmeans_init.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace oap {
namespace kern {

// Per row, keep the nearer of (best_dist, best_lab) and (dist, lab + base): strictly nearer
// only, so an earlier super-chunk (lower indices) wins ties.  first: initialise from (dist, lab).
void kmeans_merge_argmin(float* best_dist, int32_t* best_lab, const float* dist,
                         const int32_t* lab, int base, int64_t n, bool first, hipStream_t s);

}  // namespace kern
}  // namespace oap
