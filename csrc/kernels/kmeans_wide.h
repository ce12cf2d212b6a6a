// K-Means assignment for wide rows (d > 128) on the matrix cores (kernels/kmeans_wide.hip): the
// lean kernel's fp16 tier-1 distance with its rigorous error bound, looping over 128-feature
// chunks with the centroid chunk staged in LDS; rows inside the bound are re-decided by the
// exact fp32 direct form (the generic kernel's arithmetic) — so the labels equal the generic
// kernel's.  Accumulation then runs label-driven (kmeans_accumulate).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels/kernels.h"

namespace oap {
namespace kern {

// d > 128 (up to 4096) and k <= 256 in one pass.
bool kmeans_wide_supported(int d, int k);

// Labels of a.n rows (a.x, a.ld, a.d, a.xbf16; a.centers [kpad][dp], a.cnorm, a.cstat, a.k,
// a.kpad; a.labels).  Deferred rows go to `defer` (capacity a.n) counted by *defer_count (zeroed
// by the call; left on the device) and are resolved by the exact pass in the same call.
void kmeans_wide_assign(const KMeansAssignArgs& a, int num_cus, int32_t* defer,
                        unsigned* defer_count, hipStream_t s);

// Per-row fp32 cost against the labelled centers (direct form), one fp64 partial per block into
// slab (returns the number of partials); mindist (optional) gets the per-row cost.
int kmeans_wide_cost(const KMeansAssignArgs& a, double* slab, int max_blocks, hipStream_t s);

}  // namespace kern
}  // namespace oap
