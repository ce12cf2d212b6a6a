// Internal interface between the K-Means kernel translation units.
#pragma once

#include "kernels/kernels.h"

namespace oap {
namespace kern {

constexpr int kAssignThreads = 512;  // 8 waves: 2 per SIMD with one workgroup per CU
constexpr size_t kLdsLimit = 160 * 1024;
// Deferral sub-segments per workgroup (one per wave of the lean kernel; count stride)
constexpr int kDeferSubs = 16;
// Exact-list sub-segments per workgroup (one per wave of the general kernel)
constexpr int kExactSubs = kAssignThreads / 64;

// Launches the MFMA assign kernel (d <= 128, centroids fit the LDS plan).  `grid` blocks.
void launch_kmeans_assign_mfma(const KMeansAssignArgs& a, int grid, hipStream_t s);
// mindist/labels of the chunked path seeded from labels (the previous assignment).
void launch_kmeans_seed_mindist(const KMeansAssignArgs& a, hipStream_t s);
// -1 when the k centers do not fit LDS, else the number of fp64 partials written to slab
int launch_kmeans_label_cost(const KMeansAssignArgs& a, double* slab, int max_blocks,
                             hipStream_t s);
// Largest kpad (multiple of 32) whose centroid planes fit LDS for d features.
int kmeans_mfma_kmax(int d, bool precise);
// Grid the MFMA assign kernel uses for n rows (>= 256 blocks once there is work for them, so the
// per-block row bound used by the fixed-point scale is device independent).
int kmeans_mfma_grid(int64_t n, int num_cus);

}  // namespace kern
}  // namespace oap
