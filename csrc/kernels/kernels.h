// Host-side launch API for every hand-written CDNA4 (gfx950) kernel.  Kernel names are chosen
// to be greppable in `rocprofv3 --kernel-trace` output (prefix "oap_").
#pragma once

#include <cstdint>

#include "runtime/common.h"

namespace oap {
namespace kern {

// ----------------------------------------------------------------------------- data layout
// Row stride (elements) the MFMA K-Means kernels expect for d features (zero padded).
int kmeans_ld(int d);
// Dense ingestion: src rows (f64 or f32, row stride src_ld) -> dst rows (f32 or bf16, row
// stride dst_ld, zero padded).  Both pointers are device pointers.
void convert_pad(const void* src, DType src_t, int64_t rows, int cols, int64_t src_ld, void* dst,
                 DType dst_t, int64_t dst_ld, hipStream_t s);
// Per-column max |x| over rows (atomicMax on the float bit pattern), out[cols] must be zeroed.
void column_absmax(const float* x, int64_t rows, int cols, int64_t ld, float* out, hipStream_t s);
// Deterministic synthetic Gaussian-blob generator (Philox-style hash), rows [row0, row0+rows)
// of a global dataset: x = center[label] + sigma * N(0,1); centers uniform in [-box, box].
void synth_blobs(float* x, int64_t rows, int cols, int64_t ld, int64_t row0, int ncenters,
                 float box, float sigma, uint64_t seed, hipStream_t s);

// ----------------------------------------------------------------------------- K-Means
struct KMeansAssignArgs {
  const float* x = nullptr;  // [n][ld] f32, ld = kmeans_ld(d)
  int64_t n = 0;
  int ld = 0;
  int d = 0;
  const float* centers = nullptr;  // [k][d] f32
  const float* cnorm = nullptr;    // [kpad] f32, +inf for j >= k
  int k = 0;
  int kpad = 0;                      // multiple of 32
  const float* scale = nullptr;      // [d] fixed-point scales (powers of two)
  unsigned long long* sums = nullptr;    // [k][d] int64 fixed point (accumulate)
  unsigned long long* counts = nullptr;  // [k]
  double* cost_slab = nullptr;           // [grid] per-block cost (deterministic)
  const float* weights = nullptr;        // optional [n] instance weights (nullptr => 1)
  int32_t* labels = nullptr;             // optional [n]
  float* mindist = nullptr;              // optional [n] exact squared distance to best center
  bool accumulate = true;     // accumulate counts (+ sums when `sums_too`)
  bool sums_too = true;
};
// Returns the number of blocks used (== entries written to cost_slab).
int kmeans_assign(const KMeansAssignArgs& a, int num_cus, hipStream_t s);
int kmeans_cost_slab_size(int num_cus);

struct KMeansFinalizeArgs {
  const unsigned long long* sums = nullptr;  // global (allreduced) fixed-point sums [k][d]
  const unsigned long long* counts = nullptr;
  const double* inv_scale = nullptr;  // [d]
  double* centers64 = nullptr;        // [k][d] in/out (empty clusters keep their center)
  float* centers32 = nullptr;         // [k][d] out
  float* cnorm = nullptr;             // [kpad] out (entries >= k untouched)
  int k = 0;
  int d = 0;
  double tol = 0.0;
  const double* cost_in = nullptr;  // allreduced cost (1 value)
  void* flags = nullptr;            // KMeansFlags out
};
struct KMeansFlags {
  int converged;
  int nonempty;
  double cost;
  double max_shift2;
};
void kmeans_finalize(const KMeansFinalizeArgs& a, hipStream_t s);
// Sums cost_slab[0..m) in a fixed order into out[0].
void sum_f64(const double* in, int m, double* out, hipStream_t s);
// centers32 = (float)centers64 and cnorm = |c|^2 (+inf padding for j in [k, kpad)).
void kmeans_prepare_centers(const double* centers64, int k, int d, float* centers32, float* cnorm,
                            int kpad, hipStream_t s);

// Deterministic float sum: per-block partials into slab[grid] then a fixed-order pass.
// Returns the number of partials written (<= 256).
int reduce_sum_f32(const float* v, int64_t n, double* slab, hipStream_t s);
// out[i][0..cols) = x[idx[i]][0..cols)  (device pointers)
void gather_rows(const float* x, int64_t ld, int cols, const int64_t* idx, int64_t m, float* out,
                 hipStream_t s);
// Appends i to out_idx for every flag[i] != 0 (unordered; count via *counter, zeroed by caller).
void compact_flags(const int32_t* flag, int64_t n, int64_t* out_idx, unsigned long long* counter,
                   hipStream_t s);

// k-means|| helpers
void elementwise_min(float* acc, const float* v, int64_t n, hipStream_t s);
// flag[i] = u(seed, step, row0+i) < factor * cost[i]   (u ~ U[0,1))
void bernoulli_select(const float* cost, int64_t n, int64_t row0, double factor, uint64_t seed,
                      int step, int32_t* flag, hipStream_t s);

}  // namespace kern
}  // namespace oap
