// Fused score + top-k of ALSModel.recommendForAll* (kernels/als_recommend.hip): the role of
// Spark's blocked recommendForAll (spark-3.1.1/mllib/src/main/scala/org/apache/spark/ml/
// recommendation/ALS.scala:365-505, GEMM blocks + a bounded priority queue per source row),
// with the scores never leaving registers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace oap {
namespace kern {

// Packed operand image of a factor matrix: per row `rec_row_slots(rank)` 16-byte slots, slot
// (plane p, k-step s, half h) = p * 2 KS + 2 s + h holding 8 fp16 features 16 s + 8 h .. + 7 of
// plane p (0: hi = fp16(x * 2^e), 1: lo = fp16(x * 2^e - hi)), KS = ceil(rank / 16); 2^e puts
// the matrix's max |x| (destinations) or each row's (sources, row_exp) in [128, 256).  Rows are
// padded to `rows_pad` with zeros.
int rec_ks(int rank);
int rec_row_slots(int rank);
// largest num the kernel's per-row lists hold at this rank (0: rank not supported)
int rec_max_num(int rank);
// largest num of the HBM-buffer variant (rec_topk_big), and its candidate scratch per workgroup
int rec_big_max_num(int rank);
size_t rec_big_scratch_per_wg(int num);
// source rows per workgroup of the top-k kernel at (rank, num): pad the source image to this
size_t rec_src_granule(int rank, int num);
// max |x| of rows [n][ld] (first `rank` columns) as float bits into *amax (atomicMax; zero it
// first)
void rec_absmax(const float* x, int64_t n, int rank, int64_t ld, unsigned* amax, hipStream_t s);
// per-row scale exponents e of rows [n][ld] (sources)
void rec_row_exp(const float* x, int64_t n, int rank, int64_t ld, int32_t* row_exp,
                 hipStream_t s);
// the image at the matrix's scale (amax, row_exp null) or at per-row scales (row_exp)
void rec_pack(const float* x, int64_t n, int rank, int64_t ld, const unsigned* amax,
              const int32_t* row_exp, void* img, int64_t rows_pad, hipStream_t s);
// Top-`num` destinations of every source row: score(i, j) = src_i . dst_j in split-fp16
// (hi.hi + hi.lo + lo.hi on v_mfma_f32_32x32x16_f16, fp32 accumulation: ~2^-21 relative to
// sum |src_ik dst_jk|), ties by lower destination index.  src_img rows padded to a multiple
// of rec_src_granule(rank, num), dst_img rows to a multiple of 64.  out_idx / out_val
// [n_src][num] (idx -1 / val -inf where n_dst < num).
void rec_topk(const void* src_img, const int32_t* src_exp, int64_t n_src, const void* dst_img,
              const unsigned* dst_amax, int64_t n_dst, int rank, int num, int32_t* out_idx,
              float* out_val, hipStream_t s);
// The same for num beyond the LDS lists (rec_max_num < num <= rec_big_max_num): per-lane
// candidate buffers in `scratch` (HBM; workgroups run in chunks of scratch_bytes /
// rec_big_scratch_per_wg(num)), sorted by the wave when one could overflow.  src_img rows
// padded to a multiple of rec_src_granule(rank, num).
void rec_topk_big(const void* src_img, const int32_t* src_exp, int64_t n_src,
                  const void* dst_img, const unsigned* dst_amax, int64_t n_dst, int rank, int num,
                  int32_t* out_idx, float* out_val, void* scratch, size_t scratch_bytes,
                  hipStream_t s);

}  // namespace kern
}  // namespace oap
