/* oap_mllib C ABI — the language-neutral entry points of liboap_mllib.so.
 *
 * MI355X-native counterpart of the reference's JNI surface (mllib-dal/src/main/native/javah/
 * *.h): the JNI shim (csrc/jni/, built when a JDK is present) and any other
 * host language call these.  Differences from the reference by design: typed row buffers
 * instead of oneDAL NumericTable handles (no per-scalar JNI calls, OneDAL.cpp:35-43), a
 * persistent context + communicator instead of one oneCCL KVS per fit (OneCCL.cpp:47-99), error
 * codes + oap_last_error() instead of exit() (error_handling.cpp:30-57), and explicit free
 * functions for every result (the reference leaks its `new SharedPtr` handles).
 *
 * Every call returns 0 on success, < 0 on failure (message in oap_last_error(), thread-local).
 * A context owns one device (or the CPU engine) and one communicator; it is not thread-safe.
 */
#ifndef OAP_CAPI_H_
#define OAP_CAPI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OAP_API __attribute__((visibility("default")))
#define OAP_CAPI_VERSION 1
#define OAP_UNIQUE_ID_BYTES 128

typedef struct oap_ctx oap_ctx;
typedef struct oap_als_result oap_als_result;

OAP_API int oap_capi_version(void);
OAP_API const char* oap_last_error(void);

/* Visible HIP devices (0 without a GPU).  Counts without creating a HIP context. */
OAP_API int oap_device_count(void);
/* 1 when device `device` is a gfx950 (MI355X-class) GPU, else 0 — the reference's
 * cCheckPlatformCompatibility (OneDAL.cpp:96-102) for this backend. */
OAP_API int oap_check_platform(int device);

/* device >= 0: that GPU (HBM arena = hbm_fraction of free memory); device < 0: native CPU engine.
 * cpu_threads <= 0: min(cores, 16).  The context starts with a world-size-1 communicator. */
OAP_API oap_ctx* oap_ctx_create(int device, double hbm_fraction, int cpu_threads);
OAP_API void oap_ctx_destroy(oap_ctx* ctx);

/* RCCL rendezvous: rank 0 creates the id, the launcher distributes it (e.g. Spark
 * BarrierTaskContext.allGather), every rank joins.  Replaces the oneCCL KVS + port scan. */
OAP_API int oap_rccl_unique_id(unsigned char out[OAP_UNIQUE_ID_BYTES]);
OAP_API int oap_ctx_join(oap_ctx* ctx, const unsigned char id[OAP_UNIQUE_ID_BYTES], int world,
                         int rank, double timeout_s);
/* The reference's KVS contract: OneCCL.init(size, rank, "ip_port") (OneCCL.cpp:47-86).  Rank 0
 * listens on ip:port (a port from c_getAvailPort's bind scan), the others connect to it.  GPU
 * contexts: rank 0's RCCL unique id travels over that store, then every rank joins RCCL.  CPU
 * contexts: the store's sockets carry the host collectives (TcpComm, star through rank 0).
 * Accepts "ip_port" or "ip:port". */
OAP_API int oap_ctx_join_kvs(oap_ctx* ctx, const char* ip_port, int world, int rank,
                             double timeout_s);
OAP_API int oap_ctx_world_size(const oap_ctx* ctx);
OAP_API int oap_ctx_rank(const oap_ctx* ctx);

/* K-Means (Lloyd) on this rank's row shard x[rows][cols] (row-major f64), starting from
 * init_centers[k][cols] (identical on every rank).  storage_bf16 != 0 stores rows as bf16.
 * Outputs (every rank): out_centers[k][cols], *out_cost (Spark trainingCost of the last
 * assignment), *out_iters.  Mirrors cKMeansDALComputeWithInitCenters (KMeansDALImpl.cpp:175). */
OAP_API int oap_kmeans_fit(oap_ctx* ctx, const double* x, int64_t rows, int cols,
                   const double* init_centers, int k, int max_iter, double tol, int storage_bf16,
                   double* out_centers, double* out_cost, int* out_iters);
/* k-means|| (init_steps rounds) or random ("random") initial centers; out_centers[k][cols],
 * *out_k = centers found (<= k when the data has fewer distinct rows). */
OAP_API int oap_kmeans_init(oap_ctx* ctx, const double* x, int64_t rows, int cols, int k,
                    const char* mode, int init_steps, uint64_t seed, double* out_centers,
                    int* out_k);
/* Nearest center per local row (labels) and its squared distance (optional, may be NULL). */
OAP_API int oap_kmeans_predict(oap_ctx* ctx, const double* x, int64_t rows, int cols,
                       const double* centers, int k, int32_t* labels, double* dist2);

/* PCA: top-k principal components of the (globally) mean-centered rows.  out_pc[cols][k]
 * row-major (column j = component j), out_explained[k] = |lambda_j| / sum |lambda| (Spark
 * RowMatrix semantics).  Mirrors cPCATrainDAL (PCADALImpl.cpp:38-190). */
OAP_API int oap_pca_fit(oap_ctx* ctx, const double* x, int64_t rows, int cols, int k,
                        double* out_pc, double* out_explained);

/* ALS: this rank's (user, item, rating) triples, any ids.  Spark computeFactors semantics
 * (implicit: c = alpha |r|, lambda * n_u).  Mirrors cShuffleData + cDALImplictALS
 * (ALSDALImpl.cpp:456-576); results are owned by the returned handle. */
OAP_API int oap_als_fit(oap_ctx* ctx, const int32_t* users, const int32_t* items,
                        const float* ratings, int64_t n, int rank, int max_iter, double reg,
                        double alpha, int implicit, uint64_t seed, oap_als_result** out);
/* which = 0: users, 1: items.  *ids / *factors ([count][rank]) stay valid until the free. */
OAP_API int64_t oap_als_result_count(const oap_als_result* res, int which);
OAP_API int oap_als_result_rank(const oap_als_result* res);
OAP_API const int32_t* oap_als_result_ids(const oap_als_result* res, int which);
OAP_API const float* oap_als_result_factors(const oap_als_result* res, int which);
OAP_API void oap_als_result_free(oap_als_result* res);

/* The reference's ratings shuffle (ALSShuffle.cpp:62-127 behind cShuffleData): records are
 * packed 20-byte little-endian {int64 key; int64 other; float rating}; each goes to rank
 * min(key / max(n_total_keys / n_blocks, 1), n_blocks - 1) (n_blocks == world size).  *out gets
 * this rank's received records sorted by (key, other) (free with oap_free), *out_n their number
 * and *out_distinct the number of distinct keys (the CSR row count). */
OAP_API int oap_shuffle_ratings(oap_ctx* ctx, const void* records, int64_t n,
                                int64_t n_total_keys, int n_blocks, void** out, int64_t* out_n,
                                int64_t* out_distinct);
/* In-place allreduce of count int64 values across the context's world (op: 0 sum, 1 max,
 * 2 min). */
OAP_API int oap_allreduce_i64(oap_ctx* ctx, int64_t* vals, int count, int op);
OAP_API void oap_free(void* p);

#ifdef __cplusplus
}
#endif

#endif  // OAP_CAPI_H_
