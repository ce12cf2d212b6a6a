// JNI shim: the reference's native methods (mllib-dal/src/main/native/javah/*.h)
// with the reference's exact JNI names AND signatures, implemented over the C ABI
// (capi/oap_capi.h).  Compiled into liboap_mllib.so only when JAVA_HOME points at a JDK
// (oap_mllib_amd/build.py); the test suite compiles it against tests/native/jni_stub and drives
// every entry point through a recording JNIEnv (tests/native/jni_harness.cpp).
//
// Mapping (reference -> here):
//  * OneCCL$: c_init(size, rank, "ip_port" | hex unique id, CCLParam{long commSize, rankId}).
//    With size > 1 the string is either the reference's KVS address "ip_port" (rank 0 serves
//    a TCP rendezvous there: the RCCL unique id for GPU contexts, the host collectives
//    themselves for CPU contexts — comm/tcp_comm.h), or the hex RCCL unique id that rank 0 made
//    with c_uniqueId() and the launcher distributed (Spark BarrierTaskContext.allGather).  One
//    persistent context per executor process.
//    setEnv / c_getAvailPort keep the reference's behaviour (OneCCL.cpp:127-247).
//  * OneDAL$: native row tables (f64, row-major) — setNumericTableValue (one value,
//    OneDAL.cpp:35-43), cSetDoubleBatch (row batch, :50-60), cAddNumericTable (append, :67-76),
//    cFreeDataMemory, cCheckPlatformCompatibility (gfx950 present, :96-102) and
//    cNewCSRNumericTable (1-based CSR from Java arrays, :109-145).  Results are read back with
//    cNumRows / cNumCols / cGetDoubleArray (the reference reads oneDAL Java NumericTables).
//  * KMeansDALImpl / PCADALImpl / ALSDALImpl: the train entry points with the reference
//    signatures; ALS runs the shuffle (cShuffleData: range partition by key + alltoallv + sort,
//    ALSShuffle.cpp:62-127) and cDALImplictALS(csr, nUsers, ...) returns this rank's contiguous
//    user / item factor blocks with their offsets (ALSDALImpl.cpp:500-576 contract).
// Errors raise java.lang.RuntimeException (never exit()).
#include <arpa/inet.h>
#include <ifaddrs.h>
#include <jni.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <vector>

#include "capi/oap_capi.h"

namespace {

struct RowTable {
  int64_t rows = 0;
  int cols = 0;
  std::vector<double> data;
};

// 0-based CSR (the reference's oneDAL CSRNumericTable is 1-based; converted on entry)
struct CsrTable {
  int64_t rows = 0, cols = 0;
  std::vector<int64_t> rowptr, colidx;
  std::vector<float> vals;
};

std::mutex g_mu;
oap_ctx* g_ctx = nullptr;  // one per executor process
// last cShuffleData output (the reference also keeps it in a native global, ALSShuffle.cpp:28):
// the records handed to Java as a direct ByteBuffer, and the distinct keys (CSR row -> key)
void* g_shuffled = nullptr;
std::vector<int64_t> g_shuffle_keys;

void throw_java(JNIEnv* env, const std::string& msg) {
  jclass ex = env->FindClass("java/lang/RuntimeException");
  if (ex) env->ThrowNew(ex, msg.c_str());
}

bool check(JNIEnv* env, int rc) {
  if (rc >= 0) return true;
  throw_java(env, std::string("oap_mllib native error: ") + oap_last_error());
  return false;
}

// Field setters: a missing field leaves Java's NoSuchFieldError pending and writes nothing.
bool set_int(JNIEnv* env, jobject o, const char* f, jint v) {
  jfieldID id = env->GetFieldID(env->GetObjectClass(o), f, "I");
  if (!id) return false;
  env->SetIntField(o, id, v);
  return true;
}
bool set_long(JNIEnv* env, jobject o, const char* f, jlong v) {
  jfieldID id = env->GetFieldID(env->GetObjectClass(o), f, "J");
  if (!id) return false;
  env->SetLongField(o, id, v);
  return true;
}
bool set_double(JNIEnv* env, jobject o, const char* f, jdouble v) {
  jfieldID id = env->GetFieldID(env->GetObjectClass(o), f, "D");
  if (!id) return false;
  env->SetDoubleField(o, id, v);
  return true;
}

RowTable* table(jlong h) { return reinterpret_cast<RowTable*>(h); }
CsrTable* csr(jlong h) { return reinterpret_cast<CsrTable*>(h); }

int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}

bool ensure_ctx(JNIEnv* env) {
  if (g_ctx) return true;
  const int dev = oap_device_count() > 0 ? 0 : -1;  // an executor sees its own GPU as device 0
  g_ctx = oap_ctx_create(dev, 0.9, 0);
  return check(env, g_ctx ? 0 : -1);
}

// Is `ip` one of this host's IPv4 addresses (OneCCL.cpp:141-200)?
bool is_local_ip(const char* ip) {
  struct ifaddrs* ifs = nullptr;
  if (getifaddrs(&ifs) != 0) return false;
  bool found = false;
  for (struct ifaddrs* p = ifs; p && !found; p = p->ifa_next) {
    if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET) continue;
    char buf[INET_ADDRSTRLEN] = {0};
    auto* sin = reinterpret_cast<struct sockaddr_in*>(p->ifa_addr);
    if (inet_ntop(AF_INET, &sin->sin_addr, buf, sizeof(buf)) && std::strcmp(buf, ip) == 0)
      found = true;
  }
  freeifaddrs(ifs);
  return found;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- OneCCL$ (communicator)
JNIEXPORT jstring JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_c_1uniqueId(JNIEnv* env,
                                                                                jobject) {
  unsigned char id[OAP_UNIQUE_ID_BYTES];
  if (!check(env, oap_rccl_unique_id(id))) return nullptr;
  std::string hex;
  char b[3];
  for (unsigned char v : id) {
    std::snprintf(b, sizeof(b), "%02x", v);
    hex += b;
  }
  return env->NewStringUTF(hex.c_str());
}

// (IILjava/lang/String;Lorg/apache/spark/ml/util/CCLParam;)I
JNIEXPORT jint JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_c_1init(JNIEnv* env, jobject,
                                                                         jint size, jint rank,
                                                                         jstring uid_hex,
                                                                         jobject param) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!ensure_ctx(env)) return -1;
  if (size > 1) {
    const char* s = env->GetStringUTFChars(uid_hex, nullptr);
    const std::string str = s ? s : "";
    if (s) env->ReleaseStringUTFChars(uid_hex, s);
    unsigned char id[OAP_UNIQUE_ID_BYTES] = {0};
    bool hex = str.size() == 2 * OAP_UNIQUE_ID_BYTES;
    for (size_t i = 0; hex && i < str.size(); i += 2) {
      const int hi = hexval(str[i]), lo = hexval(str[i + 1]);
      hex = hi >= 0 && lo >= 0;
      id[i / 2] = static_cast<unsigned char>(hi * 16 + lo);
    }
    // the hex RCCL unique id from c_uniqueId(), or the reference's KVS string "ip_port"
    // (KMeansDALImpl.scala:39-50): rank 0 serves the rendezvous at that address
    const int rc = hex ? oap_ctx_join(g_ctx, id, size, rank, 600.0)
                       : oap_ctx_join_kvs(g_ctx, str.c_str(), size, rank, 600.0);
    if (!check(env, rc)) return -1;
  }
  // CCLParam.commSize / rankId are Java longs (CCLParam.java:20-21)
  if (!set_long(env, param, "commSize", oap_ctx_world_size(g_ctx))) return -1;
  if (!set_long(env, param, "rankId", oap_ctx_rank(g_ctx))) return -1;
  return 0;
}

JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_c_1cleanup(JNIEnv*, jobject) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_ctx) oap_ctx_destroy(g_ctx);
  g_ctx = nullptr;
  oap_free(g_shuffled);
  g_shuffled = nullptr;
  g_shuffle_keys.clear();
}

JNIEXPORT jboolean JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_isRoot(JNIEnv*, jobject) {
  return g_ctx && oap_ctx_rank(g_ctx) == 0;
}

JNIEXPORT jint JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_rankID(JNIEnv*, jobject) {
  return g_ctx ? oap_ctx_rank(g_ctx) : -1;
}

// (Ljava/lang/String;Ljava/lang/String;Z)I
JNIEXPORT jint JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_setEnv(JNIEnv* env, jobject,
                                                                        jstring key,
                                                                        jstring value,
                                                                        jboolean overwrite) {
  const char* k = env->GetStringUTFChars(key, nullptr);
  const char* v = env->GetStringUTFChars(value, nullptr);
  const int rc = (k && v) ? setenv(k, v, overwrite ? 1 : 0) : -1;
  if (k) env->ReleaseStringUTFChars(key, k);
  if (v) env->ReleaseStringUTFChars(value, v);
  return rc;
}

// (Ljava/lang/String;)I: first bindable TCP port >= 3000 on `ip` (which must be local), else -1
JNIEXPORT jint JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_c_1getAvailPort(JNIEnv* env,
                                                                                 jobject,
                                                                                 jstring ip) {
  const char* s = env->GetStringUTFChars(ip, nullptr);
  if (!s) return -1;
  std::string addr(s);
  env->ReleaseStringUTFChars(ip, s);
  if (!is_local_ip(addr.c_str())) return -1;
  for (int port = 3000; port < 65535; ++port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return -1;
    struct sockaddr_in sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sin_family = AF_INET;
    sa.sin_port = htons(static_cast<uint16_t>(port));
    inet_pton(AF_INET, addr.c_str(), &sa.sin_addr);
    const int rc = bind(fd, reinterpret_cast<struct sockaddr*>(&sa), sizeof(sa));
    close(fd);
    if (rc == 0) return port;
  }
  return -1;
}

// ---------------------------------------------------------------- OneDAL$ (row tables)
JNIEXPORT jboolean JNICALL
Java_org_apache_spark_ml_util_OneDAL_00024_cCheckPlatformCompatibility(JNIEnv*, jobject) {
  return oap_device_count() > 0 && oap_check_platform(0) == 1;
}

JNIEXPORT jlong JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cNewRowTable(JNIEnv*, jobject,
                                                                               jlong rows,
                                                                               jint cols) {
  auto* t = new RowTable;
  t->rows = rows;
  t->cols = cols;
  t->data.assign(size_t(rows) * cols, 0.0);
  return reinterpret_cast<jlong>(t);
}

// (JIID)V
JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_setNumericTableValue(
    JNIEnv* env, jobject, jlong h, jint row, jint col, jdouble v) {
  RowTable* t = table(h);
  if (!t || row < 0 || row >= t->rows || col < 0 || col >= t->cols) {
    throw_java(env, "setNumericTableValue: index out of the table's bounds");
    return;
  }
  t->data[size_t(row) * t->cols + col] = v;
}

// (JI[DII)V
JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cSetDoubleBatch(
    JNIEnv* env, jobject, jlong h, jint row0, jdoubleArray batch, jint nrows, jint cols) {
  RowTable* t = table(h);
  if (!t || cols != t->cols || row0 < 0 || nrows < 0 || int64_t(row0) + nrows > t->rows) {
    throw_java(env, "cSetDoubleBatch: batch out of the table's bounds");
    return;
  }
  env->GetDoubleArrayRegion(batch, 0, nrows * cols, t->data.data() + size_t(row0) * cols);
}

JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cAddNumericTable(JNIEnv* env,
                                                                                  jobject,
                                                                                  jlong dst,
                                                                                  jlong src) {
  RowTable *a = table(dst), *b = table(src);
  if (!a || !b || (a->rows && a->cols != b->cols)) {
    throw_java(env, "cAddNumericTable: column mismatch");
    return;
  }
  if (a->rows == 0) a->cols = b->cols;
  a->data.insert(a->data.end(), b->data.begin(), b->data.end());
  a->rows += b->rows;
}

// frees a row table or a CSR table handle (the reference frees its oneDAL tables here)
JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cFreeDataMemory(JNIEnv*, jobject,
                                                                                 jlong h) {
  delete table(h);
}

JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cFreeCSRTable(JNIEnv*, jobject,
                                                                               jlong h) {
  delete csr(h);
}

// ([F[J[JJJ)J: 1-based CSR arrays (values, column indices, row offsets), nFeatures columns,
// nVectors rows (OneDAL.cpp:109-145)
JNIEXPORT jlong JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cNewCSRNumericTable(
    JNIEnv* env, jobject, jfloatArray data, jlongArray col_indices, jlongArray row_offsets,
    jlong n_features, jlong n_vectors) {
  const jsize nnz = env->GetArrayLength(data);
  const jsize n_off = env->GetArrayLength(row_offsets);
  // The reference's bufferToCSRNumericTable (ALSDALImpl.scala:184-230) starts from offsets [1]
  // at row 0, so a partition whose lowest key has no ratings (or no ratings at all) carries a
  // leading empty row: [1, 1, ...] with csrRowNum + 2 entries.  That leading row is dropped —
  // CSR row i stays the i-th distinct key, as cShuffleData's key table maps it.
  if (env->GetArrayLength(col_indices) != nnz || n_vectors < 0 ||
      (n_off != n_vectors + 1 && n_off != n_vectors + 2)) {
    throw_java(env, "cNewCSRNumericTable: inconsistent CSR array lengths");
    return 0;
  }
  std::vector<int64_t> offs(static_cast<size_t>(n_off));
  if (n_off) env->GetLongArrayRegion(row_offsets, 0, n_off, reinterpret_cast<jlong*>(offs.data()));
  if (n_off == n_vectors + 2) {
    if (offs[0] != 1 || offs[1] != 1) {
      throw_java(env, "cNewCSRNumericTable: inconsistent CSR array lengths");
      return 0;
    }
    offs.erase(offs.begin());
  }
  auto* t = new CsrTable;
  t->rows = n_vectors;
  t->cols = n_features;
  t->vals.resize(size_t(nnz));
  t->colidx.resize(size_t(nnz));
  t->rowptr = std::move(offs);
  if (nnz) {
    env->GetFloatArrayRegion(data, 0, nnz, t->vals.data());
    env->GetLongArrayRegion(col_indices, 0, nnz, reinterpret_cast<jlong*>(t->colidx.data()));
  }
  bool ok = t->rowptr[0] == 1 && t->rowptr[size_t(n_vectors)] == int64_t(nnz) + 1;
  for (int64_t i = 0; ok && i < n_vectors; ++i) ok = t->rowptr[i] <= t->rowptr[i + 1];
  for (auto& v : t->rowptr) --v;
  for (auto& c : t->colidx) {
    ok = ok && c >= 1 && c <= n_features;
    --c;
  }
  if (!ok) {
    delete t;
    throw_java(env, "cNewCSRNumericTable: not a valid 1-based CSR");
    return 0;
  }
  return reinterpret_cast<jlong>(t);
}

JNIEXPORT jlong JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cNumRows(JNIEnv*, jobject,
                                                                           jlong h) {
  return table(h) ? table(h)->rows : -1;
}

JNIEXPORT jint JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cNumCols(JNIEnv*, jobject,
                                                                          jlong h) {
  return table(h) ? table(h)->cols : -1;
}

JNIEXPORT jdoubleArray JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cGetDoubleArray(
    JNIEnv* env, jobject, jlong h) {
  RowTable* t = table(h);
  if (!t) return nullptr;
  jdoubleArray out = env->NewDoubleArray(static_cast<jsize>(t->data.size()));
  env->SetDoubleArrayRegion(out, 0, static_cast<jsize>(t->data.size()), t->data.data());
  return out;
}

// ---------------------------------------------------------------- K-Means
// (JJIDIIILorg/apache/spark/ml/clustering/KMeansResult;)J: (data, initial centers) tables ->
// new centers table (every rank; the reference returns it on rank 0 only).
JNIEXPORT jlong JNICALL
Java_org_apache_spark_ml_clustering_KMeansDALImpl_cKMeansDALComputeWithInitCenters(
    JNIEnv* env, jobject, jlong data, jlong centers, jint k, jdouble tol, jint max_iter,
    jint /*executor_num*/, jint /*executor_cores*/, jobject result) {
  RowTable *x = table(data), *c0 = table(centers);
  if (!g_ctx || !x || !c0 || c0->rows != k || c0->cols != x->cols) {
    throw_java(env, "cKMeansDALComputeWithInitCenters: not initialised or bad tables");
    return 0;
  }
  auto* out = new RowTable;
  out->rows = k;
  out->cols = x->cols;
  out->data.resize(size_t(k) * x->cols);
  double cost = 0.0;
  int iters = 0;
  if (!check(env, oap_kmeans_fit(g_ctx, x->data.data(), x->rows, x->cols, c0->data.data(), k,
                                 max_iter, tol, 0, out->data.data(), &cost, &iters))) {
    delete out;
    return 0;
  }
  if (!set_int(env, result, "iterationNum", iters) ||
      !set_double(env, result, "totalCost", cost)) {
    delete out;
    return 0;
  }
  return reinterpret_cast<jlong>(out);
}

// ---------------------------------------------------------------- PCA
// (JIIILorg/apache/spark/ml/feature/PCAResult;)J
JNIEXPORT jlong JNICALL Java_org_apache_spark_ml_feature_PCADALImpl_cPCATrainDAL(
    JNIEnv* env, jobject, jlong data, jint k, jint /*executor_num*/, jint /*executor_cores*/,
    jobject result) {
  RowTable* x = table(data);
  if (!g_ctx || !x) {
    throw_java(env, "cPCATrainDAL: not initialised or bad table");
    return 0;
  }
  auto* pc = new RowTable;  // cols x k, row-major (column j = component j)
  pc->rows = x->cols;
  pc->cols = k;
  pc->data.resize(size_t(x->cols) * k);
  auto* ev = new RowTable;  // 1 x k explained variance
  ev->rows = 1;
  ev->cols = k;
  ev->data.resize(k);
  if (!check(env, oap_pca_fit(g_ctx, x->data.data(), x->rows, x->cols, k, pc->data.data(),
                              ev->data.data()))) {
    delete pc;
    delete ev;
    return 0;
  }
  if (!set_long(env, result, "pcNumericTable", reinterpret_cast<jlong>(pc)) ||
      !set_long(env, result, "explainedVarianceNumericTable", reinterpret_cast<jlong>(ev))) {
    delete pc;
    delete ev;
  }
  return 0;
}

// ---------------------------------------------------------------- ALS
// (Ljava/nio/ByteBuffer;IILorg/apache/spark/ml/recommendation/ALSPartitionInfo;)
// Ljava/nio/ByteBuffer;  — packed 20-byte little-endian {int64 key; int64 other; float rating}
// records (ALSShuffle.h:22-28), range-partitioned by key over the world, sorted by (key, other);
// the returned direct buffer stays valid until the next call or c_cleanup.
JNIEXPORT jobject JNICALL Java_org_apache_spark_ml_recommendation_ALSDALImpl_cShuffleData(
    JNIEnv* env, jobject, jobject data_buffer, jint n_total_keys, jint n_blocks, jobject info) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ctx) {
    throw_java(env, "cShuffleData: OneCCL.init first");
    return nullptr;
  }
  const auto* rec = static_cast<const unsigned char*>(env->GetDirectBufferAddress(data_buffer));
  const jlong cap = env->GetDirectBufferCapacity(data_buffer);
  if ((!rec && cap > 0) || cap < 0 || cap % 20 != 0) {
    throw_java(env, "cShuffleData: ratings must be a direct ByteBuffer of 20-byte records");
    return nullptr;
  }
  oap_free(g_shuffled);
  g_shuffled = nullptr;
  g_shuffle_keys.clear();
  int64_t n = 0, distinct = 0;
  if (!check(env, oap_shuffle_ratings(g_ctx, rec, cap / 20, n_total_keys, n_blocks, &g_shuffled,
                                      &n, &distinct)))
    return nullptr;
  if (n > std::numeric_limits<jint>::max()) {  // ALSPartitionInfo fields are Java ints
    throw_java(env, "cShuffleData: more ratings on one rank than a Java int holds");
    return nullptr;
  }
  const auto* out = static_cast<const unsigned char*>(g_shuffled);
  g_shuffle_keys.reserve(size_t(distinct));
  for (int64_t i = 0; i < n; ++i) {
    int64_t key;
    std::memcpy(&key, out + 20 * i, 8);
    if (g_shuffle_keys.empty() || g_shuffle_keys.back() != key) g_shuffle_keys.push_back(key);
  }
  if (!set_int(env, info, "ratingsNum", jint(n)) ||
      !set_int(env, info, "csrRowNum", jint(distinct)))
    return nullptr;
  return env->NewDirectByteBuffer(g_shuffled, n * 20);
}

// (JJIIDDIIILorg/apache/spark/ml/recommendation/ALSResult;)J: the CSR of this rank's shuffled
// ratings (rows = its distinct keys in order — the reference's transposed items — columns =
// user index + 1), nUsers, rank, iterations, regParam, alpha.  Spark computeFactors semantics
// (regParam and alpha honoured, unlike the reference).  ALSResult gets this rank's contiguous
// blocks of the user and item factors ([offset, offset + rows) with ceil(n / P) ids per rank;
// ids without ratings get zero rows) as row tables of nFactors columns.
JNIEXPORT jlong JNICALL Java_org_apache_spark_ml_recommendation_ALSDALImpl_cDALImplictALS(
    JNIEnv* env, jobject, jlong csr_handle, jlong n_users, jint n_factors, jint max_iter,
    jdouble reg, jdouble alpha, jint /*executor_num*/, jint /*executor_cores*/,
    jint partition_id, jobject result) {
  std::lock_guard<std::mutex> lk(g_mu);
  CsrTable* t = csr(csr_handle);
  if (!g_ctx || !t) {
    throw_java(env, "cDALImplictALS: not initialised or bad CSR table");
    return 0;
  }
  if (int64_t(g_shuffle_keys.size()) != t->rows) {
    throw_java(env, "cDALImplictALS: the CSR rows do not match the last cShuffleData output");
    return 0;
  }
  const int64_t nnz = int64_t(t->vals.size());
  constexpr int64_t kMaxId = std::numeric_limits<int32_t>::max();
  std::vector<int32_t> u(static_cast<size_t>(nnz)), it(static_cast<size_t>(nnz));
  int64_t max_item = -1;
  for (int64_t row = 0; row < t->rows; ++row) {
    const int64_t key = g_shuffle_keys[size_t(row)];
    if (key < 0 || key > kMaxId) {
      throw_java(env, "cDALImplictALS: item id beyond the int32 range");
      return 0;
    }
    max_item = std::max(max_item, key);
    for (int64_t j = t->rowptr[row]; j < t->rowptr[row + 1]; ++j) {
      if (t->colidx[j] > kMaxId) {
        throw_java(env, "cDALImplictALS: user id beyond the int32 range");
        return 0;
      }
      u[size_t(j)] = int32_t(t->colidx[j]);
      it[size_t(j)] = int32_t(key);
    }
  }
  int64_t n_items = max_item + 1;
  if (!check(env, oap_allreduce_i64(g_ctx, &n_items, 1, 1))) return 0;
  oap_als_result* res = nullptr;
  if (!check(env, oap_als_fit(g_ctx, u.data(), it.data(), t->vals.data(), nnz, n_factors,
                              max_iter, reg, alpha, 1, 0, &res)))
    return 0;
  const int P = oap_ctx_world_size(g_ctx), me = oap_ctx_rank(g_ctx);
  auto block = [&](int which, int64_t n_ids, int64_t* offset) {
    const int64_t per = (n_ids + P - 1) / P;
    const int64_t lo = std::min<int64_t>(n_ids, per * me), hi = std::min<int64_t>(n_ids, lo + per);
    auto* tab = new RowTable;
    tab->rows = hi - lo;
    tab->cols = n_factors;
    tab->data.assign(size_t(hi - lo) * n_factors, 0.0);
    const int64_t cnt = oap_als_result_count(res, which);
    const int32_t* ids = oap_als_result_ids(res, which);  // ascending
    const float* f = oap_als_result_factors(res, which);
    const int32_t* b = std::lower_bound(ids, ids + cnt, int32_t(std::min<int64_t>(lo, kMaxId)));
    for (; b != ids + cnt && *b < hi; ++b) {
      const int64_t i = b - ids;
      for (int j = 0; j < n_factors; ++j)
        tab->data[size_t(*b - lo) * n_factors + j] = f[size_t(i) * n_factors + j];
    }
    *offset = lo;
    return reinterpret_cast<jlong>(tab);
  };
  int64_t uoff = 0, ioff = 0;
  const jlong ut = block(0, n_users, &uoff), itab = block(1, n_items, &ioff);
  oap_als_result_free(res);
  if (partition_id != me)
    std::fprintf(stderr, "cDALImplictALS: partition %d runs as rank %d\n", partition_id, me);
  if (!set_long(env, result, "rankId", me) || !set_long(env, result, "cUsersFactorsNumTab", ut) ||
      !set_long(env, result, "cItemsFactorsNumTab", itab) ||
      !set_long(env, result, "cUserOffset", uoff) || !set_long(env, result, "cItemOffset", ioff)) {
    delete table(ut);
    delete table(itab);
  }
  return 0;
}

}  // extern "C"
