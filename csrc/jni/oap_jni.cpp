// JNI shim: the reference's native method names (mllib-dal/src/main/native/javah/*.h, SURVEY.md
// §2.8) implemented over the C ABI (capi/oap_capi.h).  Compiled into liboap_mllib.so only when
// JAVA_HOME points at a JDK (oap_mllib_amd/build.py); no JDK exists in the build container, so
// this file is exercised by the Scala shadow classes on a Spark cluster, not by the test suite.
//
// Mapping (reference -> here):
//  * OneCCL$.c_init(size, rank, "ip_port", CCLParam): the string carries the hex-encoded RCCL
//    unique id that rank 0 made with c_uniqueId() and Spark's BarrierTaskContext.allGather
//    distributed — no KVS server, no port scan (OneCCL.cpp:47-247).  One persistent context
//    per executor process (device = the executor's GPU), reused across fits.
//  * OneDAL$ tables: a native row buffer handle (f64, row-major) filled by cSetDoubleBatch
//    (one JNI call per row batch, OneDAL.cpp:50-60); cAddNumericTable appends rows;
//    cGetDoubleArray / cNumRows / cNumCols read results back (replaces the oneDAL Java
//    NumericTable accessors, OneDAL.scala:37-52).
//  * KMeansDALImpl / PCADALImpl / ALSDALImpl train entry points call oap_kmeans_fit /
//    oap_pca_fit / oap_als_fit; errors raise java.lang.RuntimeException (never exit()).
#include <jni.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
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

std::mutex g_mu;
oap_ctx* g_ctx = nullptr;  // one per executor process

void throw_java(JNIEnv* env, const std::string& msg) {
  jclass ex = env->FindClass("java/lang/RuntimeException");
  if (ex) env->ThrowNew(ex, msg.c_str());
}

bool check(JNIEnv* env, int rc) {
  if (rc >= 0) return true;
  throw_java(env, std::string("oap_mllib native error: ") + oap_last_error());
  return false;
}

void set_int(JNIEnv* env, jobject o, const char* f, jint v) {
  jclass c = env->GetObjectClass(o);
  env->SetIntField(o, env->GetFieldID(c, f, "I"), v);
}
void set_long(JNIEnv* env, jobject o, const char* f, jlong v) {
  jclass c = env->GetObjectClass(o);
  env->SetLongField(o, env->GetFieldID(c, f, "J"), v);
}
void set_double(JNIEnv* env, jobject o, const char* f, jdouble v) {
  jclass c = env->GetObjectClass(o);
  env->SetDoubleField(o, env->GetFieldID(c, f, "D"), v);
}

RowTable* table(jlong h) { return reinterpret_cast<RowTable*>(h); }

int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
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

JNIEXPORT jint JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_c_1init(JNIEnv* env, jobject,
                                                                         jint size, jint rank,
                                                                         jstring uid_hex,
                                                                         jobject param) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ctx) {
    const int dev = oap_device_count() > 0 ? 0 : -1;  // executor sees its own GPU as device 0
    g_ctx = oap_ctx_create(dev, 0.9, 0);
    if (!g_ctx) {
      check(env, -1);
      return -1;
    }
  }
  if (size > 1) {
    const char* s = env->GetStringUTFChars(uid_hex, nullptr);
    unsigned char id[OAP_UNIQUE_ID_BYTES] = {0};
    const size_t n = std::strlen(s);
    for (size_t i = 0; i + 1 < n && i / 2 < OAP_UNIQUE_ID_BYTES; i += 2)
      id[i / 2] = static_cast<unsigned char>(hexval(s[i]) * 16 + hexval(s[i + 1]));
    env->ReleaseStringUTFChars(uid_hex, s);
    if (!check(env, oap_ctx_join(g_ctx, id, size, rank, 600.0))) return -1;
  }
  set_int(env, param, "commSize", oap_ctx_world_size(g_ctx));
  set_int(env, param, "rankId", oap_ctx_rank(g_ctx));
  return 0;
}

JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_c_1cleanup(JNIEnv*, jobject) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_ctx) oap_ctx_destroy(g_ctx);
  g_ctx = nullptr;
}

JNIEXPORT jboolean JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_isRoot(JNIEnv*, jobject) {
  return g_ctx && oap_ctx_rank(g_ctx) == 0;
}

JNIEXPORT jint JNICALL Java_org_apache_spark_ml_util_OneCCL_00024_rankID(JNIEnv*, jobject) {
  return g_ctx ? oap_ctx_rank(g_ctx) : -1;
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

JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cSetDoubleBatch(
    JNIEnv* env, jobject, jlong h, jint row0, jdoubleArray batch, jint nrows, jint cols) {
  RowTable* t = table(h);
  if (!t || cols != t->cols || row0 < 0 || int64_t(row0) + nrows > t->rows) {
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

JNIEXPORT void JNICALL Java_org_apache_spark_ml_util_OneDAL_00024_cFreeDataMemory(JNIEnv*, jobject,
                                                                                 jlong h) {
  delete table(h);
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
// (data, initial centers) tables -> new centers table (every rank; the reference returns it on
// rank 0 only, KMeansDALImpl.cpp:175-249).
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
  set_int(env, result, "iterationNum", iters);
  set_double(env, result, "totalCost", cost);
  return reinterpret_cast<jlong>(out);
}

// ---------------------------------------------------------------- PCA
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
  set_long(env, result, "pcNumericTable", reinterpret_cast<jlong>(pc));
  set_long(env, result, "explainedVarianceNumericTable", reinterpret_cast<jlong>(ev));
  return 0;
}

// ---------------------------------------------------------------- ALS
// Ratings arrive as the reference's packed 20-byte little-endian records {int64 user; int64 item;
// float rating} in a direct ByteBuffer (ALSShuffle.h:22-28); the id shuffle, CSR build and the
// factor exchange happen inside oap_als_fit.  Factor tables: rows = owned ids, cols = 1 + rank
// (column 0 = the id as a double, exact below 2^53).
JNIEXPORT jlong JNICALL Java_org_apache_spark_ml_recommendation_ALSDALImpl_cDALImplictALS(
    JNIEnv* env, jobject, jobject ratings_buf, jlong n, jint rank, jint max_iter,
    jdouble reg, jdouble alpha, jint /*executor_num*/, jint /*executor_cores*/, jlong seed,
    jobject result) {
  if (!g_ctx) {
    throw_java(env, "cDALImplictALS: not initialised");
    return 0;
  }
  const auto* rec = static_cast<const unsigned char*>(env->GetDirectBufferAddress(ratings_buf));
  if (!rec && n > 0) {
    throw_java(env, "cDALImplictALS: ratings must be a direct ByteBuffer");
    return 0;
  }
  std::vector<int32_t> u(n), it(n);
  std::vector<float> r(n);
  for (int64_t i = 0; i < n; ++i) {
    int64_t uu, ii;
    float rv;
    std::memcpy(&uu, rec + 20 * i, 8);
    std::memcpy(&ii, rec + 20 * i + 8, 8);
    std::memcpy(&rv, rec + 20 * i + 16, 4);
    u[i] = static_cast<int32_t>(uu);
    it[i] = static_cast<int32_t>(ii);
    r[i] = rv;
  }
  oap_als_result* res = nullptr;
  if (!check(env, oap_als_fit(g_ctx, u.data(), it.data(), r.data(), n, rank, max_iter, reg, alpha,
                              1, static_cast<uint64_t>(seed), &res)))
    return 0;
  auto factors = [&](int which) {
    const int64_t cnt = oap_als_result_count(res, which);
    const int32_t* ids = oap_als_result_ids(res, which);
    const float* f = oap_als_result_factors(res, which);
    auto* t = new RowTable;
    t->rows = cnt;
    t->cols = 1 + rank;
    t->data.resize(size_t(cnt) * (1 + rank));
    for (int64_t i = 0; i < cnt; ++i) {
      t->data[size_t(i) * (1 + rank)] = ids[i];
      for (int j = 0; j < rank; ++j) t->data[size_t(i) * (1 + rank) + 1 + j] = f[i * rank + j];
    }
    return reinterpret_cast<jlong>(t);
  };
  set_int(env, result, "rankId", oap_ctx_rank(g_ctx));
  set_long(env, result, "cUsersFactorsNumTab", factors(0));
  set_long(env, result, "cItemsFactorsNumTab", factors(1));
  set_long(env, result, "cUserOffset", 0);  // ids travel inside the tables (no range offsets)
  set_long(env, result, "cItemOffset", 0);
  oap_als_result_free(res);
  return 0;
}

}  // extern "C"
