// Drives the JNI shim (csrc/jni/oap_jni.cpp) on the CPU engine through a fake, type-checking
// JNIEnv (no JVM in the container).  Objects of the reference's result / param classes declare
// exactly the fields of the reference's Java sources (mllib-dal/src/main/java/org/apache/spark/
// ml/{clustering/KMeansResult, feature/PCAResult, recommendation/ALSResult,
// recommendation/ALSPartitionInfo, util/CCLParam}.java): GetFieldID with a wrong name or type
// signature returns NULL and records a NoSuchFieldError, as a real VM does, and the harness fails.
// Prints "JNI_HARNESS_OK" on success.
#include <jni.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include <sys/wait.h>
#include <unistd.h>

// ---------------------------------------------------------------- fake VM objects
struct _jfieldID {
  std::string name, sig;
};

struct FakeObject : _jobject {
  std::string cls;
  std::map<std::string, std::string> decl;  // field -> JNI type signature
  std::map<std::string, double> vals;       // field -> value (as double; longs < 2^53 here)
};
struct FakeString : _jobject {
  std::string s;
};
struct FakeDoubles : _jobject {
  std::vector<double> v;
};
struct FakeFloats : _jobject {
  std::vector<float> v;
};
struct FakeLongs : _jobject {
  std::vector<jlong> v;
};
struct FakeBuffer : _jobject {
  void* addr = nullptr;
  jlong cap = 0;
};

static std::vector<std::string> g_errors;
static std::vector<_jfieldID*> g_fids;

#define REQUIRE(c)                                                          \
  do {                                                                      \
    if (!(c)) {                                                             \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

FakeObject* make_obj(const std::string& cls) {
  auto* o = new FakeObject;
  o->cls = cls;
  if (cls == "CCLParam") o->decl = {{"commSize", "J"}, {"rankId", "J"}};
  if (cls == "KMeansResult") o->decl = {{"iterationNum", "I"}, {"totalCost", "D"}};
  if (cls == "PCAResult")
    o->decl = {{"pcNumericTable", "J"}, {"explainedVarianceNumericTable", "J"}};
  if (cls == "ALSResult")
    o->decl = {{"rankId", "J"}, {"cUsersFactorsNumTab", "J"}, {"cItemsFactorsNumTab", "J"},
               {"cUserOffset", "J"}, {"cItemOffset", "J"}};
  if (cls == "ALSPartitionInfo") o->decl = {{"ratingsNum", "I"}, {"csrRowNum", "I"}};
  return o;
}

jclass JNIEnv::FindClass(const char* name) { return make_obj(name); }
jint JNIEnv::ThrowNew(jclass, const char* msg) {
  g_errors.push_back(std::string("RuntimeException: ") + msg);
  return 0;
}
jclass JNIEnv::GetObjectClass(jobject o) { return o; }
jfieldID JNIEnv::GetFieldID(jclass c, const char* name, const char* sig) {
  auto* o = dynamic_cast<FakeObject*>(c);
  REQUIRE(o);
  auto it = o->decl.find(name);
  if (it == o->decl.end() || it->second != sig) {
    g_errors.push_back(std::string("NoSuchFieldError: ") + o->cls + "." + name + " " + sig);
    return nullptr;
  }
  g_fids.push_back(new _jfieldID{name, sig});
  return g_fids.back();
}
static void set_field(jobject o, jfieldID f, const char* sig, double v) {
  auto* ob = dynamic_cast<FakeObject*>(o);
  REQUIRE(ob && f && f->sig == sig);
  ob->vals[f->name] = v;
}
void JNIEnv::SetIntField(jobject o, jfieldID f, jint v) { set_field(o, f, "I", v); }
void JNIEnv::SetLongField(jobject o, jfieldID f, jlong v) { set_field(o, f, "J", double(v)); }
void JNIEnv::SetDoubleField(jobject o, jfieldID f, jdouble v) { set_field(o, f, "D", v); }
jstring JNIEnv::NewStringUTF(const char* s) {
  auto* o = new FakeString;
  o->s = s;
  return o;
}
const char* JNIEnv::GetStringUTFChars(jstring s, jboolean*) {
  return dynamic_cast<FakeString*>(s)->s.c_str();
}
void JNIEnv::ReleaseStringUTFChars(jstring, const char*) {}
jsize JNIEnv::GetArrayLength(jarray a) {
  if (auto* d = dynamic_cast<FakeDoubles*>(a)) return jsize(d->v.size());
  if (auto* f = dynamic_cast<FakeFloats*>(a)) return jsize(f->v.size());
  if (auto* l = dynamic_cast<FakeLongs*>(a)) return jsize(l->v.size());
  REQUIRE(false);
  return 0;
}
void JNIEnv::GetDoubleArrayRegion(jdoubleArray a, jsize s, jsize n, jdouble* out) {
  auto* d = dynamic_cast<FakeDoubles*>(a);
  REQUIRE(d && s >= 0 && size_t(s + n) <= d->v.size());
  std::memcpy(out, d->v.data() + s, sizeof(double) * n);
}
void JNIEnv::GetFloatArrayRegion(jfloatArray a, jsize s, jsize n, jfloat* out) {
  auto* d = dynamic_cast<FakeFloats*>(a);
  REQUIRE(d && s >= 0 && size_t(s + n) <= d->v.size());
  std::memcpy(out, d->v.data() + s, sizeof(float) * n);
}
void JNIEnv::GetLongArrayRegion(jlongArray a, jsize s, jsize n, jlong* out) {
  auto* d = dynamic_cast<FakeLongs*>(a);
  REQUIRE(d && s >= 0 && size_t(s + n) <= d->v.size());
  std::memcpy(out, d->v.data() + s, sizeof(jlong) * n);
}
jdoubleArray JNIEnv::NewDoubleArray(jsize n) {
  auto* d = new FakeDoubles;
  d->v.assign(size_t(n), 0.0);
  return d;
}
void JNIEnv::SetDoubleArrayRegion(jdoubleArray a, jsize s, jsize n, const jdouble* in) {
  auto* d = dynamic_cast<FakeDoubles*>(a);
  REQUIRE(d && size_t(s + n) <= d->v.size());
  std::memcpy(d->v.data() + s, in, sizeof(double) * n);
}
void* JNIEnv::GetDirectBufferAddress(jobject b) { return dynamic_cast<FakeBuffer*>(b)->addr; }
jlong JNIEnv::GetDirectBufferCapacity(jobject b) { return dynamic_cast<FakeBuffer*>(b)->cap; }
jobject JNIEnv::NewDirectByteBuffer(void* p, jlong cap) {
  auto* b = new FakeBuffer;
  b->addr = p;
  b->cap = cap;
  return b;
}

// ---------------------------------------------------------------- the shim's entry points
extern "C" {
jint Java_org_apache_spark_ml_util_OneCCL_00024_c_1init(JNIEnv*, jobject, jint, jint, jstring,
                                                       jobject);
void Java_org_apache_spark_ml_util_OneCCL_00024_c_1cleanup(JNIEnv*, jobject);
jboolean Java_org_apache_spark_ml_util_OneCCL_00024_isRoot(JNIEnv*, jobject);
jint Java_org_apache_spark_ml_util_OneCCL_00024_rankID(JNIEnv*, jobject);
jint Java_org_apache_spark_ml_util_OneCCL_00024_setEnv(JNIEnv*, jobject, jstring, jstring,
                                                      jboolean);
jint Java_org_apache_spark_ml_util_OneCCL_00024_c_1getAvailPort(JNIEnv*, jobject, jstring);
jlong Java_org_apache_spark_ml_util_OneDAL_00024_cNewRowTable(JNIEnv*, jobject, jlong, jint);
void Java_org_apache_spark_ml_util_OneDAL_00024_setNumericTableValue(JNIEnv*, jobject, jlong, jint,
                                                                    jint, jdouble);
void Java_org_apache_spark_ml_util_OneDAL_00024_cSetDoubleBatch(JNIEnv*, jobject, jlong, jint,
                                                               jdoubleArray, jint, jint);
void Java_org_apache_spark_ml_util_OneDAL_00024_cAddNumericTable(JNIEnv*, jobject, jlong, jlong);
void Java_org_apache_spark_ml_util_OneDAL_00024_cFreeDataMemory(JNIEnv*, jobject, jlong);
void Java_org_apache_spark_ml_util_OneDAL_00024_cFreeCSRTable(JNIEnv*, jobject, jlong);
jlong Java_org_apache_spark_ml_util_OneDAL_00024_cNewCSRNumericTable(JNIEnv*, jobject, jfloatArray,
                                                                    jlongArray, jlongArray, jlong,
                                                                    jlong);
jlong Java_org_apache_spark_ml_util_OneDAL_00024_cNumRows(JNIEnv*, jobject, jlong);
jint Java_org_apache_spark_ml_util_OneDAL_00024_cNumCols(JNIEnv*, jobject, jlong);
jdoubleArray Java_org_apache_spark_ml_util_OneDAL_00024_cGetDoubleArray(JNIEnv*, jobject, jlong);
jboolean Java_org_apache_spark_ml_util_OneDAL_00024_cCheckPlatformCompatibility(JNIEnv*, jobject);
jlong Java_org_apache_spark_ml_clustering_KMeansDALImpl_cKMeansDALComputeWithInitCenters(
    JNIEnv*, jobject, jlong, jlong, jint, jdouble, jint, jint, jint, jobject);
jlong Java_org_apache_spark_ml_feature_PCADALImpl_cPCATrainDAL(JNIEnv*, jobject, jlong, jint, jint,
                                                               jint, jobject);
jobject Java_org_apache_spark_ml_recommendation_ALSDALImpl_cShuffleData(JNIEnv*, jobject, jobject,
                                                                        jint, jint, jobject);
jlong Java_org_apache_spark_ml_recommendation_ALSDALImpl_cDALImplictALS(JNIEnv*, jobject, jlong,
                                                                        jlong, jint, jint, jdouble,
                                                                        jdouble, jint, jint, jint,
                                                                        jobject);
}

static jlong table_from(JNIEnv* env, const std::vector<double>& rows, int cols) {
  const jlong n = jlong(rows.size() / cols);
  const jlong h = Java_org_apache_spark_ml_util_OneDAL_00024_cNewRowTable(env, nullptr, n, cols);
  auto* batch = new FakeDoubles;
  batch->v = rows;
  Java_org_apache_spark_ml_util_OneDAL_00024_cSetDoubleBatch(env, nullptr, h, 0, batch, jint(n),
                                                            cols);
  return h;
}

static std::vector<double> table_values(JNIEnv* env, jlong h) {
  return dynamic_cast<FakeDoubles*>(
             Java_org_apache_spark_ml_util_OneDAL_00024_cGetDoubleArray(env, nullptr, h))
      ->v;
}

// ---- a 2-process world through the reference's KVS string: c_init(2, r, "127.0.0.1_<port>")
// (OneCCL.scala:32-46 -> OneCCL.cpp:47-86), then K-Means on each rank's half of a 3-blob
// dataset from the same initial centers; both ranks must return the single-process centers.
static std::vector<double> blobs3(int n) {
  std::vector<double> X;
  for (int i = 0; i < n; ++i) {
    const int c = i % 3;
    for (int j = 0; j < 3; ++j)
      X.push_back(10.0 * c + j + 0.01 * double((i * 37 + j * 11) % 17) - 0.08);
  }
  return X;
}

static std::vector<double> kmeans_rank(JNIEnv* env, int world, int rank, const std::string& kvs,
                                       double* cost) {
  FakeObject* param = make_obj("CCLParam");
  auto* ipport = new FakeString;
  ipport->s = kvs;
  REQUIRE(Java_org_apache_spark_ml_util_OneCCL_00024_c_1init(env, nullptr, world, rank, ipport,
                                                             param) == 0);
  REQUIRE(g_errors.empty());
  REQUIRE(param->vals.at("commSize") == world && param->vals.at("rankId") == rank);
  const int n = 300;
  const std::vector<double> X = blobs3(n);
  std::vector<double> mine;
  for (int i = rank; i < n; i += world)  // a strided (non-range) partition
    mine.insert(mine.end(), X.begin() + 3 * i, X.begin() + 3 * i + 3);
  const jlong xt = table_from(env, mine, 3);
  const jlong ct = table_from(env, std::vector<double>(X.begin(), X.begin() + 9), 3);
  FakeObject* kres = make_obj("KMeansResult");
  const jlong centers =
      Java_org_apache_spark_ml_clustering_KMeansDALImpl_cKMeansDALComputeWithInitCenters(
          env, nullptr, xt, ct, 3, 1e-6, 20, world, 1, kres);
  REQUIRE(g_errors.empty() && centers != 0);
  *cost = kres->vals.at("totalCost");
  std::vector<double> cv = table_values(env, centers);
  for (jlong h : {xt, ct, centers})
    Java_org_apache_spark_ml_util_OneDAL_00024_cFreeDataMemory(env, nullptr, h);
  Java_org_apache_spark_ml_util_OneCCL_00024_c_1cleanup(env, nullptr);
  return cv;
}

static int world2(const char* port) {
  const std::string kvs = std::string("127.0.0.1_") + port;
  int fds[2][2];
  pid_t pid[2];
  for (int r = 0; r < 2; ++r) {  // fork before anything initialises a runtime
    REQUIRE(pipe(fds[r]) == 0);
    pid[r] = fork();
    REQUIRE(pid[r] >= 0);
    if (pid[r] == 0) {
      close(fds[r][0]);
      JNIEnv e;
      double cost = 0.0;
      std::vector<double> cv = kmeans_rank(&e, 2, r, kvs, &cost);
      cv.push_back(cost);
      const ssize_t w = write(fds[r][1], cv.data(), cv.size() * sizeof(double));
      _exit(w == ssize_t(cv.size() * sizeof(double)) ? 0 : 3);
    }
    close(fds[r][1]);
  }
  std::vector<double> got[2];
  for (int r = 0; r < 2; ++r) {
    got[r].resize(10);
    size_t off = 0;
    while (off < 10 * sizeof(double)) {
      const ssize_t n = read(fds[r][0], reinterpret_cast<char*>(got[r].data()) + off,
                             10 * sizeof(double) - off);
      if (n <= 0) break;
      off += size_t(n);
    }
    int st = 0;
    waitpid(pid[r], &st, 0);
    REQUIRE(WIFEXITED(st) && WEXITSTATUS(st) == 0 && off == 10 * sizeof(double));
  }
  JNIEnv e;
  double cost1 = 0.0;
  std::vector<double> one = kmeans_rank(&e, 1, 0, kvs, &cost1);
  for (int r = 0; r < 2; ++r) {
    for (int j = 0; j < 9; ++j) REQUIRE(std::fabs(got[r][j] - one[j]) < 1e-12);
    REQUIRE(std::fabs(got[r][9] - cost1) < 1e-9 * (1.0 + cost1));
  }
  std::printf("JNI_WORLD2_OK\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 3 && std::string(argv[1]) == "world2") return world2(argv[2]);
  JNIEnv env_obj;
  JNIEnv* env = &env_obj;

  // ---- OneCCL$: world of one on the CPU engine; CCLParam's fields are longs
  FakeObject* param = make_obj("CCLParam");
  auto* ipport = new FakeString;
  ipport->s = "127.0.0.1_3000";
  REQUIRE(Java_org_apache_spark_ml_util_OneCCL_00024_c_1init(env, nullptr, 1, 0, ipport, param) ==
          0);
  REQUIRE(g_errors.empty());
  REQUIRE(param->vals.at("commSize") == 1 && param->vals.at("rankId") == 0);
  REQUIRE(Java_org_apache_spark_ml_util_OneCCL_00024_isRoot(env, nullptr));
  REQUIRE(Java_org_apache_spark_ml_util_OneCCL_00024_rankID(env, nullptr) == 0);
  auto *k = new FakeString, *v = new FakeString;
  k->s = "OAP_JNI_HARNESS_ENV";
  v->s = "ofi";
  REQUIRE(Java_org_apache_spark_ml_util_OneCCL_00024_setEnv(env, nullptr, k, v, 1) == 0);
  REQUIRE(std::string(std::getenv("OAP_JNI_HARNESS_ENV")) == "ofi");
  auto* lo = new FakeString;
  lo->s = "127.0.0.1";
  const jint port = Java_org_apache_spark_ml_util_OneCCL_00024_c_1getAvailPort(env, nullptr, lo);
  REQUIRE(port >= 3000 && port < 65535);
  auto* bad = new FakeString;
  bad->s = "203.0.113.7";  // TEST-NET-3: never a local address
  REQUIRE(Java_org_apache_spark_ml_util_OneCCL_00024_c_1getAvailPort(env, nullptr, bad) == -1);
  (void)Java_org_apache_spark_ml_util_OneDAL_00024_cCheckPlatformCompatibility(env, nullptr);

  // ---- K-Means on the reference example (examples/data/sample_kmeans_data.txt, 6 x 3)
  const std::vector<double> X = {0.0, 0.0, 0.0, 0.1, 0.1, 0.1, 0.2, 0.2, 0.2,
                                 9.0, 9.0, 9.0, 9.1, 9.1, 9.1, 9.2, 9.2, 9.2};
  const jlong xt = table_from(env, X, 3);
  const jlong ct = Java_org_apache_spark_ml_util_OneDAL_00024_cNewRowTable(env, nullptr, 2, 3);
  for (int j = 0; j < 3; ++j) {  // initial centers = rows 0 and 3, one value per call
    Java_org_apache_spark_ml_util_OneDAL_00024_setNumericTableValue(env, nullptr, ct, 0, j, X[j]);
    Java_org_apache_spark_ml_util_OneDAL_00024_setNumericTableValue(env, nullptr, ct, 1, j,
                                                                   X[9 + j]);
  }
  FakeObject* kres = make_obj("KMeansResult");
  const jlong centers =
      Java_org_apache_spark_ml_clustering_KMeansDALImpl_cKMeansDALComputeWithInitCenters(
          env, nullptr, xt, ct, 2, 1e-4, 10, 1, 1, kres);
  REQUIRE(g_errors.empty() && centers != 0);
  REQUIRE(kres->vals.at("iterationNum") >= 1);
  REQUIRE(std::fabs(kres->vals.at("totalCost") - 0.12) < 1e-9);
  const auto cv = table_values(env, centers);
  REQUIRE(cv.size() == 6 && std::fabs(cv[0] - 0.1) < 1e-12 && std::fabs(cv[3] - 9.1) < 1e-12);

  // ---- PCA on the reference toy data (examples/data/pca_data.csv semantics: 3 x 5)
  const std::vector<double> P = {0.0, 1.0, 0.0, 7.0, 0.0, 2.0, 0.0, 3.0, 4.0, 5.0,
                                 4.0, 0.0, 0.0, 6.0, 7.0};
  const jlong pt = table_from(env, P, 5);
  FakeObject* pres = make_obj("PCAResult");
  Java_org_apache_spark_ml_feature_PCADALImpl_cPCATrainDAL(env, nullptr, pt, 2, 1, 1, pres);
  REQUIRE(g_errors.empty());
  const auto ev = table_values(env, jlong(pres->vals.at("explainedVarianceNumericTable")));
  REQUIRE(ev.size() == 2 && ev[0] >= ev[1] && ev[0] + ev[1] <= 1.0 + 1e-12 && ev[0] > 0.5);
  REQUIRE(Java_org_apache_spark_ml_util_OneDAL_00024_cNumRows(
              env, nullptr, jlong(pres->vals.at("pcNumericTable"))) == 5);

  // ---- ALS: the reference's transposed records {item, user, rating}, shuffle, CSR, train
  const int n_users = 6, n_items = 4;
  std::vector<unsigned char> recs;
  int n_r = 0;
  for (int u = 0; u < n_users; ++u)
    for (int i = 0; i < n_items; ++i) {
      if ((u + i) % 3 == 0) continue;
      const int64_t key = i, other = u;
      const float r = float(1 + (u * 7 + i) % 5);
      unsigned char b[20];
      std::memcpy(b, &key, 8);
      std::memcpy(b + 8, &other, 8);
      std::memcpy(b + 16, &r, 4);
      recs.insert(recs.end(), b, b + 20);
      ++n_r;
    }
  auto* buf = new FakeBuffer;
  buf->addr = recs.data();
  buf->cap = jlong(recs.size());
  FakeObject* info = make_obj("ALSPartitionInfo");
  auto* shuffled = dynamic_cast<FakeBuffer*>(
      Java_org_apache_spark_ml_recommendation_ALSDALImpl_cShuffleData(env, nullptr, buf, n_items,
                                                                      1, info));
  REQUIRE(g_errors.empty() && shuffled && shuffled->cap == 20 * n_r);
  REQUIRE(info->vals.at("ratingsNum") == n_r && info->vals.at("csrRowNum") == n_items);
  // bufferToCSRNumericTable (ALSDALImpl.scala:184-230): 1-based CSR, rows = keys
  auto* vals = new FakeFloats;
  auto *cols = new FakeLongs, *offs = new FakeLongs;
  offs->v.push_back(1);
  int64_t cur = 0;
  const auto* sb = static_cast<const unsigned char*>(shuffled->addr);
  for (int i = 0; i < n_r; ++i) {
    int64_t key, other;
    float r;
    std::memcpy(&key, sb + 20 * i, 8);
    std::memcpy(&other, sb + 20 * i + 8, 8);
    std::memcpy(&r, sb + 20 * i + 16, 4);
    REQUIRE(key >= cur);  // sorted by key
    if (key > cur) {
      cur = key;
      offs->v.push_back(i + 1);
    }
    vals->v.push_back(r);
    cols->v.push_back(other + 1);
  }
  offs->v.push_back(n_r + 1);
  const jlong csr = Java_org_apache_spark_ml_util_OneDAL_00024_cNewCSRNumericTable(
      env, nullptr, vals, cols, offs, n_users, n_items);
  REQUIRE(g_errors.empty() && csr != 0);
  FakeObject* ares = make_obj("ALSResult");
  Java_org_apache_spark_ml_recommendation_ALSDALImpl_cDALImplictALS(env, nullptr, csr, n_users, 3,
                                                                    5, 0.01, 40.0, 1, 1, 0, ares);
  REQUIRE(g_errors.empty());
  REQUIRE(ares->vals.at("rankId") == 0 && ares->vals.at("cUserOffset") == 0 &&
          ares->vals.at("cItemOffset") == 0);
  const jlong uf = jlong(ares->vals.at("cUsersFactorsNumTab"));
  const jlong itf = jlong(ares->vals.at("cItemsFactorsNumTab"));
  REQUIRE(Java_org_apache_spark_ml_util_OneDAL_00024_cNumRows(env, nullptr, uf) == n_users);
  REQUIRE(Java_org_apache_spark_ml_util_OneDAL_00024_cNumRows(env, nullptr, itf) == n_items);
  REQUIRE(Java_org_apache_spark_ml_util_OneDAL_00024_cNumCols(env, nullptr, uf) == 3);
  const auto U = table_values(env, uf), I = table_values(env, itf);
  double fit_pos = 0.0, fit_neg = 0.0;
  int npos = 0, nneg = 0;
  for (int u = 0; u < n_users; ++u)
    for (int i = 0; i < n_items; ++i) {
      double p = 0.0;
      for (int j = 0; j < 3; ++j) p += U[u * 3 + j] * I[i * 3 + j];
      if ((u + i) % 3 == 0) {
        fit_neg += p;
        ++nneg;
      } else {
        fit_pos += p;
        ++npos;
      }
    }
  REQUIRE(fit_pos / npos > fit_neg / nneg);  // implicit preference: observed pairs score higher

  // ---- bufferToCSRNumericTable's leading empty row (ALSDALImpl.scala:198-222): a partition
  // whose lowest key is unrated emits offsets [1, 1, ...] (csrRowNum + 2 entries); an empty
  // partition emits [1, 1] with csrRowNum = 0
  {
    auto* v2 = new FakeFloats;
    auto *c2 = new FakeLongs, *o2 = new FakeLongs;
    v2->v = {1.f, 2.f, 3.f};
    c2->v = {1, 3, 2};
    o2->v = {1, 1, 3, 4};  // leading empty row, then rows {1,3} and {2}
    const jlong h2 = Java_org_apache_spark_ml_util_OneDAL_00024_cNewCSRNumericTable(
        env, nullptr, v2, c2, o2, 3, 2);
    REQUIRE(g_errors.empty() && h2 != 0);
    Java_org_apache_spark_ml_util_OneDAL_00024_cFreeCSRTable(env, nullptr, h2);
    auto* v3 = new FakeFloats;
    auto *c3 = new FakeLongs, *o3 = new FakeLongs;
    o3->v = {1, 1};
    const jlong h3 = Java_org_apache_spark_ml_util_OneDAL_00024_cNewCSRNumericTable(
        env, nullptr, v3, c3, o3, 3, 0);
    REQUIRE(g_errors.empty() && h3 != 0);
    Java_org_apache_spark_ml_util_OneDAL_00024_cFreeCSRTable(env, nullptr, h3);
    auto* o4 = new FakeLongs;
    o4->v = {1, 2, 3, 4};  // rows + 2 entries without the leading empty row: rejected
    Java_org_apache_spark_ml_util_OneDAL_00024_cNewCSRNumericTable(env, nullptr, v2, c2, o4, 3,
                                                                  2);
    REQUIRE(!g_errors.empty());
    g_errors.clear();
  }

  // ---- a wrong field type is caught like a real VM would (NoSuchFieldError, nothing written)
  FakeObject* wrong = make_obj("KMeansResult");
  wrong->decl["iterationNum"] = "J";
  g_errors.clear();
  Java_org_apache_spark_ml_clustering_KMeansDALImpl_cKMeansDALComputeWithInitCenters(
      env, nullptr, xt, ct, 2, 1e-4, 10, 1, 1, wrong);
  REQUIRE(!g_errors.empty() && wrong->vals.empty());

  Java_org_apache_spark_ml_util_OneDAL_00024_cFreeCSRTable(env, nullptr, csr);
  for (jlong h : {xt, ct, pt, centers, uf, itf})
    Java_org_apache_spark_ml_util_OneDAL_00024_cFreeDataMemory(env, nullptr, h);
  Java_org_apache_spark_ml_util_OneCCL_00024_c_1cleanup(env, nullptr);
  std::printf("JNI_HARNESS_OK\n");
  return 0;
}
