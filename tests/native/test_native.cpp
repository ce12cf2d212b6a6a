// Host-side native unit tests, built with AddressSanitizer+UBSan and with ThreadSanitizer by
// tests/test_native_sanitizers.py (SURVEY.md §5 "race detection / sanitizers").  Covers the
// pure-C++ parts of the runtime: the thread pool (partitioning, exception propagation, reuse),
// the symmetric eigensolver and the parallel text readers.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "io/text_reader.h"
#include "linalg/eigen.h"
#include "runtime/thread_pool.h"

static int failures = 0;
#define EXPECT(cond)                                                      \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

static void test_thread_pool() {
  for (int threads : {1, 2, 3, 8}) {
    oap::ThreadPool pool(threads);
    for (int64_t n : {0, 1, 2, 7, 1000, 100003}) {
      std::vector<std::atomic<int>> hit(static_cast<size_t>(n));
      for (auto& h : hit) h.store(0);
      pool.parallel_for(n, [&](int chunk, int64_t b, int64_t e) {
        EXPECT(chunk >= 0 && chunk < pool.size());
        for (int64_t i = b; i < e; ++i) hit[size_t(i)].fetch_add(1);
      });
      for (auto& h : hit) EXPECT(h.load() == 1);
    }
    // exceptions from any chunk surface after all chunks are done; the pool stays usable
    for (int rep = 0; rep < 3; ++rep) {
      bool caught = false;
      try {
        pool.parallel_for(64, [&](int, int64_t b, int64_t) {
          if (b >= 32) throw std::runtime_error("boom");
        });
      } catch (const std::runtime_error&) {
        caught = true;
      }
      EXPECT(caught == (threads > 1));
      std::atomic<int64_t> sum{0};
      pool.parallel_for(1000, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) sum += i;
      });
      EXPECT(sum.load() == 999 * 1000 / 2);
    }
  }
}

static void test_eigen() {
  std::mt19937_64 rng(7);
  std::normal_distribution<double> g;
  oap::ThreadPool pool(4);
  for (int n : {1, 2, 5, 33, 90}) {
    std::vector<double> A(size_t(n) * n);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j <= i; ++j) A[size_t(i) * n + j] = A[size_t(j) * n + i] = g(rng);
    for (int k : {1, n}) {
      oap::SymEig e = oap::sym_eig_topk(A, n, k, &pool);
      EXPECT(int(e.values.size()) == n);
      double res = 0.0, orth = 0.0;
      for (int c = 0; c < k; ++c) {
        for (int i = 0; i < n; ++i) {
          double s = 0.0;
          for (int j = 0; j < n; ++j) s += A[size_t(i) * n + j] * e.vectors[size_t(j) * k + c];
          res = std::max(res, std::fabs(s - e.values[c] * e.vectors[size_t(i) * k + c]));
        }
        for (int c2 = 0; c2 < k; ++c2) {
          double s = 0.0;
          for (int i = 0; i < n; ++i)
            s += e.vectors[size_t(i) * k + c] * e.vectors[size_t(i) * k + c2];
          orth = std::max(orth, std::fabs(s - (c == c2 ? 1.0 : 0.0)));
        }
      }
      EXPECT(res < 1e-10 * n);
      EXPECT(orth < 1e-10);
      for (int i = 1; i < n; ++i) EXPECT(std::fabs(e.values[i - 1]) >= std::fabs(e.values[i]));
    }
  }
}

static void test_readers(const std::string& dir) {
  oap::ThreadPool pool(3);
  const std::string csv = dir + "/t.csv";
  {
    std::ofstream f(csv);
    for (int i = 0; i < 500; ++i) f << i << "," << i * 0.5 << ",-" << i << "\n";
  }
  oap::DenseText t = oap::read_csv_dense(csv, ',', pool);
  EXPECT(t.rows == 500 && t.cols == 3);
  bool ok = true;
  for (int i = 0; i < 500; ++i)
    ok = ok && t.values[size_t(i) * 3] == i && t.values[size_t(i) * 3 + 1] == i * 0.5 &&
         t.values[size_t(i) * 3 + 2] == -i;
  EXPECT(ok);
  const std::string svm = dir + "/t.svm";
  {
    std::ofstream f(svm);
    f << "1 1:2 4:3\n\n0 2:1.5\n";
  }
  oap::LibSvmText s = oap::read_libsvm(svm, pool);
  EXPECT(s.labels.size() == 2 && s.indptr.size() == 3 && s.max_index == 4);
  EXPECT(s.indices.size() == 3 && s.indices[1] == 3 && s.values[2] == 1.5);
  const std::string rat = dir + "/t.ratings";
  {
    std::ofstream f(rat);
    for (int i = 0; i < 100; ++i) f << i << "::" << i + 1 << "::" << i * 0.25 << "\n";
  }
  oap::RatingsText r = oap::read_ratings(rat, "::", pool);
  EXPECT(r.users.size() == 100 && r.items[10] == 11 && r.ratings[8] == 2.0f);
  // files shorter than the thread count: early line cuts fall on byte 0 (the splitter must not
  // read the byte before the mapping — ASan catches it here)
  oap::ThreadPool wide(8);
  const std::string tiny = dir + "/tiny.csv";
  {
    std::ofstream f(tiny);
    f << "1,2\n";
  }
  oap::DenseText tt = oap::read_csv_dense(tiny, ',', wide);
  EXPECT(tt.rows == 1 && tt.cols == 2 && tt.values[1] == 2.0);
  bool threw = false;
  try {
    oap::read_csv_dense(dir + "/does-not-exist.csv", ',', pool);
  } catch (const std::exception&) {
    threw = true;
  }
  EXPECT(threw);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_thread_pool();
  test_eigen();
  test_readers(dir);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("native tests ok\n");
  return 0;
}
