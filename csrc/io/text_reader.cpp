// Parallel text readers: dense CSV, LIBSVM and "u<sep>i<sep>r" rating files.
//
// The reference's service utilities carry single-threaded CSV/CSR readers
// (mllib-dal/src/main/native/service.cpp:26-146) and the examples feed Spark's own
// "libsvm" / text readers (examples/data/sample_kmeans_data.txt, pca_data.csv,
// onedal_als_csr_ratings.txt).  Here a file is mapped once, split at line boundaries into one
// range per pool thread, parsed with strtod/strtol in place, and the per-thread pieces are
// concatenated in file order — the output does not depend on the thread count.
#include "io/text_reader.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "runtime/common.h"

namespace oap {

namespace {

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  explicit Mapped(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    OAP_CHECK(fd >= 0, "cannot open " << path << ": " << std::strerror(errno));
    struct stat st;
    OAP_CHECK(::fstat(fd, &st) == 0, "cannot stat " << path);
    n = size_t(st.st_size);
    if (n) {
      void* m = ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
      OAP_CHECK(m != MAP_FAILED, "cannot map " << path);
      p = static_cast<const char*>(m);
    }
  }
  ~Mapped() {
    if (p) ::munmap(const_cast<char*>(p), n);
    if (fd >= 0) ::close(fd);
  }
};

// Thread ranges [b, e) aligned to line starts.
std::vector<size_t> line_ranges(const Mapped& m, int parts) {
  std::vector<size_t> cut(parts + 1, m.n);
  cut[0] = 0;
  for (int t = 1; t < parts; ++t) {
    size_t pos = m.n * t / parts;
    if (pos < cut[t - 1]) pos = cut[t - 1];
    // (pos 0 is a line start: a file shorter than the thread count puts early cuts there —
    // reading m.p[-1] would touch the page before the mapping)
    while (pos > 0 && pos < m.n && m.p[pos - 1] != '\n') ++pos;
    cut[t] = pos;
  }
  return cut;
}

bool blank_or_comment(const char* s, const char* e) {
  while (s < e && (*s == ' ' || *s == '\t' || *s == '\r')) ++s;
  return s == e || *s == '#';
}

// strtod over [s, e): the mapped file is not NUL-terminated, so copy short tokens.
double parse_num(const char*& s, const char* e, bool& ok) {
  char buf[64];
  size_t k = 0;
  while (s < e && (*s == ' ' || *s == '\t')) ++s;
  while (s < e && k < sizeof(buf) - 1 && *s != ',' && *s != ' ' && *s != '\t' && *s != '\r' &&
         *s != ':' && *s != ';' && *s != '\n')
    buf[k++] = *s++;
  buf[k] = 0;
  char* end = nullptr;
  const double v = std::strtod(buf, &end);
  ok = k > 0 && end == buf + k;
  return v;
}

}  // namespace

DenseText read_csv_dense(const std::string& path, char sep, ThreadPool& pool) {
  Mapped m(path);
  const int parts = pool.size();
  const std::vector<size_t> cut = line_ranges(m, parts);
  std::vector<std::vector<double>> vals(parts);
  std::vector<int64_t> rows(parts, 0);
  std::vector<int> cols(parts, -1);
  std::vector<std::string> err(parts);
  pool.parallel_for(parts, [&](int, int64_t b, int64_t e) {
    for (int64_t t = b; t < e; ++t) {
      const char* s = m.p + cut[t];
      const char* end = m.p + cut[t + 1];
      while (s < end) {
        const char* nl = static_cast<const char*>(std::memchr(s, '\n', end - s));
        const char* le = nl ? nl : end;
        if (!blank_or_comment(s, le)) {
          int c = 0;
          const char* q = s;
          while (q < le) {
            bool ok;
            const double v = parse_num(q, le, ok);
            if (!ok) {
              err[t] = "bad number in " + path;
              return;
            }
            vals[t].push_back(v);
            ++c;
            while (q < le && (*q == sep || *q == ' ' || *q == '\t' || *q == '\r')) ++q;
          }
          if (cols[t] < 0) cols[t] = c;
          if (c != cols[t]) {
            err[t] = "ragged rows in " + path;
            return;
          }
          ++rows[t];
        }
        s = le + 1;
      }
    }
  });
  DenseText out;
  for (int t = 0; t < parts; ++t) {
    OAP_CHECK(err[t].empty(), err[t]);
    if (rows[t] == 0) continue;
    if (out.cols == 0) out.cols = cols[t];
    OAP_CHECK(cols[t] == out.cols, "ragged rows in " << path);
    out.values.insert(out.values.end(), vals[t].begin(), vals[t].end());
    out.rows += rows[t];
  }
  return out;
}

LibSvmText read_libsvm(const std::string& path, ThreadPool& pool) {
  Mapped m(path);
  const int parts = pool.size();
  const std::vector<size_t> cut = line_ranges(m, parts);
  std::vector<LibSvmText> piece(parts);
  std::vector<std::string> err(parts);
  pool.parallel_for(parts, [&](int, int64_t b, int64_t e) {
    for (int64_t t = b; t < e; ++t) {
      LibSvmText& P = piece[t];
      P.indptr.push_back(0);
      const char* s = m.p + cut[t];
      const char* end = m.p + cut[t + 1];
      while (s < end) {
        const char* nl = static_cast<const char*>(std::memchr(s, '\n', end - s));
        const char* le = nl ? nl : end;
        if (!blank_or_comment(s, le)) {
          const char* q = s;
          bool ok;
          P.labels.push_back(parse_num(q, le, ok));
          if (!ok) {
            err[t] = "bad label in " + path;
            return;
          }
          int64_t prev = 0;
          while (true) {
            while (q < le && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
            if (q >= le) break;
            const double idx = parse_num(q, le, ok);
            if (!ok || q >= le || *q != ':') {
              err[t] = "bad index:value pair in " + path;
              return;
            }
            ++q;
            const double v = parse_num(q, le, ok);
            if (!ok || idx < 1 || int64_t(idx) <= prev) {
              err[t] = "indices must be one-based and ascending in " + path;
              return;
            }
            prev = int64_t(idx);
            P.indices.push_back(int32_t(idx - 1));
            P.values.push_back(v);
            P.max_index = std::max<int64_t>(P.max_index, int64_t(idx));
          }
          P.indptr.push_back(int64_t(P.indices.size()));
        }
        s = le + 1;
      }
    }
  });
  LibSvmText out;
  out.indptr.push_back(0);
  for (int t = 0; t < parts; ++t) {
    OAP_CHECK(err[t].empty(), err[t]);
    const int64_t base = int64_t(out.indices.size());
    out.labels.insert(out.labels.end(), piece[t].labels.begin(), piece[t].labels.end());
    out.indices.insert(out.indices.end(), piece[t].indices.begin(), piece[t].indices.end());
    out.values.insert(out.values.end(), piece[t].values.begin(), piece[t].values.end());
    for (size_t i = 1; i < piece[t].indptr.size(); ++i)
      out.indptr.push_back(base + piece[t].indptr[i]);
    out.max_index = std::max(out.max_index, piece[t].max_index);
  }
  return out;
}

RatingsText read_ratings(const std::string& path, const std::string& sep, ThreadPool& pool) {
  Mapped m(path);
  const int parts = pool.size();
  const std::vector<size_t> cut = line_ranges(m, parts);
  std::vector<RatingsText> piece(parts);
  std::vector<std::string> err(parts);
  pool.parallel_for(parts, [&](int, int64_t b, int64_t e) {
    for (int64_t t = b; t < e; ++t) {
      const char* s = m.p + cut[t];
      const char* end = m.p + cut[t + 1];
      while (s < end) {
        const char* nl = static_cast<const char*>(std::memchr(s, '\n', end - s));
        const char* le = nl ? nl : end;
        if (!blank_or_comment(s, le)) {
          double f[3];
          const char* q = s;
          int k = 0;
          while (k < 3) {
            bool ok;
            const double v = parse_num(q, le, ok);
            if (!ok) break;
            f[k++] = v;
            if (size_t(le - q) >= sep.size() && std::memcmp(q, sep.data(), sep.size()) == 0)
              q += sep.size();
            else
              break;
          }
          if (k < 2) {
            err[t] = "bad rating line in " + path;
            return;
          }
          piece[t].users.push_back(int32_t(f[0]));
          piece[t].items.push_back(int32_t(f[1]));
          piece[t].ratings.push_back(k == 3 ? float(f[2]) : 1.f);
        }
        s = le + 1;
      }
    }
  });
  RatingsText out;
  for (int t = 0; t < parts; ++t) {
    OAP_CHECK(err[t].empty(), err[t]);
    out.users.insert(out.users.end(), piece[t].users.begin(), piece[t].users.end());
    out.items.insert(out.items.end(), piece[t].items.begin(), piece[t].items.end());
    out.ratings.insert(out.ratings.end(), piece[t].ratings.begin(), piece[t].ratings.end());
  }
  return out;
}

}  // namespace oap
