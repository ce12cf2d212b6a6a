// Parallel text readers (dense CSV, LIBSVM, "u::i::r" ratings) — see text_reader.cpp.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "runtime/thread_pool.h"

namespace oap {

struct DenseText {
  int64_t rows = 0;
  int cols = 0;
  std::vector<double> values;  // rows x cols, row-major
};

struct LibSvmText {  // CSR with zero-based column indices
  std::vector<double> labels;
  std::vector<int64_t> indptr;
  std::vector<int32_t> indices;
  std::vector<double> values;
  int64_t max_index = 0;  // largest one-based index seen
};

struct RatingsText {
  std::vector<int32_t> users, items;
  std::vector<float> ratings;  // 1.0 when the line has no rating field
};

DenseText read_csv_dense(const std::string& path, char sep, ThreadPool& pool);
LibSvmText read_libsvm(const std::string& path, ThreadPool& pool);
RatingsText read_ratings(const std::string& path, const std::string& sep, ThreadPool& pool);

}  // namespace oap
