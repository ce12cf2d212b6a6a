// Text-reader bindings (numpy arrays out; the GIL is released while parsing).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "bindings/bindings.h"
#include "io/text_reader.h"

namespace py = pybind11;
using namespace oap;

namespace {
template <class T>
py::array_t<T> arr(const std::vector<T>& v) {
  py::array_t<T> a(int64_t(v.size()));
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}
}  // namespace

void register_io(py::module_& m) {
  m.def(
      "read_csv",
      [](const std::string& path, const std::string& sep, int threads) {
        DenseText t;
        {
          py::gil_scoped_release rel;
          ThreadPool pool(threads > 0 ? threads : 1);
          t = read_csv_dense(path, sep.empty() ? ',' : sep[0], pool);
        }
        py::array_t<double> a({t.rows, int64_t(t.cols)});
        if (!t.values.empty()) std::memcpy(a.mutable_data(), t.values.data(), t.values.size() * 8);
        return a;
      },
      py::arg("path"), py::arg("sep") = ",", py::arg("threads") = 8);
  m.def(
      "read_libsvm",
      [](const std::string& path, int threads) {
        LibSvmText t;
        {
          py::gil_scoped_release rel;
          ThreadPool pool(threads > 0 ? threads : 1);
          t = read_libsvm(path, pool);
        }
        return py::make_tuple(arr(t.labels), arr(t.indptr), arr(t.indices), arr(t.values),
                              t.max_index);
      },
      py::arg("path"), py::arg("threads") = 8);
  m.def(
      "read_ratings",
      [](const std::string& path, const std::string& sep, int threads) {
        RatingsText t;
        {
          py::gil_scoped_release rel;
          ThreadPool pool(threads > 0 ? threads : 1);
          t = read_ratings(path, sep, pool);
        }
        return py::make_tuple(arr(t.users), arr(t.items), arr(t.ratings));
      },
      py::arg("path"), py::arg("sep") = "::", py::arg("threads") = 8);
}
