// Registration hooks for the per-algorithm binding units.
#pragma once

#include <pybind11/pybind11.h>

namespace oap {
namespace py_bind {

}  // namespace py_bind
}  // namespace oap

void register_pca(pybind11::module_& m);
void register_als(pybind11::module_& m);
void register_io(pybind11::module_& m);
