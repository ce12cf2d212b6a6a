#include "bindings/bindings.h"

void register_als(pybind11::module_& m) { (void)m; }
