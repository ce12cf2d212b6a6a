#include "bindings/bindings.h"

void register_pca(pybind11::module_& m) { (void)m; }
