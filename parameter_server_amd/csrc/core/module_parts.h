// Registration hooks: each translation unit of the host runtime adds its own
// bindings to the _pscore module.
#pragma once
#include <pybind11/pybind11.h>

namespace pscore {
void register_util(pybind11::module_& m);
void register_data(pybind11::module_& m);
void register_runtime(pybind11::module_& m);
void register_setops(pybind11::module_& m);
}  // namespace pscore
