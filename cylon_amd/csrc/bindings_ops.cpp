// Bindings for the extended relational operators (set ops, unique, group-by,
// aggregates, range partition, distributed sort).
#include <torch/extension.h>

#include "cylon/kernels/kernels.hpp"
#include "cylon/ops/api_ext.hpp"
#include "cylon/ops/relational.hpp"
#include "cylon/table.hpp"

namespace py = pybind11;
using namespace cylon;

static std::vector<ops::AggSpec> make_specs(const std::vector<int> &cols, const std::vector<int> &op_ids,
                                            const std::vector<double> &qs, const std::vector<int> &ddofs) {
  CYLON_CHECK(cols.size() == op_ids.size(), Code::Invalid, "aggregate columns and ops differ in length");
  std::vector<ops::AggSpec> specs;
  for (size_t i = 0; i < cols.size(); ++i) {
    ops::AggSpec s{cols[i], op_ids[i]};
    if (i < qs.size()) s.quantile = qs[i];
    if (i < ddofs.size()) s.ddof = ddofs[i];
    specs.push_back(s);
  }
  return specs;
}

void register_extended_ops(py::module &m) {
  auto rel = py::call_guard<py::gil_scoped_release>();

  py::enum_<AggOp>(m, "AggregationOp")
      .value("SUM", AGG_SUM).value("MIN", AGG_MIN).value("MAX", AGG_MAX).value("COUNT", AGG_COUNT)
      .value("MEAN", AGG_MEAN).value("VAR", AGG_VAR).value("NUNIQUE", AGG_NUNIQUE)
      .value("QUANTILE", AGG_QUANTILE).value("STDDEV", AGG_STDDEV);

  m.def("union", &ops::Union, rel);
  m.def("subtract", &ops::Subtract, rel);
  m.def("intersect", &ops::Intersect, rel);
  m.def("distributed_union", &ops::DistributedUnion, rel);
  m.def("distributed_subtract", &ops::DistributedSubtract, rel);
  m.def("distributed_intersect", &ops::DistributedIntersect, rel);
  m.def("unique", &ops::Unique, rel);
  m.def("distributed_unique", &ops::DistributedUnique, rel);

  m.def("group_ids", [](const TablePtr &t, const std::vector<int> &cols, bool presorted) {
    auto g = ops::GroupIds(t, cols, presorted);
    return py::make_tuple(g.gid, g.ngroups, g.first_rows);
  });

  auto groupby_fn = [](TablePtr (*fn)(const TablePtr &, const std::vector<int> &, const std::vector<ops::AggSpec> &)) {
    return [fn](const TablePtr &t, const std::vector<int> &keys, const std::vector<int> &cols,
                const std::vector<int> &op_ids, const std::vector<double> &qs, const std::vector<int> &ddofs) {
      py::gil_scoped_release nogil;
      return fn(t, keys, make_specs(cols, op_ids, qs, ddofs));
    };
  };
  m.def("hash_groupby", groupby_fn(&ops::HashGroupBy));
  m.def("pipeline_groupby", groupby_fn(&ops::PipelineGroupBy));
  m.def("distributed_hash_groupby", groupby_fn(&ops::DistributedHashGroupBy));
  m.def("distributed_pipeline_groupby", groupby_fn(&ops::DistributedPipelineGroupBy));

  m.def("aggregate", &ops::Aggregate, py::arg("table"), py::arg("col"), py::arg("op"), py::arg("quantile") = 0.5,
        py::arg("ddof") = 1, py::arg("distributed") = true, rel);

  m.def(
      "distributed_sort",
      [](const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &asc, uint32_t num_bins,
         uint64_t num_samples) {
        SortOptions o;
        o.num_bins = num_bins;
        o.num_samples = num_samples;
        return ops::DistributedSort(t, cols, asc, o);
      },
      rel);
  m.def("map_to_sort_partitions", &ops::MapToSortPartitions, rel);
  m.def("partition_reorder", &ops::PartitionReorder, rel);
  m.def("all_to_all_table", &ops::AllToAllTable, rel);
}
