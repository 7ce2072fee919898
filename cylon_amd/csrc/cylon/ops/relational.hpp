// Set operations, unique, group-by and aggregates (L3 local + L4 distributed).
#pragma once
#include "../table.hpp"

namespace cylon {
namespace ops {

// Dense group ids in first-occurrence order (reference HashGroupBy order).
struct GroupInfo {
  at::Tensor gid;         // int64 [rows]
  int64_t ngroups = 0;
  at::Tensor first_rows;  // int64 [ngroups], ascending
};
GroupInfo GroupIds(const TablePtr &t, const std::vector<int> &cols, bool presorted = false);

struct AggSpec {
  int col;
  int op;  // AggOp
  double quantile = 0.5;
  int ddof = 1;
};

const char *AggPrefix(int op);

TablePtr HashGroupBy(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs);
TablePtr PipelineGroupBy(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs);
TablePtr DistributedHashGroupBy(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs);
TablePtr DistributedPipelineGroupBy(const TablePtr &t, const std::vector<int> &keys,
                                    const std::vector<AggSpec> &aggs);

// Scalar aggregate of one column, global across ranks when distributed=true (1-row table).
TablePtr Aggregate(const TablePtr &t, int col, int op, double quantile, int ddof, bool distributed);

TablePtr Unique(const TablePtr &t, const std::vector<int> &cols, bool keep_first);
TablePtr DistributedUnique(const TablePtr &t, const std::vector<int> &cols, bool keep_first);

TablePtr Union(const TablePtr &l, const TablePtr &r);
TablePtr Subtract(const TablePtr &l, const TablePtr &r);
TablePtr Intersect(const TablePtr &l, const TablePtr &r);
TablePtr DistributedUnion(const TablePtr &l, const TablePtr &r);
TablePtr DistributedSubtract(const TablePtr &l, const TablePtr &r);
TablePtr DistributedIntersect(const TablePtr &l, const TablePtr &r);

// Sample sort across ranks (range partition on the first sort column, then local sort).
TablePtr DistributedSort(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending,
                         const SortOptions &opts);
// Range partition ids (K13): returns pid + counts; ascending/descending like the reference.
std::pair<at::Tensor, std::vector<int64_t>> MapToSortPartitions(const TablePtr &t, int col, uint32_t nparts,
                                                                bool ascending, uint64_t num_samples,
                                                                uint32_t num_bins);

}  // namespace ops
}  // namespace cylon
