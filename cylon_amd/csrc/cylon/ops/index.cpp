// Index lookups (C27 / K16).
//
// Reference: cpp/src/cylon/indexing/index.hpp:81-700 (HashIndex: an
// unordered_multimap value -> row positions; LinearIndex: a scan per lookup),
// indexer.hpp:76-260 (loc by value / list / range).  On the device a lookup of
// m labels in an index of n values is one K5 hash join of the label column
// against the index column (build = the smaller side), then a (label order,
// row order) sort of the matching pairs, which is pandas' loc order.
#include "util.hpp"

namespace cylon {
namespace ops {

at::Tensor IndexLookup(const std::shared_ptr<CylonContext> &ctx, const Column &index, const Column &labels) {
  const at::Device dev = index.data.device();
  Exec ex(dev);
  if (index.length == 0 || labels.length == 0) return ex.empty_i64(0);
  TablePtr it = Table::Make(ctx, {index.with_name("i")});
  TablePtr lt = Table::Make(ctx, {labels.to(dev).with_name("l")});
  auto pr = JoinIndices(lt, it, join::config::JoinConfig::InnerJoin(0, 0, join::config::JoinAlgorithm::HASH));
  if (pr.first.numel() == 0) return ex.empty_i64(0);
  std::vector<Column> pc{Column("l", DataType(Type::INT64), pr.first.numel(), pr.first),
                         Column("i", DataType(Type::INT64), pr.second.numel(), pr.second)};
  TablePtr pairs = Table::Make(ctx, std::move(pc));
  at::Tensor perm = SortIndices(pairs, {0, 1}, {true});
  return pr.second.index_select(0, perm);
}

}  // namespace ops
}  // namespace cylon
