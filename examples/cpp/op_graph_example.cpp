// Streaming op-graph example (reference: cpp/src/examples/ops/join_op_example.cpp, task_test.cpp).
//   usage: op_graph_example <device: cpu | cuda:0 | tcp | rccl> <csv_left> <csv_right> [batches]
// Feeds both tables to a DisJoinOP (partition -> all-to-all -> split -> local join per
// sub-partition, one exchange round per input batch) and a DisUnionOp in `batches` slices each,
// collects the emitted tables through the result callback and checks them against the one-shot
// DistributedJoin / DistributedUnion; prints "name value" lines.
#include <cstdlib>

#include "cylon/ops/graph.hpp"
#include "example_common.hpp"

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <device> <csv_left> <csv_right> [batches]\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  const int batches = argc > 4 ? std::atoi(argv[4]) : 4;
  cylon::TablePtr l, r, joined, uni;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], l));
  CHECK_OK(cylon::FromCSV(ctx, argv[3], r));
  auto slices = [&](const cylon::TablePtr &t) {  // `batches` row ranges (the last may be empty)
    std::vector<cylon::TablePtr> out;
    const int64_t n = t->Rows(), step = (n + batches - 1) / batches;
    for (int b = 0; b < batches; ++b) {
      const int64_t off = std::min<int64_t>(n, b * step);
      out.push_back(cylon::ops::Slice(t, off, std::min<int64_t>(step, n - off)));
    }
    return out;
  };

  const cylon::graph::DisJoinOpConfig cfg{
      8, cylon::join::config::JoinConfig::InnerJoin(0, 0, cylon::join::config::HASH, "l_", "r_")};
  int64_t op_rows = 0, emitted = 0;
  {
    cylon::graph::DisJoinOP op(ctx, 0, [&](int, const cylon::TablePtr &t) { op_rows += t->Rows(); ++emitted; }, cfg);
    const auto ls = slices(l), rs = slices(r);
    for (int b = 0; b < batches; ++b) {  // interleaved: batch b of both relations
      op.InsertTable(cylon::graph::DisJoinOP::kLeftTag, ls[b]);
      op.InsertTable(cylon::graph::DisJoinOP::kRightTag, rs[b]);
    }
    op.WaitForCompletion();
  }
  CHECK_OK(cylon::DistributedJoin(l, r, cfg.join_config, joined));
  example::report("op_join_rows", op_rows);
  example::report("op_join_tables", emitted);
  example::report("direct_join_rows", joined);

  int64_t union_rows = 0;
  {
    cylon::graph::DisUnionOp op(ctx, 1, [&](int, const cylon::TablePtr &t) { union_rows += t->Rows(); });
    for (const auto &t : slices(l)) op.InsertTable(0, t);
    for (const auto &t : slices(r)) op.InsertTable(0, t);
    op.WaitForCompletion();
  }
  CHECK_OK(cylon::DistributedUnion(l, r, uni));
  example::report("op_union_rows", union_rows);
  example::report("direct_union_rows", uni);
  ctx->Finalize();
  return 0;
}
