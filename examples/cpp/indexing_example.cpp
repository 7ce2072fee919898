// Indexing example (reference: cpp/src/examples/indexing_example.cpp).
//   usage: indexing_example <device: cpu | cuda:0> <csv>
// Builds a hash index and a sorted (BinaryTree) index on column 0, then selects rows by
// label (loc), by label range, and by position (iloc).
#include "example_common.hpp"
#include "cylon/indexing/index.hpp"

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <device> <csv>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  cylon::TablePtr t;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], t));
  example::report("rows", t);
  namespace ix = cylon::indexing;
  const cylon::Column &c0 = t->column(0);
  // labels: the first three values of column 0
  cylon::Column labels(c0.name, c0.type, 3, c0.data.slice(0, 0, 3).clone());
  for (auto schema : {ix::IndexingSchema::Hash, ix::IndexingSchema::BinaryTree, ix::IndexingSchema::Linear}) {
    t->SetIndex(ix::BuildIndex(t, 0, schema));
    const std::string tag = schema == ix::IndexingSchema::Hash ? "hash" : (schema == ix::IndexingSchema::Linear ? "linear" : "sorted");
    auto loc = ix::LocIndexer(schema).Loc(t, labels);
    example::report(("loc_" + tag).c_str(), loc);
  }
  t->SetIndex(ix::BuildIndex(t, 0, ix::IndexingSchema::BinaryTree));
  cylon::Column lo(c0.name, c0.type, 1, c0.data.slice(0, 1, 2).clone()), hi(c0.name, c0.type, 1, c0.data.slice(0, 2, 3).clone());
  auto rng = ix::LocIndexer(ix::IndexingSchema::BinaryTree).LocRange(t, lo, hi);
  example::report("loc_range", rng);
  auto il = ix::ILocIndexer().ILocRange(t, 2, 7);
  example::report("iloc_range", il);
  ctx->Finalize();
  return 0;
}
