// Unique example (reference: cpp/src/examples/unique_example.cpp).
//   usage: unique_example <device: cpu | cuda:0 | tcp | rccl> <csv>
// Distinct rows over column 0 keeping the first / last occurrence, distinct over all
// columns, and the distributed unique (shuffle on the columns, then unique).
#include "example_common.hpp"

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <device> <csv>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  cylon::TablePtr t, first, last, all, dist;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], t));
  example::report("rows", t);
  CHECK_OK(cylon::Unique(t, {0}, first, true));
  CHECK_OK(cylon::Unique(t, {0}, last, false));
  CHECK_OK(cylon::Unique(t, {}, all, true));
  CHECK_OK(cylon::DistributedUnique(t, {0}, dist));
  example::report("unique_first", first);
  example::report("unique_last", last);
  example::report("unique_all_columns", all);
  example::report("distributed_unique", dist);
  ctx->Finalize();
  return 0;
}
