// Partition example (reference: cpp/src/examples/partition_example.cpp).
//   usage: partition_example <device: cpu | cuda:0 | tcp | rccl> <csv> <partitions>
// Hash partition on column 0 into N tables (the reference's modulo / Murmur3 partition
// ids), then a shuffle; row counts are conserved.
#include "example_common.hpp"

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <device> <csv> <partitions>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  const int np = std::atoi(argv[3]);
  cylon::TablePtr t, shuffled;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], t));
  example::report("rows", t);
  std::map<int, cylon::TablePtr> parts;
  CHECK_OK(cylon::HashPartition(t, {0}, np, &parts));
  int64_t total = 0;
  for (const auto &kv : parts) {
    const std::string name = "partition_" + std::to_string(kv.first);
    example::report(name.c_str(), kv.second);
    total += kv.second->Rows();
  }
  example::report("partition_total", total);
  CHECK_OK(cylon::Shuffle(t, {0}, shuffled));
  example::report("shuffled", shuffled);
  ctx->Finalize();
  return 0;
}
