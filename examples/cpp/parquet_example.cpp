// Parquet example (reference: cpp/src/examples/parquet_from_csv_test.cpp, parquet_test.cpp,
// parquet_join_example.cpp, parquet_union_example.cpp).
//   usage: parquet_example <device: cpu | cuda:0 | tcp | rccl> <csv_left> <csv_right> <out_dir>
// CSV -> Parquet (snappy, and zstd with small row groups) -> back into the context's device,
// a bit-exact round trip check, a two-file read, a column-subset read, and the join / union of
// the tables read from Parquet; prints "name value" lines.
#include "example_common.hpp"

static bool same_table(const cylon::TablePtr &a, const cylon::TablePtr &b) {
  if (a->Rows() != b->Rows() || a->Columns() != b->Columns()) return false;
  for (int c = 0; c < a->Columns(); ++c) {
    const at::Tensor x = a->column(c).data.slice(0, 0, a->Rows()).to(at::kCPU);
    const at::Tensor y = b->column(c).data.slice(0, 0, b->Rows()).to(at::kCPU);
    if (!at::equal(x, y)) return false;
  }
  return true;
}

int main(int argc, char **argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s <device> <csv_left> <csv_right> <out_dir>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  const std::string dir = argv[4], tag = std::to_string(ctx->GetRank());
  const std::string pl = dir + "/left_" + tag + ".parquet", pr = dir + "/right_" + tag + ".parquet";
  cylon::TablePtr l, r, l2, r2, sub, joined, uni;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], l));
  CHECK_OK(cylon::FromCSV(ctx, argv[3], r));

  cylon::io::ParquetOptions snappy;  // defaults: snappy, 1M-row groups
  cylon::io::ParquetOptions zstd;
  zstd.compression = "zstd";
  zstd.chunk_size = 4;  // several row groups even for a small file
  CHECK_OK(cylon::WriteParquet(l, pl, snappy));
  CHECK_OK(cylon::WriteParquet(r, pr, zstd));

  CHECK_OK(cylon::FromParquet(ctx, pl, l2));
  CHECK_OK(cylon::FromParquet(ctx, pr, r2));
  example::report("left_rows", l2);
  example::report("right_rows", r2);
  example::report("roundtrip_equal", same_table(l, l2) && same_table(r, r2) ? 1 : 0);

  std::vector<cylon::TablePtr> both;  // one read of two files (one thread per file)
  CHECK_OK(cylon::FromParquet(ctx, std::vector<std::string>{pl, pr}, both));
  example::report("multi_file_rows", both.size() == 2 ? both[0]->Rows() + both[1]->Rows() : -1);

  cylon::io::ParquetOptions cols;  // column subset (the second column only)
  cols.columns = {l->ColumnNames()[1]};
  CHECK_OK(cylon::FromParquet(ctx, pl, sub, cols));
  example::report("subset_columns", sub->Columns());

  // relational algebra on the tables read back from Parquet (distributed when ranks > 1)
  const auto cfg = cylon::join::config::JoinConfig::InnerJoin(0, 0, cylon::join::config::HASH, "l_", "r_");
  CHECK_OK(cylon::DistributedJoin(l2, r2, cfg, joined));
  CHECK_OK(cylon::DistributedUnion(l2, r2, uni));
  example::report("join_rows", joined);
  example::report("union_rows", uni);
  ctx->Finalize();
  return 0;
}
