// Group-by example (reference: cpp/src/examples/groupby_example.cpp,
// groupby_pipeline_example.cpp, compute_example.cpp).
//   usage: groupby_example <device: cpu | cuda:0 | tcp | rccl> <csv>
// Hash group-by on column 0 with every aggregation of column 1, the pipeline group-by
// of the table sorted by column 0, and the scalar aggregates; prints "name value" lines.
#include "example_common.hpp"

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <device> <csv>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  cylon::TablePtr t, g, sorted, pg, sum, cnt, mn, mx, mm;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], t));
  example::report("rows", t);
  const std::vector<cylon::AggOp> ops = {cylon::AGG_SUM, cylon::AGG_COUNT, cylon::AGG_MIN,  cylon::AGG_MAX,
                                         cylon::AGG_MEAN, cylon::AGG_VAR, cylon::AGG_STDDEV, cylon::AGG_NUNIQUE};
  CHECK_OK(cylon::DistributedHashGroupBy(t, {0}, std::vector<int32_t>(ops.size(), 1), ops, g));
  example::report("hash_groups", g);
  example::report("hash_columns", g->Columns());

  // pipeline group-by: input pre-sorted on the key (reference PipelineGroupBy)
  CHECK_OK(cylon::Sort(t, 0, sorted, true));
  CHECK_OK(cylon::DistributedPipelineGroupBy(sorted, 0, {1, 1, 1, 1}, {cylon::AGG_SUM, cylon::AGG_COUNT, cylon::AGG_MIN,
                                                                       cylon::AGG_MAX}, pg));
  example::report("pipeline_groups", pg);

  // both group-bys agree: same keys, same sums (hash output sorted by key first)
  cylon::TablePtr gs;
  CHECK_OK(cylon::Sort(g, 0, gs, true));
  const bool keys_eq = at::equal(example::host_i64(gs, 0), example::host_i64(pg, 0));
  const bool sums_eq = at::allclose(example::host_f64(gs, 1), example::host_f64(pg, 1), 1e-9, 1e-9);
  example::report("pipeline_matches_hash", keys_eq && sums_eq ? 1 : 0);

  // scalar aggregates (global over ranks); the group sums add up to the column sum
  CHECK_OK(cylon::compute::Sum(t, 1, sum));
  CHECK_OK(cylon::compute::Count(t, 1, cnt));
  CHECK_OK(cylon::compute::Min(t, 1, mn));
  CHECK_OK(cylon::compute::Max(t, 1, mx));
  CHECK_OK(cylon::compute::MinMax(t, 1, mm));
  cylon::TablePtr gsum;  // global over ranks too: each rank holds only its share of the groups
  CHECK_OK(cylon::compute::Sum(g, 1, gsum));
  const double total = example::host_f64(sum, 0)[0].item<double>();
  const double gtotal = example::host_f64(gsum, 0)[0].item<double>();
  example::report("count_col1", example::host_i64(cnt, 0)[0].item<int64_t>());
  example::report("group_sums_match_total", std::abs(total - gtotal) <= 1e-6 * std::max(1.0, std::abs(total)) ? 1 : 0);
  example::report("minmax_consistent", example::host_f64(mm, 0)[0].item<double>() == example::host_f64(mn, 0)[0].item<double>() &&
                                               example::host_f64(mm, 1)[0].item<double>() == example::host_f64(mx, 0)[0].item<double>()
                                           ? 1 : 0);
  ctx->Finalize();
  return 0;
}
