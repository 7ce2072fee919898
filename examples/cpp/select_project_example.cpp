// Select / project / merge example (reference: cpp/src/examples/select_example.cpp,
// project_example.cpp, table_from_vectors_example.cpp).
//   usage: select_project_example <device: cpu | cuda:0> <csv>
// A row-predicate selection (Row accessors), a projection, a vertical merge, and a table
// built from std::vector columns.
#include "example_common.hpp"

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <device> <csv>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  cylon::TablePtr t, even, proj, merged;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], t));
  example::report("rows", t);
  CHECK_OK(cylon::Select(t, [](const cylon::Row &r) { return r.GetInt64(0) % 2 == 0; }, even));
  example::report("select_even_col0", even);
  CHECK_OK(cylon::Project(t, {1}, proj));
  example::report("project_columns", proj->Columns());
  CHECK_OK(cylon::Merge({t, even}, merged));
  example::report("merge_rows", merged);

  // a table from host vectors (zero-copy wrap, then moved to the context's device)
  std::vector<int64_t> ids = {5, 3, 9, 1, 3};
  std::vector<double> vals = {0.5, 1.5, 2.5, 3.5, 4.5};
  std::vector<cylon::Column> cols;
  cols.emplace_back("id", cylon::DataType(cylon::Type::INT64), (int64_t)ids.size(),
                    at::from_blob(ids.data(), {(int64_t)ids.size()}, at::kLong).clone().to(ctx->GetDevice()));
  cols.emplace_back("val", cylon::DataType(cylon::Type::DOUBLE), (int64_t)vals.size(),
                    at::from_blob(vals.data(), {(int64_t)vals.size()}, at::kDouble).clone().to(ctx->GetDevice()));
  auto vt = cylon::Table::Make(ctx, std::move(cols));
  cylon::TablePtr vs, vsum;
  CHECK_OK(cylon::Sort(vt, 0, vs, true));
  CHECK_OK(cylon::compute::Sum(vt, 1, vsum));
  example::report("vector_table_rows", vt);
  example::report("vector_table_first_id", example::host_i64(vs, 0)[0].item<int64_t>());
  example::report("vector_table_sum_x10", (int64_t)(example::host_f64(vsum, 0)[0].item<double>() * 10));
  ctx->Finalize();
  return 0;
}
