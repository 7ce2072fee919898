// Scalar aggregates (reference: cpp/src/examples/compute_example.cpp).
//   usage: compute_example <device: cpu | cuda:0 | tcp | rccl> <csv>
// Sum / Count / Min / Max / MinMax of every numeric column; distributed contexts reduce over
// all ranks.  Values are printed x1000, rounded, as integers ("name value" lines).
#include <cmath>

#include "example_common.hpp"

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <device> <csv>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  cylon::TablePtr t;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], t));
  example::report("rows", t);
  auto scaled = [](const cylon::TablePtr &r, int c) {
    return (int64_t)std::llround(example::host_f64(r, c)[0].item<double>() * 1000.0);
  };
  for (int c = 0; c < t->Columns(); ++c) {
    if (!t->column(c).type.is_numeric()) continue;
    cylon::TablePtr s, n, mn, mx, mm;
    CHECK_OK(cylon::compute::Sum(t, c, s));
    CHECK_OK(cylon::compute::Count(t, c, n));
    CHECK_OK(cylon::compute::Min(t, c, mn));
    CHECK_OK(cylon::compute::Max(t, c, mx));
    CHECK_OK(cylon::compute::MinMax(t, c, mm));
    const std::string p = "col" + std::to_string(c) + "_";
    example::report((p + "sum_x1000").c_str(), scaled(s, 0));
    example::report((p + "count").c_str(), example::host_i64(n, 0)[0].item<int64_t>());
    example::report((p + "min_x1000").c_str(), scaled(mn, 0));
    example::report((p + "max_x1000").c_str(), scaled(mx, 0));
    example::report((p + "minmax_consistent").c_str(), scaled(mm, 0) == scaled(mn, 0) && scaled(mm, 1) == scaled(mx, 0));
  }
  ctx->Finalize();
  return 0;
}
