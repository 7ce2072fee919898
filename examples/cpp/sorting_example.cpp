// Sorting example (reference: cpp/src/examples/sorting_example.cpp,
// multicolumn_sorting_example.cpp).
//   usage: sorting_example <device: cpu | cuda:0 | tcp | rccl> <csv>
// Single-column sort (both directions), multi-column sort with per-column directions and
// the distributed (sample) sort; each result is checked for order on the host.
#include "example_common.hpp"

// rows of t non-decreasing (dir[c] true) / non-increasing on columns cols, lexicographically
static bool ordered(const cylon::TablePtr &t, const std::vector<int32_t> &cols, const std::vector<bool> &asc) {
  std::vector<at::Tensor> v;
  for (int c : cols) v.push_back(example::host_f64(t, c));
  for (int64_t r = 1; r < t->Rows(); ++r) {
    for (size_t k = 0; k < cols.size(); ++k) {
      const double a = v[k][r - 1].item<double>(), b = v[k][r].item<double>();
      if (a == b) continue;
      if ((a < b) != asc[k]) return false;
      break;
    }
  }
  return true;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <device> <csv>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  cylon::TablePtr t, s1, s2, s3, s4;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], t));
  example::report("rows", t);
  CHECK_OK(cylon::Sort(t, 1, s1, true));
  example::report("sort_asc_rows", s1);
  example::report("sort_asc_ok", ordered(s1, {1}, {true}) ? 1 : 0);
  CHECK_OK(cylon::Sort(t, 1, s2, false));
  example::report("sort_desc_ok", ordered(s2, {1}, {false}) ? 1 : 0);
  CHECK_OK(cylon::Sort(t, {0, 1}, s3, {false, true}));
  example::report("sort_multi_ok", ordered(s3, {0, 1}, {false, true}) ? 1 : 0);
  CHECK_OK(cylon::DistributedSort(t, {0, 1}, s4, {true, true}));
  example::report("dist_sort_rows", s4);
  example::report("dist_sort_ok", ordered(s4, {0, 1}, {true, true}) ? 1 : 0);
  ctx->Finalize();
  return 0;
}
