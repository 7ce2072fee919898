// In-memory data generation + relational algebra (reference:
// cpp/src/examples/ra_test_inmem_datagen_example.cpp).
//   usage: datagen_join_example <device: cpu | cuda:0 | tcp | rccl> <rows per rank> [key range]
// Each rank generates its relations directly where the context computes (HBM on a GPU):
// int64 keys in [0, range) from a per-rank seed and a float64 payload, then runs the
// (distributed) hash join, union and intersect of the key columns and a key sort.
#include "example_common.hpp"

namespace jc = cylon::join::config;

static cylon::TablePtr make(const std::shared_ptr<cylon::CylonContext> &ctx, int64_t n, int64_t range, uint64_t seed) {
  at::Generator g = at::make_generator<at::CPUGeneratorImpl>(seed);
  at::Tensor k = at::randint(range, {n}, g, at::TensorOptions().dtype(at::kLong)).to(ctx->GetDevice());
  at::Tensor v = at::rand({n}, g, at::TensorOptions().dtype(at::kDouble)).to(ctx->GetDevice());
  std::vector<cylon::Column> cols;
  cols.emplace_back("k", cylon::DataType(cylon::Type::INT64), n, k);
  cols.emplace_back("v", cylon::DataType(cylon::Type::DOUBLE), n, v);
  return cylon::Table::Make(ctx, std::move(cols));
}

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <device> <rows per rank> [key range]\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  const int64_t n = std::atoll(argv[2]);
  const int64_t range = argc > 3 ? std::atoll(argv[3]) : 4 * n;
  const bool dist = ctx->GetWorldSize() > 1;
  const uint64_t rank = (uint64_t)ctx->GetRank();
  cylon::TablePtr l = make(ctx, n, range, 1000 + 2 * rank), r = make(ctx, n, range, 1001 + 2 * rank);
  cylon::TablePtr j, lk, rk, u, i, s;
  jc::JoinConfig cfg(jc::JoinType::INNER, 0, 0, jc::JoinAlgorithm::HASH, "l_", "r_");
  CHECK_OK(dist ? cylon::DistributedJoin(l, r, cfg, j) : cylon::Join(l, r, cfg, j));
  CHECK_OK(cylon::Project(l, {0}, lk));
  CHECK_OK(cylon::Project(r, {0}, rk));
  CHECK_OK(dist ? cylon::DistributedUnion(lk, rk, u) : cylon::Union(lk, rk, u));
  CHECK_OK(dist ? cylon::DistributedIntersect(lk, rk, i) : cylon::Intersect(lk, rk, i));
  CHECK_OK(dist ? cylon::DistributedSort(l, {0}, s, {true}) : cylon::Sort(l, 0, s, true));
  example::report("join_rows", j);
  example::report("union_rows", u);
  example::report("intersect_rows", i);
  example::report("sorted_rows", s);
  at::Tensor ks = example::host_i64(s, 0);
  example::report("sorted_ok", ks.numel() < 2 || (ks.slice(0, 1) >= ks.slice(0, 0, -1)).all().item<bool>() ? 1 : 0);
  ctx->Finalize();
  return 0;
}
