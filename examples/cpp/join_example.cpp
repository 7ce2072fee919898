// Join example (reference: cpp/src/examples/join_example.cpp, multi_idx_join_example.cpp).
//   usage: join_example <device: cpu | cuda:0 | tcp | rccl> <csv_left> <csv_right>
// Every join type with both algorithms on column 0, and a two-column (multi-index) join;
// prints one "<type>_<algorithm> rows" line per result, plus whether hash and sort agree.
#include "example_common.hpp"

namespace jc = cylon::join::config;

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <device> <csv_left> <csv_right>\n", argv[0]);
    return 2;
  }
  auto ctx = example::make_context(argv[1]);
  const bool dist = ctx->GetWorldSize() > 1;
  cylon::TablePtr l, r;
  CHECK_OK(cylon::FromCSV(ctx, argv[2], l));
  CHECK_OK(cylon::FromCSV(ctx, argv[3], r));
  struct Kind {
    const char *name;
    jc::JoinType type;
  };
  const Kind kinds[] = {{"inner", jc::JoinType::INNER},
                        {"left", jc::JoinType::LEFT},
                        {"right", jc::JoinType::RIGHT},
                        {"outer", jc::JoinType::FULL_OUTER}};
  for (const Kind &k : kinds) {
    int64_t rows[2] = {0, 0};
    for (int a = 0; a < 2; ++a) {
      const jc::JoinAlgorithm alg = a == 0 ? jc::JoinAlgorithm::HASH : jc::JoinAlgorithm::SORT;
      jc::JoinConfig cfg(k.type, 0, 0, alg, "l_", "r_");
      cylon::TablePtr out;
      CHECK_OK(dist ? cylon::DistributedJoin(l, r, cfg, out) : cylon::Join(l, r, cfg, out));
      rows[a] = out->Rows();
      std::printf("%s_%s %lld\n", k.name, a == 0 ? "hash" : "sort", static_cast<long long>(rows[a]));
    }
    std::printf("%s_algorithms_agree %d\n", k.name, rows[0] == rows[1] ? 1 : 0);
  }
  // multi-index join: columns (0, 1) of both sides
  jc::JoinConfig multi(jc::JoinType::INNER, std::vector<int>{0, 1}, std::vector<int>{0, 1}, jc::JoinAlgorithm::HASH,
                       "l_", "r_");
  cylon::TablePtr m;
  CHECK_OK(dist ? cylon::DistributedJoin(l, r, multi, m) : cylon::Join(l, r, multi, m));
  example::report("inner_multi_idx", m);
  ctx->Finalize();
  return 0;
}
