// C++ API example (reference: cpp/src/examples/join_example.cpp, union_example.cpp,
// groupby_example.cpp, sorting_example.cpp, parquet_join_example.cpp).
//
// Links only the native core library (cylon_amd/libcylon_amd.so) + libtorch; no Python.
//   usage: relational_example <device: cpu | cuda:0 | tcp | rccl> <csv1> <csv2> <out_dir>
// "tcp" / "rccl" bring up a distributed context natively from the torchrun
// environment (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT, LOCAL_RANK) -- the
// reference's CylonContext::InitDistributed(MPIConfig) -- and "%r" in the paths
// becomes the rank (per-rank input partitions, per-rank outputs).
// Reads two CSV tables, then runs join (hash + sort), union / intersect / subtract,
// unique, sort, a group-by and a scalar aggregate, writes the join result as CSV
// and Parquet, reads the Parquet file back, and prints one "name rows" line per result.
#include <cstdio>
#include <string>

#include "cylon/api.hpp"

using cylon::Status;
using cylon::TablePtr;
namespace jc = cylon::join::config;

#define CHECK_OK(expr)                                                               \
  do {                                                                               \
    Status _s = (expr);                                                              \
    if (!_s.is_ok()) {                                                               \
      std::fprintf(stderr, "%s failed: %s\n", #expr, _s.get_msg().c_str());         \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static void report(const char *what, const TablePtr &t) {
  std::printf("%s %lld\n", what, static_cast<long long>(t->Rows()));
}

int main(int argc, char **argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s <device> <csv1> <csv2> <out_dir>\n", argv[0]);
    return 2;
  }
  const std::string dev = argv[1], out = argv[4];
  std::shared_ptr<cylon::CylonContext> ctx;
  if (dev == "tcp" || dev == "rccl") {
    cylon::net::CommConfig cfg;
    cfg.type = dev == "tcp" ? cylon::net::CommType::TCP : cylon::net::CommType::RCCL;
    ctx = cylon::CylonContext::InitDistributed(cfg);
  } else {
    ctx = cylon::CylonContext::Init(at::Device(dev));
  }
  const std::string rank = std::to_string(ctx->GetRank());
  auto path = [&](std::string p) {
    for (size_t i = p.find("%r"); i != std::string::npos; i = p.find("%r")) p.replace(i, 2, rank);
    return p;
  };

  TablePtr a, b, j, js, u, i, s, q, srt, g, sum, back;
  CHECK_OK(cylon::FromCSV(ctx, path(argv[2]), a));
  CHECK_OK(cylon::FromCSV(ctx, path(argv[3]), b, cylon::io::CSVReadOptions().WithDelimiter(',').UseThreads(true).BlockSize(1 << 20)));
  report("left", a);
  report("right", b);

  CHECK_OK(cylon::DistributedJoin(a, b, jc::JoinConfig::InnerJoin(0, 0, jc::HASH, "l_", "r_"), j));
  report("join_hash", j);
  CHECK_OK(cylon::Join(a, b, jc::JoinConfig::InnerJoin(0, 0, jc::SORT, "l_", "r_"), js));
  report("join_sort", js);

  CHECK_OK(cylon::DistributedUnion(a, b, u));
  report("union", u);
  CHECK_OK(cylon::DistributedIntersect(a, b, i));
  report("intersect", i);
  CHECK_OK(cylon::DistributedSubtract(a, b, s));
  report("subtract", s);
  CHECK_OK(cylon::Unique(a, {0}, q));
  report("unique_col0", q);

  CHECK_OK(cylon::Sort(a, 0, srt, true));
  report("sort", srt);
  CHECK_OK(cylon::DistributedHashGroupBy(a, {0}, {1}, {cylon::AGG_SUM}, g));
  report("groupby_sum", g);
  CHECK_OK(cylon::compute::Sum(a, 1, sum));
  report("sum_col1", sum);

  const std::string stem = out + (ctx->IsDistributed() ? "/join_" + rank : "/join");
  CHECK_OK(cylon::WriteCSV(j, stem + ".csv"));
  CHECK_OK(cylon::WriteParquet(j, stem + ".parquet"));
  CHECK_OK(cylon::FromParquet(ctx, stem + ".parquet", back));
  report("parquet_roundtrip", back);
  ctx->Barrier();
  ctx->Finalize();
  return 0;
}
