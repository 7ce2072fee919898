// Overlap demonstration for the chunked distributed join (profiles/async_overlap_*):
// two ranks as two threads of ONE process on one GPU (native TCP bootstrap, rank 0
// serves the TCPStore), each wrapped by the asynchronous delay transport
// (net/async_delay_communicator.hpp), so every posted chunk exchange completes on a
// side HIP stream after a spin delay.  Under `rocprofv3 --kernel-trace` the
// k_spin_delay kernels of chunks k+1.. overlap the join kernels of chunk k.
//   usage: async_overlap_example <rows per rank> <chunks> <delay_us> <port>
#include <cstdio>
#include <thread>

#include "cylon/api.hpp"
#include "cylon/net/async_delay_communicator.hpp"

using cylon::TablePtr;
namespace jc = cylon::join::config;

static TablePtr relation(const std::shared_ptr<cylon::CylonContext> &ctx, int64_t n, int64_t hi, const char *v) {
  auto o = at::TensorOptions().device(ctx->GetDevice());
  std::vector<cylon::Column> cols;
  cols.emplace_back("k", cylon::DataType(cylon::Type::INT64), n, at::randint(0, hi, {n}, o.dtype(at::kLong)));
  cols.emplace_back(v, cylon::DataType(cylon::Type::DOUBLE), n, at::rand({n}, o.dtype(at::kDouble)));
  return cylon::Table::Make(ctx, std::move(cols));
}

int main(int argc, char **argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s <rows per rank> <chunks> <delay_us> <port>\n", argv[0]);
    return 2;
  }
  const int64_t n = std::atoll(argv[1]);
  const std::string chunks = argv[2];
  const double delay = std::atof(argv[3]);
  const int port = std::atoi(argv[4]);
  int64_t rows[2] = {0, 0}, posted[2] = {0, 0}, inflight[2] = {0, 0};
  std::string err[2];
  auto rank_main = [&](int r) {
    try {
      cylon::net::CommConfig cfg;
      cfg.type = cylon::net::CommType::TCP;
      cfg.rank = r;
      cfg.world_size = 2;
      cfg.master_addr = "127.0.0.1";
      cfg.master_port = port;
      cfg.device = "cuda:0";
      auto ctx = cylon::CylonContext::InitDistributed(cfg);
      auto adc = std::make_shared<cylon::net::AsyncDelayCommunicator>(ctx->GetCommunicator(), delay);
      ctx->setCommunicator(adc);
      ctx->AddConfig("shuffle_chunks", chunks);
      at::manual_seed(100 + r);
      TablePtr a = relation(ctx, n, 2 * n, "x"), b = relation(ctx, n, 2 * n, "y"), out;
      for (int it = 0; it < 2; ++it) {  // warm-up + traced iteration
        cylon::Status s = cylon::DistributedJoin(a, b, jc::JoinConfig::InnerJoin(0, 0, jc::HASH, "l_", "r_"), out);
        if (!s.is_ok()) throw std::runtime_error(s.get_msg());
      }
      rows[r] = out->Rows();
      posted[r] = adc->posted();
      inflight[r] = adc->observed_in_flight();
      ctx->Barrier();
      ctx->Finalize();
    } catch (const std::exception &e) {
      err[r] = e.what();
    }
  };
  std::thread t0(rank_main, 0), t1(rank_main, 1);
  t0.join();
  t1.join();
  for (int r = 0; r < 2; ++r) {
    if (!err[r].empty()) {
      std::fprintf(stderr, "rank %d: %s\n", r, err[r].c_str());
      return 1;
    }
    std::printf("rank %d rows %lld posted %lld in_flight_at_wait %lld\n", r, (long long)rows[r], (long long)posted[r],
                (long long)inflight[r]);
  }
  return 0;
}
