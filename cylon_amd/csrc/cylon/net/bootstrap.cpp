// Native distributed bootstrap: CommConfig from the torchrun environment, a c10d
// TCPStore rendezvous, then ProcessGroupNCCL (RCCL over xGMI) or the TCP mesh.
//
// Reference: cylon/ctx/cylon_context.cpp:32-43 (InitDistributed, MPI only) and
// cylon/net/mpi/mpi_communicator.cpp:51-60 (MPI_Init / Comm_rank / Comm_size).
#ifndef USE_C10D_NCCL
#define USE_C10D_NCCL 1
#endif
#include <c10/hip/HIPFunctions.h>
#include <hip/hip_runtime.h>

#include <torch/csrc/distributed/c10d/PrefixStore.hpp>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/ProcessGroupNCCL.hpp>
#include <torch/csrc/distributed/c10d/TCPStore.hpp>

#include "../ctx/cylon_context.hpp"
#include "tcp_communicator.hpp"

namespace cylon {
namespace net {

static int env_int(const char *name, int def) {
  const char *v = std::getenv(name);
  return v && *v ? std::atoi(v) : def;
}

CommConfig CommConfig::FromEnv(CommType type) {
  CommConfig c;
  c.type = type;
  return c.Resolved();
}

static int hip_devices() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

CommConfig CommConfig::Resolved() const {
  CommConfig c = *this;
  if (c.rank < 0) c.rank = env_int("RANK", 0);
  if (c.world_size < 0) c.world_size = env_int("WORLD_SIZE", 1);
  if (c.local_rank < 0) c.local_rank = env_int("LOCAL_RANK", c.rank);
  if (c.master_addr.empty()) {
    const char *a = std::getenv("MASTER_ADDR");
    c.master_addr = a && *a ? a : "127.0.0.1";
  }
  if (c.master_port < 0) c.master_port = env_int("MASTER_PORT", 29500);
  if (c.type == CommType::GLOO) c.type = CommType::TCP;
  // MPI has no transport in this image: the reference's MPIConfig maps to RCCL when
  // the process sees GPUs, else to the TCP mesh (same semantics, different wire)
  if (c.type == CommType::MPI) c.type = hip_devices() > 0 ? CommType::RCCL : CommType::TCP;
  CYLON_CHECK(c.type == CommType::RCCL || c.type == CommType::TCP, Code::NotImplemented,
              "native bootstrap supports RCCL and TCP, not " << CommTypeName(c.type));
  if (c.device.empty()) c.device = c.type == CommType::RCCL ? "cuda:" + std::to_string(c.local_rank) : "cpu";
  CYLON_CHECK(c.world_size >= 1 && c.rank >= 0 && c.rank < c.world_size, Code::Invalid,
              "bad RANK / WORLD_SIZE: " << c.rank << " / " << c.world_size);
  return c;
}

std::shared_ptr<Communicator> MakeCommunicator(const CommConfig &in, at::Device *device_out) {
  const CommConfig cfg = in.Resolved();
  const at::Device dev(cfg.device);
  if (device_out) *device_out = dev;
  c10d::TCPStoreOptions so;
  so.port = (uint16_t)cfg.master_port;
  // under torchrun the elastic agent already serves the store on MASTER_PORT
  const char *agent = std::getenv("TORCHELASTIC_USE_AGENT_STORE");
  so.isServer = cfg.rank == 0 && !(agent && std::string(agent) == "True");
  so.numWorkers = std::nullopt;
  so.waitWorkers = false;
  so.timeout = std::chrono::milliseconds((int64_t)(cfg.timeout_s * 1000.0));
  so.useLibUV = false;
  c10::intrusive_ptr<c10d::Store> base = c10::make_intrusive<c10d::TCPStore>(cfg.master_addr, so);
  // a key prefix per bootstrap generation keeps repeated contexts in one job apart
  const int64_t gen = base->add("cylon_bootstrap/generation/" + std::to_string(cfg.rank), 1);
  auto store = c10::make_intrusive<c10d::PrefixStore>("cylon/" + std::to_string(gen) + "/", base);
  if (cfg.type == CommType::TCP) return std::make_shared<TcpCommunicator>(store, cfg.rank, cfg.world_size, cfg.timeout_s);

  CYLON_CHECK(dev.is_cuda(), Code::Invalid, "RCCL needs a GPU device, got " << cfg.device);
  CYLON_CHECK(dev.index() < hip_devices(), Code::Invalid,
              "LOCAL_RANK " << dev.index() << " has no GPU (" << hip_devices() << " visible)");
  CYLON_CHECK(hipSetDevice(dev.index()) == hipSuccess, Code::ExecutionError, "hipSetDevice(" << dev.index() << ")");
  c10::hip::set_device(dev.index());
  auto opts = c10d::ProcessGroupNCCL::Options::create();
  opts->timeout = std::chrono::milliseconds((int64_t)(cfg.timeout_s * 1000.0));
  // RCCL's stream at high priority: HIP maps streams onto a few hardware queues, and a
  // normal-priority comm stream can share the compute stream's queue, which serialises every
  // all-to-all with the operator kernels (measured: 0 ms of overlap, profiles/rccl_queue_r03.txt)
  opts->is_high_priority_stream = true;
  auto backend = c10::make_intrusive<c10d::ProcessGroupNCCL>(store, cfg.rank, cfg.world_size, opts);
  auto pg = c10::make_intrusive<c10d::ProcessGroup>(store, cfg.rank, cfg.world_size);
  backend->setSequenceNumberForGroup();
  pg->setBackend(c10::DeviceType::CUDA, c10d::ProcessGroup::BackendType::NCCL, backend);
  pg->setDefaultBackend(c10d::ProcessGroup::BackendType::NCCL);
  return std::make_shared<ProcessGroupCommunicator>(pg, CommType::RCCL, dev);
}

}  // namespace net

std::shared_ptr<CylonContext> CylonContext::InitDistributed(const net::CommConfig &cfg) {
  at::Device dev(at::kCPU);
  auto comm = net::MakeCommunicator(cfg, &dev);
  auto ctx = InitDistributed(std::move(comm), dev);
  return ctx;
}

}  // namespace cylon
