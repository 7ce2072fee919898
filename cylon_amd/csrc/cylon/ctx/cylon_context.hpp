// L0 runtime context.
//
// Reference: cpp/src/cylon/ctx/cylon_context.hpp:29-146 (rank/world, config map,
// communicator, memory pool, sequence numbers used as all-to-all edge tags).
// Additions for MI355X: the context owns the device its tables live on
// (cuda:<local_rank> under one-process-per-GPU) and exposes HBM pool stats from
// the HIP caching allocator.
#pragma once
#include <ATen/ATen.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../net/communicator.hpp"
#include "../net/tcp_communicator.hpp"
#include "memory_pool.hpp"

namespace cylon {

class CylonContext {
 public:
  explicit CylonContext(bool distributed);

  // Local (rank 0 of 1) context on `device` (default: cpu).
  static std::shared_ptr<CylonContext> Init(at::Device device = at::Device(at::kCPU));
  static std::shared_ptr<CylonContext> InitDistributed(std::shared_ptr<net::Communicator> comm, at::Device device);
  // Native bootstrap (no Python): TCPStore rendezvous from the torchrun environment, then
  // RCCL (ProcessGroupNCCL, device cuda:<LOCAL_RANK>) or the TCP mesh (host tables).
  // Reference: ctx/cylon_context.cpp:32-43 InitDistributed(MPIConfig).
  static std::shared_ptr<CylonContext> InitDistributed(const net::CommConfig &cfg);

  void Finalize();
  void AddConfig(const std::string &key, const std::string &value);
  std::string GetConfig(const std::string &key, const std::string &def = "") const;
  const std::map<std::string, std::string> &GetConfigs() const { return config_; }

  std::shared_ptr<net::Communicator> GetCommunicator() const;
  void setCommunicator(std::shared_ptr<net::Communicator> comm) { communicator_ = std::move(comm); }
  void setDistributed(bool d) { distributed_ = d; }

  int GetRank() const;
  int GetWorldSize() const;
  std::vector<int> GetNeighbours(bool include_self) const;
  int GetNextSequence();
  bool IsDistributed() const { return distributed_; }
  // True when distributed operators must run their shuffle + exchange path: world > 1,
  // or a distributed world-1 context with config "force_shuffle" = "1" (env
  // CYLON_FORCE_SHUFFLE=1).  The forced form runs every exchange through the real
  // transport (RCCL self all-to-all on one GPU) instead of the world-1 local shortcut,
  // so the asynchronous exchange path can be tested and profiled on a single GPU.
  bool ShuffleRequired() const;
  net::CommType GetCommType() const;
  void Barrier();

  at::Device GetDevice() const { return device_; }
  void SetDevice(at::Device d) { device_ = d; }
  bool on_gpu() const { return device_.is_cuda(); }

  // HBM pool statistics (bytes) from the HIP caching allocator; 0 on CPU.
  int64_t BytesAllocated() const;
  // bytes the device can still hand out: free HBM + the caching allocator's cached, unused blocks
  // (config "memory_budget_mb" caps it; 0 on the CPU = unbounded)
  int64_t DeviceHeadroom() const;
  int64_t MaxMemory() const;

  // C2: the context's memory pool (default: DeviceMemoryPool / HostMemoryPool
  // for the context device; reference ctx/cylon_context.hpp GetMemoryPool).
  std::shared_ptr<MemoryPool> GetMemoryPool();
  void SetMemoryPool(std::shared_ptr<MemoryPool> pool) { pool_ = std::move(pool); }

 private:
  bool distributed_;
  int sequence_no_ = 0;
  std::shared_ptr<net::Communicator> communicator_;
  std::map<std::string, std::string> config_;
  at::Device device_{at::kCPU};
  std::shared_ptr<MemoryPool> pool_;
  mutable std::mutex mu_;
};

}  // namespace cylon
