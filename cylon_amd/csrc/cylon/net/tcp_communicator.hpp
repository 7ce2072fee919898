// Native TCP transport (CommType::TCP) and the native distributed bootstrap.
//
// Reference: cpp/src/cylon/net/comm_type.hpp:20-22 declares TCP but the
// reference never implements it (cylon_context.cpp:32-41 throws for anything
// but MPI); its MPI backend bootstraps with MPI_Init (mpi_communicator.cpp:51-60).
//
// Here a context can be brought up from pure C++ (examples, C ABI, JNI) with the
// torchrun environment (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT, LOCAL_RANK):
//   * RCCL: a c10d TCPStore rendezvous + ProcessGroupNCCL (RCCL over xGMI), one
//     GPU per rank, wrapped by the ProcessGroupCommunicator used everywhere else;
//   * TCP: this file's full-mesh socket communicator for host tables (the CPU
//     rehearsal transport of multi-process tests and of the C++ examples).  Peer
//     addresses are exchanged through the same TCPStore.
//
// TCP wire format: every message is a frame {int64 tag, int64 bytes, payload}.
// One receiver thread per peer drains its socket into per-tag queues, so a
// blocking send can never deadlock against a peer that is itself sending.
// Collectives use tags from a private sequence (all ranks issue them in the same
// order); ISend/IRecv use the caller's tag (< 2^40).
#pragma once
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <thread>

#include "communicator.hpp"

namespace c10d {
class Store;
}

namespace cylon {
namespace net {

// Distributed bootstrap configuration (reference: net/comm_config.hpp, mpi_communicator.hpp MPIConfig).
// Unset fields (-1 / empty) are read from the torchrun environment.
struct CommConfig {
  CommType type = CommType::RCCL;  // RCCL | TCP (GLOO maps to TCP natively; MPI: RCCL with GPUs, else TCP)
  int rank = -1;
  int world_size = -1;
  int local_rank = -1;
  std::string master_addr;
  int master_port = -1;
  double timeout_s = 1800.0;
  std::string device;  // default: cuda:<local_rank> for RCCL, cpu for TCP

  static CommConfig FromEnv(CommType type);
  CommConfig Resolved() const;  // env defaults filled in, type MPI/GLOO mapped
};

class TcpCommunicator : public Communicator {
 public:
  // Connects the full mesh: every rank listens, publishes host:port in `store`,
  // accepts from higher ranks and connects to lower ranks.
  TcpCommunicator(c10::intrusive_ptr<c10d::Store> store, int rank, int world, double timeout_s);
  ~TcpCommunicator() override;

  int GetRank() const override { return rank_; }
  int GetWorldSize() const override { return world_; }
  CommType GetCommType() const override { return CommType::TCP; }
  void Barrier() override;
  void Finalize() override;
  at::Tensor AllToAllV(const at::Tensor &send, const std::vector<int64_t> &send_counts,
                       const std::vector<int64_t> &recv_counts) override;
  std::vector<int64_t> ExchangeCounts(const std::vector<int64_t> &send_counts) override;
  void AllReduce(at::Tensor &t, ReduceOp op) override;
  at::Tensor AllGather(const at::Tensor &in) override;
  void Broadcast(at::Tensor &t, int root) override;
  std::shared_ptr<P2PRequest> ISend(const at::Tensor &t, int dst, int tag) override;
  std::shared_ptr<P2PRequest> IRecv(at::Tensor &t, int src, int tag) override;

  // frame-level primitives (also used by the requests)
  void SendFrame(int peer, int64_t tag, const void *data, int64_t bytes);
  bool TryRecvFrame(int peer, int64_t tag, std::vector<uint8_t> &out);
  std::vector<uint8_t> RecvFrame(int peer, int64_t tag);

 private:
  struct Peer {
    int fd = -1;
    std::mutex send_mu;
    std::thread reader;
  };
  void reader_loop(int peer);
  int64_t next_coll_tag() { return (int64_t(1) << 40) + coll_seq_++; }
  // all-to-all of host byte blocks: block[p] goes to rank p, returns the block from each rank
  std::vector<std::vector<uint8_t>> exchange(const std::vector<std::pair<const uint8_t *, int64_t>> &blocks);

  // the rendezvous store stays alive with the communicator: rank 0 serves it, and
  // other ranks may still be resolving peer addresses after rank 0's mesh is complete
  c10::intrusive_ptr<c10d::Store> store_;
  int rank_, world_;
  double timeout_s_;
  int64_t coll_seq_ = 0;
  std::vector<std::unique_ptr<Peer>> peers_;
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::map<std::pair<int, int64_t>, std::deque<std::vector<uint8_t>>> queues_;
  std::vector<std::string> peer_error_;
  bool closed_ = false;
};

// Builds the communicator for `cfg` (TCPStore rendezvous + RCCL process group, or the TCP mesh).
std::shared_ptr<Communicator> MakeCommunicator(const CommConfig &cfg, at::Device *device_out);

}  // namespace net
}  // namespace cylon
