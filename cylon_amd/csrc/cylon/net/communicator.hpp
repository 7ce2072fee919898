// L1 communication layer.
//
// Reference: cpp/src/cylon/net/communicator.hpp:24-37 (Communicator),
// comm_type.hpp:20-22 (CommType), comm_operations.hpp:26-30 (ReduceOp),
// mpi/mpi_communicator.cpp (MPI backend), net/ops/all_to_all.* and
// arrow/arrow_all_to_all.* (header+payload point-to-point shuffle protocol).
//
// MI355X design: one process per GPU; the transport is a torch.distributed
// c10d ProcessGroup.  With backend "nccl" that is RCCL over xGMI (grouped
// ncclSend/ncclRecv all-to-all, ring/tree all-reduce); with "gloo" the same
// code runs on CPU for the multi-process tests.  Instead of the reference's
// per-buffer header/payload messages and polling progress engine, a shuffle is
// ONE size exchange (all_to_all of P int64 counts) followed by one
// all_to_all_v per column buffer on data already laid out partition-major
// by the K3 scatter kernel (no packing, no host progress loop).
#pragma once
#include <ATen/ATen.h>

#include <memory>
#include <string>
#include <vector>

#include "../common.hpp"

namespace c10d {
class ProcessGroup;
}

namespace cylon {
namespace net {

// Numbering follows the reference: LOCAL=0, MPI=1, TCP=2, UCX=3; RCCL and GLOO
// are the torch.distributed-backed transports of this engine.
enum class CommType : int { LOCAL = 0, MPI = 1, TCP = 2, UCX = 3, RCCL = 4, GLOO = 5 };

enum class ReduceOp : int { SUM = 0, MIN = 1, MAX = 2, PROD = 3 };

const char *CommTypeName(CommType t);

// Scope around every blocking wait on a transport.  The core library has no Python
// dependency; the Python extension installs a hook whose region releases the GIL when
// the waiting thread holds it: c10d gloo works complete on worker threads that can
// need the GIL (future callbacks), and a rank blocked in wait() while holding it
// deadlocked the collective under CPU load.
struct BlockingRegion {
  virtual ~BlockingRegion() = default;
};
using BlockingHook = std::unique_ptr<BlockingRegion> (*)();
void SetBlockingHook(BlockingHook hook);
std::unique_ptr<BlockingRegion> EnterBlocking();

// An outstanding point-to-point transfer (ISend / IRecv).
class P2PRequest {
 public:
  virtual ~P2PRequest() = default;
  virtual bool Test() = 0;  // non-blocking completion check
  virtual void Wait() = 0;
};

class Communicator {
 public:
  virtual ~Communicator() = default;
  virtual int GetRank() const = 0;
  virtual int GetWorldSize() const = 0;
  virtual CommType GetCommType() const = 0;
  virtual void Barrier() = 0;
  virtual void Finalize() {}

  // Variable all-to-all along dim 0: send[ sum(send_counts) ] -> recv[ sum(recv_counts) ].
  virtual at::Tensor AllToAllV(const at::Tensor &send, const std::vector<int64_t> &send_counts,
                               const std::vector<int64_t> &recv_counts) = 0;
  // Posted all-to-all: returns the receive tensor and a request to Wait() on before
  // using it.  RCCL works run on the communicator's stream; kernels enqueued on the
  // compute stream between posting and waiting overlap with the transfer.
  // Default: the blocking AllToAllV with an already completed request.
  virtual std::pair<at::Tensor, std::shared_ptr<P2PRequest>> AllToAllVAsync(
      const at::Tensor &send, const std::vector<int64_t> &send_counts, const std::vector<int64_t> &recv_counts);
  // Posted all-to-all between caller-owned buffers at arbitrary per-peer offsets (elements along
  // dim 0): send[soff[r] .. +scnt[r]) goes to rank r and rank r's piece lands in
  // recv[roff[r] .. +rcnt[r]).  A zero count (e.g. this rank's own piece, kept in place by the
  // planned shuffle) moves nothing.  RCCL: one grouped send/recv per peer straight between the
  // buffers; default: a packed all-to-all plus copies, completed before returning.
  virtual std::shared_ptr<P2PRequest> AllToAllVSegmentsAsync(const at::Tensor &send, const std::vector<int64_t> &soff,
                                                             const std::vector<int64_t> &scnt, const at::Tensor &recv,
                                                             const std::vector<int64_t> &roff,
                                                             const std::vector<int64_t> &rcnt);
  // Exchange per-peer element counts (the size matrix row of this rank).
  virtual std::vector<int64_t> ExchangeCounts(const std::vector<int64_t> &send_counts) = 0;
  virtual void AllReduce(at::Tensor &t, ReduceOp op) = 0;
  // out = concat over ranks of `in` (same shape on every rank)
  virtual at::Tensor AllGather(const at::Tensor &in) = 0;
  // Gather tensors of different lengths from every rank (dim 0).
  virtual std::vector<at::Tensor> AllGatherV(const at::Tensor &in);
  virtual void Broadcast(at::Tensor &t, int root) = 0;
  // Point-to-point (C4 Channel transport; reference mpi_channel.cpp Isend/Irecv).
  // Messages between a pair with the same tag are matched in posting order.
  virtual std::shared_ptr<P2PRequest> ISend(const at::Tensor &t, int dst, int tag);
  virtual std::shared_ptr<P2PRequest> IRecv(at::Tensor &t, int src, int tag);
};

class LocalCommunicator : public Communicator {
 public:
  int GetRank() const override { return 0; }
  int GetWorldSize() const override { return 1; }
  CommType GetCommType() const override { return CommType::LOCAL; }
  void Barrier() override {}
  at::Tensor AllToAllV(const at::Tensor &send, const std::vector<int64_t> &, const std::vector<int64_t> &) override {
    return send;
  }
  std::vector<int64_t> ExchangeCounts(const std::vector<int64_t> &c) override { return c; }
  void AllReduce(at::Tensor &, ReduceOp) override {}
  at::Tensor AllGather(const at::Tensor &in) override { return in; }
  void Broadcast(at::Tensor &, int) override {}
};

// Fault injection for tests (SURVEY.md §5 failure detection): forwards to an inner
// communicator and raises CylonError(ExecutionError) on the N-th collective, so the
// failure path of every distributed operator can be exercised without a real
// failing rank.  (The reference has no failure handling: errors abort or hang.)
class FaultInjectionCommunicator : public Communicator {
 public:
  FaultInjectionCommunicator(std::shared_ptr<Communicator> inner, int64_t fail_at_call)
      : inner_(std::move(inner)), fail_at_(fail_at_call) {}
  int GetRank() const override { return inner_->GetRank(); }
  int GetWorldSize() const override { return inner_->GetWorldSize(); }
  CommType GetCommType() const override { return inner_->GetCommType(); }
  void Barrier() override {
    tick("Barrier");
    inner_->Barrier();
  }
  at::Tensor AllToAllV(const at::Tensor &s, const std::vector<int64_t> &sc, const std::vector<int64_t> &rc) override {
    tick("AllToAllV");
    return inner_->AllToAllV(s, sc, rc);
  }
  std::pair<at::Tensor, std::shared_ptr<P2PRequest>> AllToAllVAsync(const at::Tensor &s,
                                                                    const std::vector<int64_t> &sc,
                                                                    const std::vector<int64_t> &rc) override {
    tick("AllToAllV");
    return inner_->AllToAllVAsync(s, sc, rc);
  }
  std::shared_ptr<P2PRequest> AllToAllVSegmentsAsync(const at::Tensor &s, const std::vector<int64_t> &so,
                                                     const std::vector<int64_t> &sc, const at::Tensor &r,
                                                     const std::vector<int64_t> &ro,
                                                     const std::vector<int64_t> &rc) override {
    tick("AllToAllV");
    return inner_->AllToAllVSegmentsAsync(s, so, sc, r, ro, rc);
  }
  std::vector<int64_t> ExchangeCounts(const std::vector<int64_t> &c) override {
    tick("ExchangeCounts");
    return inner_->ExchangeCounts(c);
  }
  void AllReduce(at::Tensor &t, ReduceOp op) override {
    tick("AllReduce");
    inner_->AllReduce(t, op);
  }
  at::Tensor AllGather(const at::Tensor &in) override {
    tick("AllGather");
    return inner_->AllGather(in);
  }
  void Broadcast(at::Tensor &t, int root) override {
    tick("Broadcast");
    inner_->Broadcast(t, root);
  }
  std::shared_ptr<P2PRequest> ISend(const at::Tensor &t, int dst, int tag) override {
    tick("ISend");
    return inner_->ISend(t, dst, tag);
  }
  std::shared_ptr<P2PRequest> IRecv(at::Tensor &t, int src, int tag) override {
    tick("IRecv");
    return inner_->IRecv(t, src, tag);
  }
  int64_t calls() const { return calls_; }

 private:
  void tick(const char *what) {
    if (++calls_ == fail_at_) CYLON_THROW(Code::ExecutionError, "injected communication fault at call " << calls_
                                                                    << " (" << what << ")");
  }
  std::shared_ptr<Communicator> inner_;
  int64_t fail_at_;
  int64_t calls_ = 0;
};

// Communicator over a c10d ProcessGroup (RCCL on MI355X, gloo on CPU).
class ProcessGroupCommunicator : public Communicator {
 public:
  ProcessGroupCommunicator(c10::intrusive_ptr<c10d::ProcessGroup> pg, CommType type, at::Device comm_device);
  ~ProcessGroupCommunicator() override;
  int GetRank() const override { return rank_; }
  int GetWorldSize() const override { return world_; }
  CommType GetCommType() const override { return type_; }
  void Barrier() override;
  at::Tensor AllToAllV(const at::Tensor &send, const std::vector<int64_t> &send_counts,
                       const std::vector<int64_t> &recv_counts) override;
  std::pair<at::Tensor, std::shared_ptr<P2PRequest>> AllToAllVAsync(
      const at::Tensor &send, const std::vector<int64_t> &send_counts,
      const std::vector<int64_t> &recv_counts) override;
  std::shared_ptr<P2PRequest> AllToAllVSegmentsAsync(const at::Tensor &send, const std::vector<int64_t> &soff,
                                                     const std::vector<int64_t> &scnt, const at::Tensor &recv,
                                                     const std::vector<int64_t> &roff,
                                                     const std::vector<int64_t> &rcnt) override;
  std::vector<int64_t> ExchangeCounts(const std::vector<int64_t> &send_counts) override;
  void AllReduce(at::Tensor &t, ReduceOp op) override;
  at::Tensor AllGather(const at::Tensor &in) override;
  void Broadcast(at::Tensor &t, int root) override;
  std::shared_ptr<P2PRequest> ISend(const at::Tensor &t, int dst, int tag) override;
  std::shared_ptr<P2PRequest> IRecv(at::Tensor &t, int src, int tag) override;
  // drops the ProcessGroup reference, so that torch.distributed.destroy_process_group()
  // tears the group down deterministically (not at interpreter exit)
  void Finalize() override;
  // RCCL: one grouped send / receive with every peer (and self) at context creation, so the first
  // shuffle of a job does not pay the communicator's lazy p2p connection setup while its transfers
  // should be overlapping compute (the first step's overlap, profiles/r05/first_step_overlap.txt)
  void WarmUp();
  at::Device comm_device() const { return device_; }

 private:
  at::Tensor to_comm(const at::Tensor &t) const;
  c10d::ProcessGroup &pg() const;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  CommType type_;
  at::Device device_;
  int rank_;
  int world_;
};

}  // namespace net
}  // namespace cylon
