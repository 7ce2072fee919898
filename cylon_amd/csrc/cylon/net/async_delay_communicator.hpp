// Asynchronous loopback test transport.
//
// With one GPU per box, RCCL never runs at world > 1 in the tests (two RCCL ranks
// cannot share a device), so the overlapped exchange code -- chunk k consumed while
// chunk k+1 is in flight, stream-ordered request waits -- would only ever see the
// synchronous gloo path.  This decorator makes every posted all-to-all genuinely
// asynchronous on the device: the inner communicator's (blocking) exchange lands in
// a staging buffer, and the caller's receive buffer is filled by a side HIP stream
// after a spin-delay kernel; the returned request is backed by a HIP event, its
// Test() queries the event and its Wait() is a stream wait (hipStreamWaitEvent) of
// the caller's current stream -- exactly RCCL's completion semantics.  The receive
// buffer starts out poisoned (0xFF bytes), so a consumer that reads before waiting
// sees garbage instead of the right answer.
#pragma once
#include "communicator.hpp"

namespace cylon {
namespace net {

class AsyncDelayCommunicator : public Communicator {
 public:
  AsyncDelayCommunicator(std::shared_ptr<Communicator> inner, double delay_us)
      : inner_(std::move(inner)), delay_us_(delay_us) {}
  ~AsyncDelayCommunicator() override;
  int GetRank() const override { return inner_->GetRank(); }
  int GetWorldSize() const override { return inner_->GetWorldSize(); }
  CommType GetCommType() const override { return inner_->GetCommType(); }
  void Barrier() override { inner_->Barrier(); }
  void Finalize() override { inner_->Finalize(); }
  at::Tensor AllToAllV(const at::Tensor &s, const std::vector<int64_t> &sc, const std::vector<int64_t> &rc) override {
    return inner_->AllToAllV(s, sc, rc);
  }
  std::pair<at::Tensor, std::shared_ptr<P2PRequest>> AllToAllVAsync(const at::Tensor &s,
                                                                    const std::vector<int64_t> &sc,
                                                                    const std::vector<int64_t> &rc) override;
  std::shared_ptr<P2PRequest> AllToAllVSegmentsAsync(const at::Tensor &send, const std::vector<int64_t> &soff,
                                                     const std::vector<int64_t> &scnt, const at::Tensor &recv,
                                                     const std::vector<int64_t> &roff,
                                                     const std::vector<int64_t> &rcnt) override;
  std::vector<int64_t> ExchangeCounts(const std::vector<int64_t> &c) override { return inner_->ExchangeCounts(c); }
  void AllReduce(at::Tensor &t, ReduceOp op) override { inner_->AllReduce(t, op); }
  at::Tensor AllGather(const at::Tensor &in) override { return inner_->AllGather(in); }
  void Broadcast(at::Tensor &t, int root) override { inner_->Broadcast(t, root); }
  std::shared_ptr<P2PRequest> ISend(const at::Tensor &t, int dst, int tag) override { return inner_->ISend(t, dst, tag); }
  std::shared_ptr<P2PRequest> IRecv(at::Tensor &t, int src, int tag) override { return inner_->IRecv(t, src, tag); }

  int64_t posted() const { return posted_; }
  // requests whose Test() was false at their first poll (i.e. observed in flight)
  int64_t observed_in_flight() const { return *in_flight_seen_; }

 private:
  std::shared_ptr<Communicator> inner_;
  double delay_us_;
  void *side_ = nullptr;  // hipStream_t, created on first use
  int side_dev_ = -1;
  int64_t posted_ = 0;
  void *side_stream(int dev);
  std::shared_ptr<int64_t> in_flight_seen_ = std::make_shared<int64_t>(0);
};

}  // namespace net
}  // namespace cylon
