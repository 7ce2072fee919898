// Asynchronous loopback test transport (see async_delay_communicator.hpp).
#include "async_delay_communicator.hpp"

#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include "../kernels/kernels.hpp"

namespace cylon {
namespace net {

#define ADC_HIP(expr)                                                                               \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    CYLON_CHECK(_e == hipSuccess, Code::ExecutionError, #expr << ": " << hipGetErrorString(_e));    \
  } while (0)

namespace {
class DoneReq : public P2PRequest {
 public:
  bool Test() override { return true; }
  void Wait() override {}
};

class EventRequest : public P2PRequest {
 public:
  EventRequest(hipEvent_t ev, at::Tensor staged, at::Tensor out, int dev, std::shared_ptr<int64_t> seen)
      : ev_(ev), staged_(std::move(staged)), out_(std::move(out)), dev_(dev), seen_(std::move(seen)) {}
  ~EventRequest() override {
    // never let the staging / receive buffers return to the allocator under a live copy
    if (!waited_) (void)hipEventSynchronize(ev_);
    (void)hipEventDestroy(ev_);
  }
  bool Test() override {
    const hipError_t q = hipEventQuery(ev_);
    CYLON_CHECK(q == hipSuccess || q == hipErrorNotReady, Code::ExecutionError, "event query: " << hipGetErrorString(q));
    if (!polled_) {
      polled_ = true;
      if (q == hipErrorNotReady) ++*seen_;
    }
    return q == hipSuccess;
  }
  void Wait() override {
    if (waited_) return;
    if (!polled_) Test();
    hipStream_t cur = c10::hip::getCurrentHIPStream(dev_).stream();
    ADC_HIP(hipStreamWaitEvent(cur, ev_, 0));  // stream-ordered, the host does not block
    waited_ = true;
  }

 private:
  hipEvent_t ev_;
  at::Tensor staged_, out_;
  int dev_;
  std::shared_ptr<int64_t> seen_;
  bool waited_ = false, polled_ = false;
};
}  // namespace

AsyncDelayCommunicator::~AsyncDelayCommunicator() {
  if (side_) (void)hipStreamDestroy(reinterpret_cast<hipStream_t>(side_));
}

void *AsyncDelayCommunicator::side_stream(int dev) {
  if (!side_ || side_dev_ != dev) {
    hipStream_t st;
    ADC_HIP(hipSetDevice(dev));
    ADC_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    side_ = st;
    side_dev_ = dev;
  }
  return side_;
}

// segments: the inner exchange lands in a staging buffer; the caller's receive segments are
// poisoned now and filled on the side stream after the delay
std::shared_ptr<P2PRequest> AsyncDelayCommunicator::AllToAllVSegmentsAsync(
    const at::Tensor &send, const std::vector<int64_t> &soff, const std::vector<int64_t> &scnt,
    const at::Tensor &recv, const std::vector<int64_t> &roff, const std::vector<int64_t> &rcnt) {
  if (!recv.is_cuda()) return inner_->AllToAllVSegmentsAsync(send, soff, scnt, recv, roff, rcnt);
  const int w = GetWorldSize();
  std::vector<at::Tensor> pieces;
  for (int r = 0; r < w; ++r) pieces.push_back(send.slice(0, soff[r], soff[r] + scnt[r]));
  at::Tensor staged = inner_->AllToAllV(at::cat(pieces), scnt, rcnt);
  const int dev = recv.device().index();
  hipStream_t side = reinterpret_cast<hipStream_t>(side_stream(dev));
  hipStream_t cur = c10::hip::getCurrentHIPStream(dev).stream();
  const int64_t es = recv.element_size();
  uint8_t *rb = reinterpret_cast<uint8_t *>(recv.data_ptr());
  for (int r = 0; r < w; ++r)
    if (rcnt[r]) ADC_HIP(hipMemsetAsync(rb + roff[r] * es, 0xff, (size_t)(rcnt[r] * es), cur));  // poison
  hipEvent_t ready, done;
  ADC_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  ADC_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  ADC_HIP(hipEventRecord(ready, cur));
  ADC_HIP(hipStreamWaitEvent(side, ready, 0));
  (void)hipEventDestroy(ready);
  hip::spin_delay_us(delay_us_, side);
  const uint8_t *sb = reinterpret_cast<const uint8_t *>(staged.data_ptr());
  int64_t at_ = 0;
  for (int r = 0; r < w; ++r) {
    if (rcnt[r])
      ADC_HIP(hipMemcpyAsync(rb + roff[r] * es, sb + at_ * es, (size_t)(rcnt[r] * es), hipMemcpyDeviceToDevice, side));
    at_ += rcnt[r];
  }
  ADC_HIP(hipEventRecord(done, side));
  ++posted_;
  return std::make_shared<EventRequest>(done, staged, recv, dev, in_flight_seen_);
}

std::pair<at::Tensor, std::shared_ptr<P2PRequest>> AsyncDelayCommunicator::AllToAllVAsync(
    const at::Tensor &s, const std::vector<int64_t> &sc, const std::vector<int64_t> &rc) {
  at::Tensor staged = inner_->AllToAllV(s, sc, rc);
  if (!staged.is_cuda()) return {staged, std::make_shared<DoneReq>()};  // host tables: nothing to overlap
  const int dev = staged.device().index();
  hipStream_t side = reinterpret_cast<hipStream_t>(side_stream(dev));
  hipStream_t cur = c10::hip::getCurrentHIPStream(dev).stream();
  at::Tensor out = at::empty_like(staged);
  const size_t nb = (size_t)staged.numel() * staged.element_size();
  if (nb) ADC_HIP(hipMemsetAsync(out.data_ptr(), 0xff, nb, cur));  // poison
  hipEvent_t ready, done;
  ADC_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  ADC_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  ADC_HIP(hipEventRecord(ready, cur));
  ADC_HIP(hipStreamWaitEvent(side, ready, 0));
  (void)hipEventDestroy(ready);
  hip::spin_delay_us(delay_us_, side);
  if (nb) ADC_HIP(hipMemcpyAsync(out.data_ptr(), staged.data_ptr(), nb, hipMemcpyDeviceToDevice, side));
  ADC_HIP(hipEventRecord(done, side));
  ++posted_;
  return {out, std::make_shared<EventRequest>(done, staged, out, dev, in_flight_seen_)};
}

}  // namespace net
}  // namespace cylon
