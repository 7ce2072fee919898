// ProcessGroup-backed communicator (RCCL over xGMI on MI355X, gloo on CPU).
// Reference call sites replaced here: SURVEY.md §2.5 M1-M8
// (MPI_Init/Barrier/Finalize, MPI_Isend/Irecv header+payload, MPI_Allreduce).
#include <atomic>
#include <cstdlib>
#include <chrono>
#include <thread>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Types.hpp>

#include "communicator.hpp"
#include "../trace.hpp"

namespace cylon {
namespace net {

static std::atomic<BlockingHook> g_blocking_hook{nullptr};

void SetBlockingHook(BlockingHook hook) { g_blocking_hook.store(hook); }

std::unique_ptr<BlockingRegion> EnterBlocking() {
  BlockingHook h = g_blocking_hook.load();
  return h ? h() : nullptr;
}

// wait on a c10d work inside a blocking region
static void wait_work(const c10::intrusive_ptr<c10d::Work> &w) {
  auto region = EnterBlocking();
  w->wait();
}

const char *CommTypeName(CommType t) {
  switch (t) {
    case CommType::LOCAL: return "local";
    case CommType::MPI: return "mpi";
    case CommType::TCP: return "tcp";
    case CommType::UCX: return "ucx";
    case CommType::RCCL: return "rccl";
    case CommType::GLOO: return "gloo";
  }
  return "unknown";
}

std::vector<at::Tensor> Communicator::AllGatherV(const at::Tensor &in) {
  const int w = GetWorldSize();
  at::Tensor n = at::full({1}, in.size(0), at::TensorOptions().dtype(at::kLong).device(in.device()));
  at::Tensor ns = AllGather(n).to(at::kCPU);
  int64_t mx = 0;
  std::vector<int64_t> lens(w);
  for (int i = 0; i < w; ++i) {
    lens[i] = ns[i].item<int64_t>();
    mx = std::max(mx, lens[i]);
  }
  std::vector<int64_t> shape(in.sizes().begin(), in.sizes().end());
  shape[0] = mx;
  at::Tensor padded = at::zeros(shape, in.options());
  if (in.size(0)) padded.slice(0, 0, in.size(0)).copy_(in);
  at::Tensor all = AllGather(padded);
  std::vector<at::Tensor> out;
  for (int i = 0; i < w; ++i) out.push_back(all.slice(0, i * mx, i * mx + lens[i]));
  return out;
}

ProcessGroupCommunicator::ProcessGroupCommunicator(c10::intrusive_ptr<c10d::ProcessGroup> pg, CommType type,
                                                   at::Device comm_device)
    : pg_(std::move(pg)), type_(type), device_(comm_device) {
  rank_ = pg_->getRank();
  world_ = pg_->getSize();
}

ProcessGroupCommunicator::~ProcessGroupCommunicator() = default;

void ProcessGroupCommunicator::Finalize() { pg_.reset(); }

void ProcessGroupCommunicator::WarmUp() {
  if (type_ != CommType::RCCL || !device_.is_cuda()) return;
  constexpr int64_t kBytes = int64_t(4) << 20;  // per peer: large enough to use the p2p channels
  at::Tensor s = at::zeros({world_ * kBytes}, at::TensorOptions().dtype(at::kByte).device(device_));
  at::Tensor r = at::empty_like(s);
  std::vector<at::Tensor> in, out;
  for (int p = 0; p < world_; ++p) {
    in.push_back(s.slice(0, p * kBytes, (p + 1) * kBytes));
    out.push_back(r.slice(0, p * kBytes, (p + 1) * kBytes));
  }
  wait_work(pg().alltoall(out, in));
  r.sum().item<int64_t>();  // (completes on the host: the connections exist from here on)
  trace::add_counter("comm.warmup", 1);
}

c10d::ProcessGroup &ProcessGroupCommunicator::pg() const {
  CYLON_CHECK(pg_, Code::Invalid, "communicator used after finalize()");
  return *pg_;
}

at::Tensor ProcessGroupCommunicator::to_comm(const at::Tensor &t) const {
  at::Tensor c = t.device() == device_ ? t : t.to(device_);
  // bool is not a collective dtype on every backend; move it as bytes
  if (c.scalar_type() == at::kBool) c = c.view(at::kByte);
  return c.contiguous();
}

void ProcessGroupCommunicator::Barrier() {
  trace::add_counter("comm.barrier", 1);
  // an all-reduce of one element on the comm device is a barrier that works
  // identically for RCCL and gloo and orders with the current stream.
  at::Tensor t = at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(device_));
  std::vector<at::Tensor> v{t};
  wait_work(pg().allreduce(v));
  if (device_.is_cuda()) t.cpu();
}

at::Tensor ProcessGroupCommunicator::AllToAllV(const at::Tensor &send, const std::vector<int64_t> &send_counts,
                                               const std::vector<int64_t> &recv_counts) {
  trace::add_counter("comm.alltoall_blocking", 1);
  CYLON_CHECK((int)send_counts.size() == world_ && (int)recv_counts.size() == world_, Code::Invalid,
              "all-to-all counts must have world-size entries");
  int64_t total = 0;
  for (auto c : recv_counts) total += c;
  at::Tensor in = to_comm(send);
  std::vector<int64_t> shape(in.sizes().begin(), in.sizes().end());
  if (shape.empty()) shape.push_back(0);
  shape[0] = total;
  at::Tensor out = at::empty(shape, in.options());
  std::vector<int64_t> sc(send_counts), rc(recv_counts);
  wait_work(pg().alltoall_base(out, in, rc, sc));
  if (send.scalar_type() == at::kBool) out = out.view(at::kBool);
  return out.device() == send.device() ? out : out.to(send.device());
}

std::vector<int64_t> ProcessGroupCommunicator::ExchangeCounts(const std::vector<int64_t> &send_counts) {
  trace::add_counter("comm.alltoall_blocking", 1);
  CYLON_CHECK((int)send_counts.size() == world_, Code::Invalid, "counts must have world-size entries");
  at::Tensor s = at::tensor(send_counts, at::TensorOptions().dtype(at::kLong)).to(device_);
  at::Tensor r = at::empty({world_}, s.options());
  std::vector<int64_t> ones(world_, 1);
  wait_work(pg().alltoall_base(r, s, ones, ones));
  at::Tensor h = r.to(at::kCPU);
  return std::vector<int64_t>(h.data_ptr<int64_t>(), h.data_ptr<int64_t>() + world_);
}

static c10d::ReduceOp to_c10d(ReduceOp op) {
  switch (op) {
    case ReduceOp::SUM: return c10d::ReduceOp::SUM;
    case ReduceOp::MIN: return c10d::ReduceOp::MIN;
    case ReduceOp::MAX: return c10d::ReduceOp::MAX;
    case ReduceOp::PROD: return c10d::ReduceOp::PRODUCT;
  }
  return c10d::ReduceOp::SUM;
}

void ProcessGroupCommunicator::AllReduce(at::Tensor &t, ReduceOp op) {
  trace::add_counter("comm.allreduce", 1);
  at::Tensor c = to_comm(t);
  std::vector<at::Tensor> v{c};
  c10d::AllreduceOptions o;
  o.reduceOp = to_c10d(op);
  wait_work(pg().allreduce(v, o));
  if (!c.is_same(t)) t.copy_(c.view(t.scalar_type()));
}

at::Tensor ProcessGroupCommunicator::AllGather(const at::Tensor &in) {
  trace::add_counter("comm.allgather", 1);
  at::Tensor c = to_comm(in);
  std::vector<int64_t> shape(c.sizes().begin(), c.sizes().end());
  if (shape.empty()) shape.push_back(1);
  const int64_t n0 = shape[0];
  shape[0] = n0 * world_;
  at::Tensor out = at::empty(shape, c.options());
  at::Tensor src = c.dim() == 0 ? c.reshape({1}) : c;
  wait_work(pg()._allgather_base(out, src));
  if (in.scalar_type() == at::kBool) out = out.view(at::kBool);
  return out.device() == in.device() ? out : out.to(in.device());
}

void ProcessGroupCommunicator::Broadcast(at::Tensor &t, int root) {
  trace::add_counter("comm.broadcast", 1);
  at::Tensor c = to_comm(t);
  std::vector<at::Tensor> v{c};
  c10d::BroadcastOptions o;
  o.rootRank = root;
  wait_work(pg().broadcast(v, o));
  if (!c.is_same(t)) t.copy_(c.view(t.scalar_type()));
}

}  // namespace net
}  // namespace cylon

namespace cylon {
namespace net {

namespace {
class DoneRequest : public P2PRequest {
 public:
  bool Test() override { return true; }
  void Wait() override {}
};
}  // namespace

std::pair<at::Tensor, std::shared_ptr<P2PRequest>> Communicator::AllToAllVAsync(const at::Tensor &send,
                                                                                const std::vector<int64_t> &sc,
                                                                                const std::vector<int64_t> &rc) {
  return {AllToAllV(send, sc, rc), std::make_shared<DoneRequest>()};
}

static void check_segments(int world, const at::Tensor &t, const std::vector<int64_t> &off,
                           const std::vector<int64_t> &cnt, const char *what) {
  CYLON_CHECK((int)off.size() == world && (int)cnt.size() == world, Code::Invalid,
              what << " segments must have world-size entries");
  const int64_t n = t.dim() == 0 ? 1 : t.size(0);
  for (int r = 0; r < world; ++r)
    CYLON_CHECK(cnt[r] >= 0 && off[r] >= 0 && off[r] + cnt[r] <= n, Code::Invalid,
                what << " segment " << r << " [" << off[r] << ", +" << cnt[r] << ") outside " << n << " elements");
}

std::shared_ptr<P2PRequest> Communicator::AllToAllVSegmentsAsync(const at::Tensor &send,
                                                                 const std::vector<int64_t> &soff,
                                                                 const std::vector<int64_t> &scnt,
                                                                 const at::Tensor &recv,
                                                                 const std::vector<int64_t> &roff,
                                                                 const std::vector<int64_t> &rcnt) {
  const int w = GetWorldSize();
  check_segments(w, send, soff, scnt, "send");
  check_segments(w, recv, roff, rcnt, "receive");
  std::vector<at::Tensor> pieces;
  for (int r = 0; r < w; ++r) pieces.push_back(send.slice(0, soff[r], soff[r] + scnt[r]));
  at::Tensor packed = at::cat(pieces);
  auto posted = AllToAllVAsync(packed, scnt, rcnt);
  posted.second->Wait();
  const at::Tensor &got = posted.first;
  int64_t at_ = 0;
  for (int r = 0; r < w; ++r) {
    if (rcnt[r]) recv.slice(0, roff[r], roff[r] + rcnt[r]).copy_(got.slice(0, at_, at_ + rcnt[r]));
    at_ += rcnt[r];
  }
  return std::make_shared<DoneRequest>();
}

std::shared_ptr<P2PRequest> Communicator::ISend(const at::Tensor &, int, int) {
  CYLON_THROW(Code::NotImplemented, "point-to-point send needs a distributed communicator");
}

std::shared_ptr<P2PRequest> Communicator::IRecv(at::Tensor &, int, int) {
  CYLON_THROW(Code::NotImplemented, "point-to-point receive needs a distributed communicator");
}

namespace {
// A c10d work plus the staging buffers a transfer needs when the caller's tensor
// is not on the communication device (copied back once the receive completes).
// RCCL works report completion through isCompleted() (event query); gloo's
// point-to-point works only complete inside wait(), so for gloo a helper
// thread waits and Test() reads its flag.
class PGRequest : public P2PRequest {
 public:
  PGRequest(c10::intrusive_ptr<c10d::Work> w, at::Tensor staged, at::Tensor user, bool threaded)
      : work_(std::move(w)), staged_(std::move(staged)), user_(std::move(user)) {
    if (threaded) {
      st_ = std::make_shared<State>();
      auto st = st_;
      auto w2 = work_;
      std::thread([st, w2]() {
        try {
          w2->wait();  // helper thread: never holds the GIL
        } catch (...) {
          st->err = std::current_exception();
        }
        st->done.store(true);
      }).detach();
    }
  }
  bool Test() override {
    if (done_) return true;
    if (st_ ? !st_->done.load() : !work_->isCompleted()) return false;
    finish();
    return true;
  }
  void Wait() override {
    if (done_) return;
    if (st_) {
      auto region = EnterBlocking();
      while (!st_->done.load()) std::this_thread::sleep_for(std::chrono::microseconds(50));
    } else {
      wait_work(work_);
    }
    finish();
  }

 private:
  struct State {
    std::atomic<bool> done{false};
    std::exception_ptr err;
  };
  void finish() {
    done_ = true;
    if (st_ && st_->err) std::rethrow_exception(st_->err);
    if (user_.defined() && !staged_.is_same(user_)) user_.copy_(staged_.view(user_.scalar_type()));
  }
  c10::intrusive_ptr<c10d::Work> work_;
  at::Tensor staged_, user_;
  std::shared_ptr<State> st_;
  bool done_ = false;
};
}  // namespace

std::pair<at::Tensor, std::shared_ptr<P2PRequest>> ProcessGroupCommunicator::AllToAllVAsync(
    const at::Tensor &send, const std::vector<int64_t> &send_counts, const std::vector<int64_t> &recv_counts) {
  CYLON_CHECK((int)send_counts.size() == world_ && (int)recv_counts.size() == world_, Code::Invalid,
              "all-to-all counts must have world-size entries");
  trace::add_counter("comm.alltoall_posted", 1);
  int64_t total = 0;
  for (auto c : recv_counts) total += c;
  at::Tensor in = to_comm(send);
  std::vector<int64_t> shape(in.sizes().begin(), in.sizes().end());
  if (shape.empty()) shape.push_back(0);
  shape[0] = total;
  at::Tensor out = at::empty(shape, in.options());
  std::vector<int64_t> sc(send_counts), rc(recv_counts);
  auto work = pg().alltoall_base(out, in, rc, sc);
  // the receive buffer is handed out in the caller's dtype/device once waited on
  at::Tensor user = out;
  if (send.scalar_type() == at::kBool) user = out.view(at::kBool);
  if (user.device() != send.device()) {
    auto req = std::make_shared<PGRequest>(work, out, at::Tensor(), type_ != CommType::RCCL);
    req->Wait();
    return {user.to(send.device()), std::make_shared<DoneRequest>()};
  }
  if (type_ != CommType::RCCL) {
    // gloo: complete the exchange before returning.  A gloo all-to-all left in flight
    // while the caller issues further collectives deadlocked intermittently under CPU
    // oversubscription (the CPU rehearsal path only needs the semantics, not overlap).
    wait_work(work);
    return {user, std::make_shared<DoneRequest>()};
  }
  // keep `in` alive until completion: c10d works hold their tensors
  return {user, std::make_shared<PGRequest>(work, out, at::Tensor(), type_ != CommType::RCCL)};
}

std::shared_ptr<P2PRequest> ProcessGroupCommunicator::AllToAllVSegmentsAsync(
    const at::Tensor &send, const std::vector<int64_t> &soff, const std::vector<int64_t> &scnt,
    const at::Tensor &recv, const std::vector<int64_t> &roff, const std::vector<int64_t> &rcnt) {
  // gloo has no list all-to-all; a buffer off the communication device is staged anyway
  if (type_ != CommType::RCCL || send.device() != device_ || recv.device() != device_)
    return Communicator::AllToAllVSegmentsAsync(send, soff, scnt, recv, roff, rcnt);
  check_segments(world_, send, soff, scnt, "send");
  check_segments(world_, recv, roff, rcnt, "receive");
  CYLON_CHECK(send.is_contiguous() && recv.is_contiguous() && send.scalar_type() == recv.scalar_type(),
              Code::Invalid, "segment all-to-all: contiguous buffers of one dtype");
  trace::add_counter("comm.alltoall_posted", 1);
  at::Tensor s = send.scalar_type() == at::kBool ? send.view(at::kByte) : send;
  at::Tensor d = recv.scalar_type() == at::kBool ? recv.view(at::kByte) : recv;
  std::vector<at::Tensor> in, out;
  for (int r = 0; r < world_; ++r) {
    in.push_back(s.slice(0, soff[r], soff[r] + scnt[r]));
    out.push_back(d.slice(0, roff[r], roff[r] + rcnt[r]));
  }
  // ProcessGroupNCCL::alltoall: grouped ncclSend / ncclRecv per peer on the communicator's
  // stream, straight from and into the views (no staging buffer, no self copy for zero counts)
  auto work = pg().alltoall(out, in);
  return std::make_shared<PGRequest>(work, at::Tensor(), at::Tensor(), false);
}

std::shared_ptr<P2PRequest> ProcessGroupCommunicator::ISend(const at::Tensor &t, int dst, int tag) {
  CYLON_CHECK(dst >= 0 && dst < world_ && dst != rank_, Code::Invalid, "bad send target " << dst);
  at::Tensor c = to_comm(t);
  std::vector<at::Tensor> v{c};
  return std::make_shared<PGRequest>(pg().send(v, dst, tag), c, at::Tensor(), type_ != CommType::RCCL);
}

std::shared_ptr<P2PRequest> ProcessGroupCommunicator::IRecv(at::Tensor &t, int src, int tag) {
  CYLON_CHECK(src >= 0 && src < world_ && src != rank_, Code::Invalid, "bad receive source " << src);
  at::Tensor c = to_comm(t);
  const bool staged = !(c.is_same(t));
  std::vector<at::Tensor> v{c};
  return std::make_shared<PGRequest>(pg().recv(v, src, tag), c, staged ? t : at::Tensor(), type_ != CommType::RCCL);
}

}  // namespace net
}  // namespace cylon
