// Point-to-point channel (C4): see channel.hpp.
#include "channel.hpp"

namespace cylon {
namespace net {

Channel::Channel(std::shared_ptr<Communicator> comm, at::Device payload_device)
    : comm_(std::move(comm)), dev_(payload_device) {}

void Channel::init(int edge, const std::vector<int> &receives, const std::vector<int> &send_ids,
                   ChannelReceiveCallback *rcv, ChannelSendCallback *snd) {
  edge_ = edge;
  rcv_ = rcv;
  snd_ = snd;
  sends_.clear();
  recvs_.clear();
  for (int t : send_ids) sends_[t];
  for (int s : receives) recvs_[s];
}

static at::Tensor as_bytes(const at::Tensor &t) {
  at::Tensor c = t.contiguous().view({-1});
  return c.scalar_type() == at::kByte ? c : c.view(at::kByte);
}

int Channel::send(std::shared_ptr<TxRequest> req) {
  CYLON_CHECK(req && sends_.count(req->target), Code::Invalid, "channel: target not in the send set");
  CYLON_CHECK((int)req->header.size() <= kChannelHeaderInts, Code::Invalid, "channel: header too long");
  Out o;
  o.req = std::move(req);
  sends_[o.req->target].pending.push_back(std::move(o));
  return 1;
}

int Channel::sendFin(std::shared_ptr<TxRequest> req) {
  CYLON_CHECK(req && sends_.count(req->target), Code::Invalid, "channel: target not in the send set");
  Out o;
  o.req = std::move(req);
  o.fin = true;
  sends_[o.req->target].pending.push_back(std::move(o));
  return 1;
}

void Channel::progressSends() {
  for (auto &kv : sends_) {
    const int target = kv.first;
    SendState &st = kv.second;
    if (st.current) {
      bool done = true;
      for (auto &op : st.current->ops) done = op->Test() && done;
      if (!done) continue;
      std::unique_ptr<Out> fin = std::move(st.current);
      if (fin->fin) {
        st.fin_done = true;
        if (snd_) snd_->sendFinishComplete(fin->req);
      } else if (snd_) {
        snd_->sendComplete(fin->req);
      }
    }
    if (st.current || st.pending.empty()) continue;
    st.current.reset(new Out(std::move(st.pending.front())));
    st.pending.pop_front();
    Out &o = *st.current;
    at::Tensor pay = (!o.fin && o.req->buffer.defined()) ? as_bytes(o.req->buffer) : at::Tensor();
    const int64_t nbytes = pay.defined() ? pay.numel() : 0;
    o.header = at::zeros({2 + kChannelHeaderInts}, at::TensorOptions().dtype(at::kLong));
    int64_t *h = o.header.data_ptr<int64_t>();
    h[0] = nbytes;
    h[1] = o.fin ? 1 : 0;
    for (size_t i = 0; i < o.req->header.size(); ++i) h[2 + i] = o.req->header[i];
    o.ops.push_back(comm_->ISend(o.header, target, edge_));
    if (nbytes > 0) {
      o.payload = pay;
      o.ops.push_back(comm_->ISend(o.payload, target, edge_));
    }
  }
}

void Channel::progressReceives() {
  for (auto &kv : recvs_) {
    const int source = kv.first;
    RecvState &st = kv.second;
    if (st.phase == RecvState::DONE) continue;
    if (!st.op) {
      if (st.phase == RecvState::HEADER) {
        st.header = at::zeros({2 + kChannelHeaderInts}, at::TensorOptions().dtype(at::kLong));
        st.op = comm_->IRecv(st.header, source, edge_);
      }
      continue;
    }
    if (!st.op->Test()) continue;
    st.op.reset();
    if (st.phase == RecvState::HEADER) {
      const int64_t *h = st.header.data_ptr<int64_t>();
      const int64_t nbytes = h[0];
      const int fin = (int)h[1];
      std::vector<int32_t> hdr(kChannelHeaderInts);
      for (int i = 0; i < kChannelHeaderInts; ++i) hdr[i] = (int32_t)h[2 + i];
      if (rcv_) rcv_->receivedHeader(source, fin, hdr);
      if (fin) {
        st.phase = RecvState::DONE;
      } else if (nbytes > 0) {
        st.phase = RecvState::DATA;
        st.data = at::empty({nbytes}, at::TensorOptions().dtype(at::kByte).device(dev_));
        st.op = comm_->IRecv(st.data, source, edge_);
      } else {
        if (rcv_) rcv_->receivedData(source, at::empty({0}, at::TensorOptions().dtype(at::kByte).device(dev_)));
      }
    } else {  // DATA
      st.phase = RecvState::HEADER;
      at::Tensor d = st.data;
      st.data = at::Tensor();
      if (rcv_) rcv_->receivedData(source, d);
    }
  }
}

bool Channel::isComplete() const {
  for (const auto &kv : sends_)
    if (!kv.second.fin_done) return false;
  for (const auto &kv : recvs_)
    if (kv.second.phase != RecvState::DONE) return false;
  return true;
}

void Channel::close() {
  for (auto &kv : sends_)
    if (kv.second.current)
      for (auto &op : kv.second.current->ops) op->Wait();
  sends_.clear();
  recvs_.clear();
}

}  // namespace net
}  // namespace cylon
