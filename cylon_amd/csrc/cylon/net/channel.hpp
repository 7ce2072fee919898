// Point-to-point message channel (C4 Channel / Buffer / TxRequest).
//
// Reference: cpp/src/cylon/net/channel.hpp:25-117 (Channel, send / sendFin /
// progressSends / progressReceives / close, send and receive callbacks),
// TxRequest.hpp:25-60 (target, buffer, length, header[6]), mpi/mpi_channel.cpp
// (an 8-int header message, then the payload, per request; polled progress).
//
// Here the transport is the communicator's point-to-point path (c10d
// send/recv: RCCL p2p over xGMI on MI355X, gloo on CPU).  Wire format per
// request: one int64[8] header {payload bytes, fin, h0..h5} then, if non-empty,
// the payload as raw bytes; the header and the payload share the edge tag and
// are matched in posting order.  The channel is progressed by polling like the
// reference, and the bulk table shuffle does not use it (that is one
// all_to_all_v per column, see communicator.hpp).
#pragma once
#include <ATen/ATen.h>

#include <deque>
#include <map>
#include <memory>
#include <vector>

#include "communicator.hpp"

namespace cylon {
namespace net {

constexpr int kChannelHeaderInts = 6;

struct TxRequest {
  int target = -1;
  at::Tensor buffer;             // payload (any dtype, sent as its raw bytes); undefined = empty
  std::vector<int32_t> header;   // up to kChannelHeaderInts user values
  TxRequest() = default;
  TxRequest(int t, at::Tensor b, std::vector<int32_t> h) : target(t), buffer(std::move(b)), header(std::move(h)) {}
};

class ChannelReceiveCallback {
 public:
  virtual ~ChannelReceiveCallback() = default;
  // a message header arrived (finished = 1 for the sender's FIN)
  virtual void receivedHeader(int source, int finished, const std::vector<int32_t> &header) = 0;
  // the payload of the last header from `source` arrived (uint8 tensor)
  virtual void receivedData(int source, const at::Tensor &buffer) = 0;
};

class ChannelSendCallback {
 public:
  virtual ~ChannelSendCallback() = default;
  virtual void sendComplete(const std::shared_ptr<TxRequest> &req) = 0;
  virtual void sendFinishComplete(const std::shared_ptr<TxRequest> &req) = 0;
};

class Channel {
 public:
  // payloads are received on `payload_device`
  Channel(std::shared_ptr<Communicator> comm, at::Device payload_device);
  void init(int edge, const std::vector<int> &receives, const std::vector<int> &send_ids,
            ChannelReceiveCallback *rcv, ChannelSendCallback *snd);
  // queue a request; returns 1 (accepted)
  int send(std::shared_ptr<TxRequest> req);
  // queue the FIN for req->target (after every earlier request to it)
  int sendFin(std::shared_ptr<TxRequest> req);
  void progressSends();
  void progressReceives();
  // true once every FIN was sent and received
  bool isComplete() const;
  void close();

 private:
  struct Out {
    std::shared_ptr<TxRequest> req;
    bool fin = false;
    at::Tensor header, payload;
    std::vector<std::shared_ptr<P2PRequest>> ops;
  };
  struct SendState {
    std::deque<Out> pending;
    std::unique_ptr<Out> current;
    bool fin_done = false;
  };
  struct RecvState {
    enum Phase { HEADER, DATA, DONE } phase = HEADER;
    at::Tensor header, data;
    std::shared_ptr<P2PRequest> op;
  };
  std::shared_ptr<Communicator> comm_;
  at::Device dev_;
  int edge_ = 0;
  ChannelReceiveCallback *rcv_ = nullptr;
  ChannelSendCallback *snd_ = nullptr;
  std::map<int, SendState> sends_;
  std::map<int, RecvState> recvs_;
};

}  // namespace net
}  // namespace cylon
