// Full-mesh TCP communicator (see tcp_communicator.hpp).
#include "cylon/knobs.hpp"
#include "tcp_communicator.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <torch/csrc/distributed/c10d/Store.hpp>

namespace cylon {
namespace net {

namespace {

void write_all(int fd, const void *p, int64_t n) {
  const uint8_t *b = static_cast<const uint8_t *>(p);
  while (n > 0) {
    const ssize_t w = ::send(fd, b, (size_t)std::min<int64_t>(n, int64_t(1) << 30), MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    CYLON_CHECK(w > 0, Code::IOError, "tcp send failed: " << std::strerror(errno));
    b += w;
    n -= w;
  }
}

// false on orderly EOF before any byte
bool read_all(int fd, void *p, int64_t n) {
  uint8_t *b = static_cast<uint8_t *>(p);
  int64_t got = 0;
  while (got < n) {
    const ssize_t r = ::recv(fd, b + got, (size_t)std::min<int64_t>(n - got, int64_t(1) << 30), 0);
    if (r < 0 && errno == EINTR) continue;
    if (r == 0 && got == 0) return false;
    CYLON_CHECK(r > 0, Code::IOError, "tcp receive failed: " << (r == 0 ? "peer closed" : std::strerror(errno)));
    got += r;
  }
  return true;
}

void tune(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 4 << 20;
  ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

// address other ranks can reach this one at: the local end of a (UDP, unsent)
// connection towards the rendezvous host, i.e. the interface that routes there
std::string local_address(const std::string &master) {
  if (const char *h = knobs::Get("TCP_HOST")) return h;
  if (master.empty() || master == "127.0.0.1" || master == "localhost") return "127.0.0.1";
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_DGRAM;
  if (::getaddrinfo(master.c_str(), "9", &hints, &res) != 0 || !res) return "127.0.0.1";
  std::string out = "127.0.0.1";
  int fd = ::socket(AF_INET, SOCK_DGRAM, 0);
  if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
    sockaddr_in a{};
    socklen_t len = sizeof(a);
    if (::getsockname(fd, reinterpret_cast<sockaddr *>(&a), &len) == 0) {
      char buf[INET_ADDRSTRLEN];
      if (::inet_ntop(AF_INET, &a.sin_addr, buf, sizeof(buf))) out = buf;
    }
  }
  if (fd >= 0) ::close(fd);
  ::freeaddrinfo(res);
  return out;
}

std::vector<uint8_t> to_bytes(const std::string &s) { return std::vector<uint8_t>(s.begin(), s.end()); }

class DoneReq : public P2PRequest {
 public:
  bool Test() override { return true; }
  void Wait() override {}
};

class TcpRecvReq : public P2PRequest {
 public:
  TcpRecvReq(TcpCommunicator *c, at::Tensor t, int src, int64_t tag) : c_(c), t_(std::move(t)), src_(src), tag_(tag) {}
  bool Test() override {
    if (done_) return true;
    std::vector<uint8_t> b;
    if (!c_->TryRecvFrame(src_, tag_, b)) return false;
    land(b);
    return true;
  }
  void Wait() override {
    if (done_) return;
    land(c_->RecvFrame(src_, tag_));
  }

 private:
  void land(const std::vector<uint8_t> &b) {
    const int64_t nb = t_.numel() * (int64_t)t_.element_size();
    CYLON_CHECK((int64_t)b.size() == nb, Code::IOError,
                "tcp receive of " << b.size() << " bytes into a " << nb << "-byte tensor");
    at::Tensor host = t_.is_cpu() && t_.is_contiguous() ? t_ : at::empty(t_.sizes(), t_.options().device(at::kCPU));
    if (nb) std::memcpy(host.data_ptr(), b.data(), (size_t)nb);
    if (!host.is_same(t_)) t_.copy_(host);
    done_ = true;
  }
  TcpCommunicator *c_;
  at::Tensor t_;
  int src_;
  int64_t tag_;
  bool done_ = false;
};

}  // namespace

TcpCommunicator::TcpCommunicator(c10::intrusive_ptr<c10d::Store> store, int rank, int world, double timeout_s)
    : store_(store), rank_(rank), world_(world), timeout_s_(timeout_s) {
  CYLON_CHECK(world >= 1 && rank >= 0 && rank < world, Code::Invalid, "bad rank " << rank << " of " << world);
  peers_.resize(world);
  peer_error_.resize(world);
  for (auto &p : peers_) p = std::make_unique<Peer>();
  if (world == 1) return;
  const char *ma = std::getenv("MASTER_ADDR");
  const std::string host = local_address(ma ? ma : "");
  int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  CYLON_CHECK(lfd >= 0, Code::IOError, "socket: " << std::strerror(errno));
  int one = 1;
  ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = 0;
  CYLON_CHECK(::bind(lfd, reinterpret_cast<sockaddr *>(&a), sizeof(a)) == 0, Code::IOError,
              "bind: " << std::strerror(errno));
  CYLON_CHECK(::listen(lfd, world) == 0, Code::IOError, "listen: " << std::strerror(errno));
  socklen_t len = sizeof(a);
  ::getsockname(lfd, reinterpret_cast<sockaddr *>(&a), &len);
  const int port = ntohs(a.sin_port);
  store->set("cylon_tcp/addr/" + std::to_string(rank), to_bytes(host + ":" + std::to_string(port)));

  // connect to every lower rank (send our rank as the hello)
  for (int p = 0; p < rank; ++p) {
    const std::string key = "cylon_tcp/addr/" + std::to_string(p);
    store->wait({key});
    const std::vector<uint8_t> v = store->get(key);
    const std::string hp(v.begin(), v.end());
    const size_t colon = hp.rfind(':');
    const std::string ph = hp.substr(0, colon);
    const int pp = std::atoi(hp.c_str() + colon + 1);
    int fd = -1;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      fd = ::socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in pa{};
      pa.sin_family = AF_INET;
      pa.sin_port = htons((uint16_t)pp);
      ::inet_pton(AF_INET, ph.c_str(), &pa.sin_addr);
      if (::connect(fd, reinterpret_cast<sockaddr *>(&pa), sizeof(pa)) == 0) break;
      ::close(fd);
      fd = -1;
      CYLON_CHECK(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < timeout_s_,
                  Code::IOError, "tcp connect to rank " << p << " at " << hp << " timed out");
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    tune(fd);
    const int32_t me = rank;
    write_all(fd, &me, sizeof(me));
    peers_[p]->fd = fd;
  }
  // accept every higher rank
  for (int k = rank + 1; k < world; ++k) {
    pollfd pf{lfd, POLLIN, 0};
    const int rc = ::poll(&pf, 1, (int)std::min(timeout_s_ * 1000.0, 2.0e9));
    CYLON_CHECK(rc > 0, Code::IOError, "tcp accept timed out waiting for " << (world - k) << " peer(s)");
    int fd = ::accept(lfd, nullptr, nullptr);
    CYLON_CHECK(fd >= 0, Code::IOError, "accept: " << std::strerror(errno));
    tune(fd);
    int32_t who = -1;
    CYLON_CHECK(read_all(fd, &who, sizeof(who)) && who > rank && who < world && peers_[who]->fd < 0, Code::IOError,
                "bad tcp hello " << who);
    peers_[who]->fd = fd;
  }
  ::close(lfd);
  for (int p = 0; p < world; ++p)
    if (p != rank) peers_[p]->reader = std::thread([this, p] { reader_loop(p); });
}

TcpCommunicator::~TcpCommunicator() { Finalize(); }

void TcpCommunicator::Finalize() {
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (closed_) return;
    closed_ = true;
  }
  for (auto &p : peers_)
    if (p && p->fd >= 0) ::shutdown(p->fd, SHUT_RDWR);
  for (auto &p : peers_)
    if (p && p->reader.joinable()) p->reader.join();
  for (auto &p : peers_)
    if (p && p->fd >= 0) {
      ::close(p->fd);
      p->fd = -1;
    }
  q_cv_.notify_all();
}

void TcpCommunicator::reader_loop(int peer) {
  const int fd = peers_[peer]->fd;
  try {
    for (;;) {
      int64_t hdr[2];
      if (!read_all(fd, hdr, sizeof(hdr))) break;
      // a frame is never larger than one host buffer can be (64 GiB sanity cap)
      CYLON_CHECK(hdr[1] >= 0 && hdr[1] <= (int64_t(1) << 36), Code::IOError,
                  "tcp frame from rank " << peer << " has a bad length " << hdr[1]);
      std::vector<uint8_t> b((size_t)hdr[1]);
      // EOF between a header and its payload is a peer failure, never an empty frame
      if (hdr[1]) CYLON_CHECK(read_all(fd, b.data(), hdr[1]), Code::IOError,
                              "rank " << peer << " closed the connection inside a frame");
      {
        std::lock_guard<std::mutex> lk(q_mu_);
        queues_[{peer, hdr[0]}].push_back(std::move(b));
      }
      q_cv_.notify_all();
    }
  } catch (const std::exception &e) {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (!closed_) peer_error_[peer] = e.what();
  }
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (peer_error_[peer].empty() && !closed_) peer_error_[peer] = "connection closed by rank " + std::to_string(peer);
  }
  q_cv_.notify_all();
}

void TcpCommunicator::SendFrame(int peer, int64_t tag, const void *data, int64_t bytes) {
  CYLON_CHECK(peer >= 0 && peer < world_ && peer != rank_, Code::Invalid, "bad tcp peer " << peer);
  Peer &p = *peers_[peer];
  std::lock_guard<std::mutex> lk(p.send_mu);
  const int64_t hdr[2] = {tag, bytes};
  write_all(p.fd, hdr, sizeof(hdr));
  if (bytes) write_all(p.fd, data, bytes);
}

bool TcpCommunicator::TryRecvFrame(int peer, int64_t tag, std::vector<uint8_t> &out) {
  std::lock_guard<std::mutex> lk(q_mu_);
  auto it = queues_.find({peer, tag});
  if (it == queues_.end() || it->second.empty()) {
    CYLON_CHECK(peer_error_[peer].empty(), Code::IOError, "tcp peer " << peer << ": " << peer_error_[peer]);
    return false;
  }
  out = std::move(it->second.front());
  it->second.pop_front();
  if (it->second.empty()) queues_.erase(it);
  return true;
}

std::vector<uint8_t> TcpCommunicator::RecvFrame(int peer, int64_t tag) {
  auto region = EnterBlocking();
  std::unique_lock<std::mutex> lk(q_mu_);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s_);
  for (;;) {
    auto it = queues_.find({peer, tag});
    if (it != queues_.end() && !it->second.empty()) {
      std::vector<uint8_t> b = std::move(it->second.front());
      it->second.pop_front();
      if (it->second.empty()) queues_.erase(it);
      return b;
    }
    CYLON_CHECK(peer_error_[peer].empty(), Code::IOError, "tcp peer " << peer << ": " << peer_error_[peer]);
    CYLON_CHECK(!closed_, Code::Invalid, "communicator used after finalize()");
    CYLON_CHECK(std::chrono::steady_clock::now() < deadline, Code::ExecutionError,
                "tcp receive from rank " << peer << " timed out after " << timeout_s_ << " s");
    q_cv_.wait_until(lk, deadline);
  }
}

std::vector<std::vector<uint8_t>> TcpCommunicator::exchange(
    const std::vector<std::pair<const uint8_t *, int64_t>> &blocks) {
  const int64_t tag = next_coll_tag();
  std::vector<std::vector<uint8_t>> out(world_);
  // staggered send order (reference all_to_all.cpp: (t + rank) % n) spreads the load
  for (int s = 1; s < world_; ++s) {
    const int p = (rank_ + s) % world_;
    SendFrame(p, tag, blocks[p].first, blocks[p].second);
  }
  out[rank_].assign(blocks[rank_].first, blocks[rank_].first + blocks[rank_].second);
  for (int s = 1; s < world_; ++s) {
    const int p = (rank_ - s + world_) % world_;
    out[p] = RecvFrame(p, tag);
  }
  return out;
}

static at::Tensor host_contig(const at::Tensor &t) {
  at::Tensor h = t.is_cpu() ? t : t.to(at::kCPU);
  return h.contiguous();
}

at::Tensor TcpCommunicator::AllToAllV(const at::Tensor &send, const std::vector<int64_t> &send_counts,
                                      const std::vector<int64_t> &recv_counts) {
  CYLON_CHECK((int)send_counts.size() == world_ && (int)recv_counts.size() == world_, Code::Invalid,
              "all-to-all counts must have world-size entries");
  at::Tensor h = host_contig(send);
  const int64_t row = h.dim() == 0 ? h.element_size() : (h.numel() / std::max<int64_t>(h.size(0), 1)) * h.element_size();
  std::vector<std::pair<const uint8_t *, int64_t>> blocks(world_);
  const uint8_t *base = static_cast<const uint8_t *>(h.data_ptr());
  int64_t off = 0;
  for (int p = 0; p < world_; ++p) {
    blocks[p] = {base + off * row, send_counts[p] * row};
    off += send_counts[p];
  }
  auto got = exchange(blocks);
  int64_t total = 0;
  for (auto c : recv_counts) total += c;
  std::vector<int64_t> shape(h.sizes().begin(), h.sizes().end());
  if (shape.empty()) shape.push_back(0);
  shape[0] = total;
  at::Tensor out = at::empty(shape, h.options());
  uint8_t *o = static_cast<uint8_t *>(out.data_ptr());
  for (int p = 0; p < world_; ++p) {
    CYLON_CHECK((int64_t)got[p].size() == recv_counts[p] * row, Code::IOError,
                "all-to-all: rank " << p << " sent " << got[p].size() << " bytes, expected " << recv_counts[p] * row);
    if (!got[p].empty()) std::memcpy(o, got[p].data(), got[p].size());
    o += got[p].size();
  }
  return send.is_cpu() ? out : out.to(send.device());
}

std::vector<int64_t> TcpCommunicator::ExchangeCounts(const std::vector<int64_t> &send_counts) {
  CYLON_CHECK((int)send_counts.size() == world_, Code::Invalid, "counts must have world-size entries");
  std::vector<std::pair<const uint8_t *, int64_t>> blocks(world_);
  for (int p = 0; p < world_; ++p) blocks[p] = {reinterpret_cast<const uint8_t *>(&send_counts[p]), 8};
  auto got = exchange(blocks);
  std::vector<int64_t> r(world_);
  for (int p = 0; p < world_; ++p) std::memcpy(&r[p], got[p].data(), 8);
  return r;
}

at::Tensor TcpCommunicator::AllGather(const at::Tensor &in) {
  at::Tensor h = host_contig(in.dim() == 0 ? in.reshape({1}) : in);
  const int64_t nb = h.numel() * (int64_t)h.element_size();
  std::vector<std::pair<const uint8_t *, int64_t>> blocks(world_, {static_cast<const uint8_t *>(h.data_ptr()), nb});
  auto got = exchange(blocks);
  std::vector<int64_t> shape(h.sizes().begin(), h.sizes().end());
  shape[0] *= world_;
  at::Tensor out = at::empty(shape, h.options());
  uint8_t *o = static_cast<uint8_t *>(out.data_ptr());
  for (int p = 0; p < world_; ++p) {
    CYLON_CHECK((int64_t)got[p].size() == nb, Code::IOError, "all-gather: rank " << p << " sent a different size");
    if (nb) std::memcpy(o + p * nb, got[p].data(), (size_t)nb);
  }
  return in.is_cpu() ? out : out.to(in.device());
}

void TcpCommunicator::AllReduce(at::Tensor &t, ReduceOp op) {
  if (world_ == 1) return;
  at::Tensor g = AllGather(t.reshape({-1})).to(at::kCPU).reshape({world_, -1});
  const bool is_bool = g.scalar_type() == at::kBool;
  if (is_bool) g = g.to(at::kByte);
  at::Tensor r;
  switch (op) {
    case ReduceOp::SUM: r = g.sum(0, false, g.scalar_type()); break;
    case ReduceOp::MIN: r = std::get<0>(g.min(0)); break;
    case ReduceOp::MAX: r = std::get<0>(g.max(0)); break;
    case ReduceOp::PROD: r = g.prod(0, false, g.scalar_type()); break;
  }
  if (is_bool) r = r.to(at::kBool);
  t.copy_(r.reshape(t.sizes()));
}

void TcpCommunicator::Barrier() {
  if (world_ == 1) return;
  uint8_t b = 1;
  std::vector<std::pair<const uint8_t *, int64_t>> blocks(world_, {&b, 1});
  exchange(blocks);
}

void TcpCommunicator::Broadcast(at::Tensor &t, int root) {
  if (world_ == 1) return;
  const int64_t tag = next_coll_tag();
  if (rank_ == root) {
    at::Tensor h = host_contig(t);
    for (int p = 0; p < world_; ++p)
      if (p != rank_) SendFrame(p, tag, h.data_ptr(), h.numel() * (int64_t)h.element_size());
    return;
  }
  std::vector<uint8_t> b = RecvFrame(root, tag);
  at::Tensor h = at::empty(t.sizes(), t.options().device(at::kCPU));
  CYLON_CHECK((int64_t)b.size() == h.numel() * (int64_t)h.element_size(), Code::IOError, "broadcast size mismatch");
  if (!b.empty()) std::memcpy(h.data_ptr(), b.data(), b.size());
  t.copy_(h);
}

std::shared_ptr<P2PRequest> TcpCommunicator::ISend(const at::Tensor &t, int dst, int tag) {
  CYLON_CHECK(tag >= 0, Code::Invalid, "point-to-point tags must be >= 0");
  at::Tensor h = host_contig(t);
  // the peer's reader thread buffers the frame, so the send completes without a matching receive
  SendFrame(dst, tag, h.data_ptr(), h.numel() * (int64_t)h.element_size());
  return std::make_shared<DoneReq>();
}

std::shared_ptr<P2PRequest> TcpCommunicator::IRecv(at::Tensor &t, int src, int tag) {
  CYLON_CHECK(src >= 0 && src < world_ && src != rank_, Code::Invalid, "bad receive source " << src);
  CYLON_CHECK(tag >= 0, Code::Invalid, "point-to-point tags must be >= 0");
  return std::make_shared<TcpRecvReq>(this, t, src, tag);
}

}  // namespace net
}  // namespace cylon
