// epoll-driven encrypted transport (see transport.h).
#include "transport.h"

#include <stdexcept>
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>

namespace symnet {

namespace {
constexpr uint64_t kListenTag = 1ull << 62;
constexpr uint64_t kCmdTag = 1ull << 63;
constexpr size_t kMaxFrame = 8u << 20;  // bytes of one encrypted frame (message + 17-byte AEAD overhead)

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

void stream_id(const uint8_t* hh, bool initiator, uint8_t out[32]) {
  static const char kI[] = "symmetry_amd/stream/initiator";
  static const char kR[] = "symmetry_amd/stream/responder";
  const char* m = initiator ? kI : kR;
  blake2b(out, 32, (const uint8_t*)m, std::strlen(m), hh, 64);
}
}  // namespace

struct Transport::Conn {
  enum Phase { CONNECTING, HANDSHAKE, HEADER, OPEN, CLOSED } phase = CONNECTING;
  uint64_t id = 0;
  int fd = -1;
  bool initiator = false;
  bool ending = false;
  std::string host;
  int port = 0;
  std::unique_ptr<NoiseXX> hs;
  SecretStream tx, rx;
  uint8_t hh[64];
  std::string rbuf;
  size_t roff = 0;
  std::string wbuf;
  size_t woff = 0;
  std::deque<std::string> pending;  // plaintext messages written before the stream opened
  std::shared_ptr<ConnShared> shared;
  int64_t last_rx = 0, last_tx = 0;
  bool want_out = false;
  uint8_t rx_key[32];
};

Transport::Transport(const KeyPair& kp, int keepalive_ms, int timeout_ms, size_t high_watermark)
    : kp_(kp), keepalive_ms_(keepalive_ms), timeout_ms_(timeout_ms), hwm_(high_watermark) {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  event_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  cmd_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (epfd_ < 0 || event_fd_ < 0 || cmd_fd_ < 0) throw std::runtime_error("transport: epoll/eventfd failed");
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = kCmdTag;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, cmd_fd_, &ev);
  thread_ = std::thread([this] { loop(); });
}

Transport::~Transport() { close(); }

void Transport::close() {
  if (stop_.exchange(true)) return;
  wake();
  if (thread_.joinable()) thread_.join();
  for (auto& kv : conns_) {
    if (kv.second->fd >= 0) ::close(kv.second->fd);
  }
  conns_.clear();
  for (int l : listeners_) ::close(l);
  listeners_.clear();
  ::close(epfd_);
  ::close(cmd_fd_);
  ::close(event_fd_);
}

void Transport::wake() {
  uint64_t one = 1;
  ssize_t r = ::write(cmd_fd_, &one, 8);
  (void)r;
}

void Transport::push_event(Event&& e) {
  {
    std::lock_guard<std::mutex> g(ev_mu_);
    events_.push_back(std::move(e));
  }
  uint64_t one = 1;
  ssize_t r = ::write(event_fd_, &one, 8);
  (void)r;
}

std::vector<Event> Transport::poll() {
  uint64_t v;
  ssize_t r = ::read(event_fd_, &v, 8);
  (void)r;
  std::vector<Event> out;
  std::lock_guard<std::mutex> g(ev_mu_);
  out.assign(std::make_move_iterator(events_.begin()), std::make_move_iterator(events_.end()));
  events_.clear();
  return out;
}

int Transport::listen(const std::string& host, int port) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  const std::string p = std::to_string(port);
  if (getaddrinfo(host.empty() ? nullptr : host.c_str(), p.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("transport: cannot resolve listen address " + host);
  int fd = socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (bind(fd, res->ai_addr, res->ai_addrlen) != 0 || ::listen(fd, 128) != 0) {
    freeaddrinfo(res);
    ::close(fd);
    throw std::runtime_error("transport: bind/listen failed on " + host + ":" + p + ": " + std::strerror(errno));
  }
  freeaddrinfo(res);
  set_nonblock(fd);
  sockaddr_in sa{};
  socklen_t sl = sizeof sa;
  getsockname(fd, (sockaddr*)&sa, &sl);
  {
    std::lock_guard<std::mutex> g(lst_mu_);
    listeners_.push_back(fd);
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = kListenTag | (uint64_t)fd;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
  return ntohs(sa.sin_port);
}

uint64_t Transport::connect(const std::string& host, int port) {
  const uint64_t id = next_id_++;
  {
    std::lock_guard<std::mutex> g(shared_mu_);
    shared_[id] = std::make_shared<ConnShared>();
  }
  {
    std::lock_guard<std::mutex> g(cmd_mu_);
    cmds_.push_back(Cmd{Cmd::CONNECT, id, {}, host, port});
  }
  wake();
  return id;
}

void Transport::inject_fault(uint64_t id, int mode, std::string data) {
  {
    std::lock_guard<std::mutex> g(cmd_mu_);
    cmds_.push_back(Cmd{Cmd::FAULT, id, std::move(data), {}, mode});
  }
  wake();
}

bool Transport::write(uint64_t id, std::string data) {
  std::shared_ptr<ConnShared> sh;
  {
    std::lock_guard<std::mutex> g(shared_mu_);
    auto it = shared_.find(id);
    if (it == shared_.end()) return false;
    sh = it->second;
  }
  if (!sh->open.load()) return false;
  if (data.size() + SecretStream::ABYTES > kMaxFrame) throw std::runtime_error("transport: message too large");
  const size_t wire = data.size() + 3 + SecretStream::ABYTES;
  const size_t q = sh->queued.fetch_add(wire) + wire;
  {
    std::lock_guard<std::mutex> g(cmd_mu_);
    cmds_.push_back(Cmd{Cmd::WRITE, id, std::move(data), {}, 0});
  }
  wake();
  if (q >= hwm_) {
    sh->above.store(true);
    return false;
  }
  return true;
}

void Transport::end(uint64_t id) {
  {
    std::lock_guard<std::mutex> g(cmd_mu_);
    cmds_.push_back(Cmd{Cmd::END, id, {}, {}, 0});
  }
  wake();
}

void Transport::destroy(uint64_t id) {
  {
    std::lock_guard<std::mutex> g(cmd_mu_);
    cmds_.push_back(Cmd{Cmd::DESTROY, id, {}, {}, 0});
  }
  wake();
}

size_t Transport::queued(uint64_t id) {
  std::lock_guard<std::mutex> g(shared_mu_);
  auto it = shared_.find(id);
  return it == shared_.end() ? 0 : it->second->queued.load();
}

// ---------------------------------------------------------------------------------------------------
void Transport::loop() {
  epoll_event evs[64];
  while (!stop_.load()) {
    const int n = epoll_wait(epfd_, evs, 64, 100);
    for (int i = 0; i < n; ++i) {
      const uint64_t tag = evs[i].data.u64;
      if (tag == kCmdTag) {
        uint64_t v;
        ssize_t r = ::read(cmd_fd_, &v, 8);
        (void)r;
        continue;
      }
      if (tag & kListenTag) {
        on_accept((int)(tag & 0xffffffff));
        continue;
      }
      auto it = conns_.find(tag);
      if (it != conns_.end()) on_io(it->second.get(), evs[i].events);
    }
    handle_cmds();
    ticks();
  }
}

void Transport::ticks() {
  const int64_t t = now_ms();
  std::vector<Conn*> expired;
  for (auto& kv : conns_) {
    Conn* c = kv.second.get();
    if (c->phase == Conn::CLOSED) continue;
    if (timeout_ms_ > 0 && c->last_rx && t - c->last_rx > timeout_ms_) {
      expired.push_back(c);
      continue;
    }
    if (c->phase == Conn::OPEN && keepalive_ms_ > 0 && t - c->last_tx > keepalive_ms_) {
      Bytes f = c->tx.push(nullptr, 0);
      send_frame(c, f.data(), f.size());
      flush(c);
    }
  }
  for (Conn* c : expired) close_conn(c, "timeout");
  // reap closed connections
  for (auto it = conns_.begin(); it != conns_.end();) {
    if (it->second->phase == Conn::CLOSED)
      it = conns_.erase(it);
    else
      ++it;
  }
}

void Transport::handle_cmds() {
  std::deque<Cmd> cmds;
  {
    std::lock_guard<std::mutex> g(cmd_mu_);
    cmds.swap(cmds_);
  }
  for (auto& cmd : cmds) {
    if (cmd.kind == Cmd::CONNECT) {
      auto c = std::make_unique<Conn>();
      c->id = cmd.id;
      c->initiator = true;
      c->host = cmd.host;
      c->port = cmd.port;
      {
        std::lock_guard<std::mutex> g(shared_mu_);
        c->shared = shared_[cmd.id];
      }
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      const std::string p = std::to_string(cmd.port);
      if (getaddrinfo(cmd.host.c_str(), p.c_str(), &hints, &res) != 0 || !res) {
        Conn* raw = c.get();
        conns_[cmd.id] = std::move(c);
        close_conn(raw, "cannot resolve " + cmd.host);
        continue;
      }
      int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
      set_nonblock(fd);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      const int r = ::connect(fd, res->ai_addr, res->ai_addrlen);
      freeaddrinfo(res);
      c->fd = fd;
      c->last_rx = now_ms();
      Conn* raw = c.get();
      conns_[cmd.id] = std::move(c);
      if (r != 0 && errno != EINPROGRESS) {
        close_conn(raw, std::string("connect failed: ") + std::strerror(errno));
        continue;
      }
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT;
      ev.data.u64 = cmd.id;
      epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
      raw->want_out = true;
      continue;
    }
    auto it = conns_.find(cmd.id);
    if (it == conns_.end()) continue;
    Conn* c = it->second.get();
    if (c->phase == Conn::CLOSED) continue;
    if (cmd.kind == Cmd::WRITE) {
      if (c->phase != Conn::OPEN) {
        c->pending.push_back(std::move(cmd.data));
        continue;
      }
      Bytes f = c->tx.push((const uint8_t*)cmd.data.data(), cmd.data.size());
      c->shared->queued -= f.size() + 3;  // re-added by send_frame, released by flush as bytes leave
      send_frame(c, f.data(), f.size());
      c->shared->bytes_out += cmd.data.size();
    } else if (cmd.kind == Cmd::FAULT) {
      if (cmd.port == 0) {
        c->wbuf.append(cmd.data);
        if (c->shared) c->shared->queued += cmd.data.size();
      } else if (c->phase == Conn::OPEN) {
        Bytes f = c->tx.push((const uint8_t*)cmd.data.data(), cmd.data.size());
        f[f.size() / 2] ^= 0x40;
        send_frame(c, f.data(), f.size());
      }
    } else if (cmd.kind == Cmd::END) {
      c->ending = true;
    } else if (cmd.kind == Cmd::DESTROY) {
      close_conn(c, "");
      continue;
    }
    flush(c);
  }
}

void Transport::on_accept(int lfd) {
  while (true) {
    sockaddr_in sa{};
    socklen_t sl = sizeof sa;
    int fd = accept4(lfd, (sockaddr*)&sa, &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    auto c = std::make_unique<Conn>();
    c->id = next_id_++;
    c->fd = fd;
    c->initiator = false;
    char buf[64];
    inet_ntop(AF_INET, &sa.sin_addr, buf, sizeof buf);
    c->host = buf;
    c->port = ntohs(sa.sin_port);
    c->shared = std::make_shared<ConnShared>();
    {
      std::lock_guard<std::mutex> g(shared_mu_);
      shared_[c->id] = c->shared;
    }
    c->last_rx = now_ms();
    c->phase = Conn::HANDSHAKE;
    c->hs = std::make_unique<NoiseXX>(false, kp_);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = c->id;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
    conns_[c->id] = std::move(c);
  }
}

void Transport::start_handshake(Conn* c) {
  c->phase = Conn::HANDSHAKE;
  c->hs = std::make_unique<NoiseXX>(true, kp_);
  Bytes m = c->hs->write_message(nullptr, 0);
  send_frame(c, m.data(), m.size());
}

void Transport::update_interest(Conn* c) {
  const bool want = c->woff < c->wbuf.size();
  if (want == c->want_out) return;
  c->want_out = want;
  epoll_event ev{};
  ev.events = EPOLLIN | (want ? EPOLLOUT : 0);
  ev.data.u64 = c->id;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
}

void Transport::send_frame(Conn* c, const uint8_t* p, size_t n) {
  const uint8_t hdr[3] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16)};
  c->wbuf.append((const char*)hdr, 3);
  c->wbuf.append((const char*)p, n);
  c->last_tx = now_ms();
  if (c->shared) c->shared->queued += n + 3;
}

bool Transport::flush(Conn* c) {
  while (c->woff < c->wbuf.size()) {
    const ssize_t r = ::send(c->fd, c->wbuf.data() + c->woff, c->wbuf.size() - c->woff, MSG_NOSIGNAL);
    if (r > 0) {
      c->woff += (size_t)r;
      if (c->shared) c->shared->queued -= (size_t)r;
      continue;
    }
    if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    close_conn(c, std::string("send failed: ") + std::strerror(errno));
    return false;
  }
  if (c->woff == c->wbuf.size()) {
    c->wbuf.clear();
    c->woff = 0;
  } else if (c->woff > (1u << 20)) {
    c->wbuf.erase(0, c->woff);
    c->woff = 0;
  }
  const bool drained = c->shared->queued.load() < hwm_ / 2;
  if (drained && c->shared->above.exchange(false)) {
    Event e;
    e.kind = Event::DRAIN;
    e.conn = c->id;
    push_event(std::move(e));
  }
  if (c->ending && c->wbuf.empty() && c->pending.empty()) {
    close_conn(c, "");
    return false;
  }
  update_interest(c);
  return true;
}

void Transport::on_io(Conn* c, uint32_t events) {
  if (c->phase == Conn::CLOSED) return;
  if (c->phase == Conn::CONNECTING && (events & (EPOLLOUT | EPOLLERR | EPOLLHUP))) {
    int err = 0;
    socklen_t el = sizeof err;
    getsockopt(c->fd, SOL_SOCKET, SO_ERROR, &err, &el);
    if (err) {
      close_conn(c, std::string("connect failed: ") + std::strerror(err));
      return;
    }
    try {
      start_handshake(c);
    } catch (const std::exception& ex) {
      close_conn(c, ex.what());
      return;
    }
  }
  if (events & EPOLLIN) {
    char buf[65536];
    while (true) {
      const ssize_t r = ::recv(c->fd, buf, sizeof buf, 0);
      if (r > 0) {
        c->rbuf.append(buf, (size_t)r);
        c->last_rx = now_ms();
        continue;
      }
      if (r == 0) {
        process_frames(c);
        if (c->phase != Conn::CLOSED) close_conn(c, "");
        return;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      close_conn(c, std::string("recv failed: ") + std::strerror(errno));
      return;
    }
    process_frames(c);
    if (c->phase == Conn::CLOSED) return;
  } else if (events & (EPOLLERR | EPOLLHUP)) {
    close_conn(c, "connection reset by peer");
    return;
  }
  flush(c);
}

void Transport::process_frames(Conn* c) {
  while (c->phase != Conn::CLOSED) {
    const size_t avail = c->rbuf.size() - c->roff;
    if (avail < 3) break;
    const uint8_t* p = (const uint8_t*)c->rbuf.data() + c->roff;
    const size_t n = p[0] | (p[1] << 8) | ((size_t)p[2] << 16);
    if (n > kMaxFrame) {  // a peer announcing an oversized frame is broken or hostile: do not buffer it
      close_conn(c, "protocol error: frame too large");
      return;
    }
    if (avail < 3 + n) break;
    c->roff += 3 + n;
    try {
      handle_frame(c, p + 3, n);
    } catch (const std::exception& ex) {
      close_conn(c, std::string("protocol error: ") + ex.what());
      return;
    }
  }
  if (c->roff == c->rbuf.size()) {
    c->rbuf.clear();
    c->roff = 0;
  } else if (c->roff > (1u << 20)) {
    c->rbuf.erase(0, c->roff);
    c->roff = 0;
  }
}

void Transport::after_handshake(Conn* c) {
  std::memcpy(c->hh, c->hs->handshake_hash(), 64);
  uint8_t txk[32], rxk[32];
  c->hs->split(txk, rxk);
  uint8_t frame[56];
  stream_id(c->hh, c->initiator, frame);
  c->tx.init_push(txk, frame + 32);
  std::memcpy(c->rx_key, rxk, 32);  // used when the peer's header frame arrives
  wipe(txk, 32);
  wipe(rxk, 32);
  send_frame(c, frame, sizeof frame);
  c->phase = Conn::HEADER;
}

void Transport::handle_frame(Conn* c, const uint8_t* p, size_t n) {
  switch (c->phase) {
    case Conn::HANDSHAKE: {
      c->hs->read_message(p, n);
      if (!c->hs->complete()) {
        Bytes m = c->hs->write_message(nullptr, 0);
        send_frame(c, m.data(), m.size());
      }
      if (c->hs->complete()) after_handshake(c);
      break;
    }
    case Conn::HEADER: {
      if (n != 56) throw CryptoError("bad stream header");
      uint8_t expect[32];
      stream_id(c->hh, !c->initiator, expect);
      if (!ct_equal(expect, p, 32)) throw CryptoError("stream id mismatch");
      c->rx.init_pull(c->rx_key, p + 32);
      wipe(c->rx_key, 32);
      c->phase = Conn::OPEN;
      Event e;
      e.kind = Event::OPEN;
      e.conn = c->id;
      e.remote_pk.assign((const char*)c->hs->remote_static(), 32);
      e.handshake_hash.assign((const char*)c->hh, 64);
      e.host = c->host;
      e.port = c->port;
      e.initiator = c->initiator;
      push_event(std::move(e));
      c->hs.reset();
      while (!c->pending.empty()) {
        std::string m = std::move(c->pending.front());
        c->pending.pop_front();
        Bytes f = c->tx.push((const uint8_t*)m.data(), m.size());
        c->shared->queued -= f.size() + 3;
        send_frame(c, f.data(), f.size());
        c->shared->bytes_out += m.size();
      }
      break;
    }
    case Conn::OPEN: {
      Bytes m;
      uint8_t tag;
      if (!c->rx.pull(p, n, m, tag)) throw CryptoError("message authentication failed");
      if (m.empty()) break;  // keep-alive
      c->shared->bytes_in += m.size();
      Event e;
      e.kind = Event::DATA;
      e.conn = c->id;
      e.data.assign((const char*)m.data(), m.size());
      push_event(std::move(e));
      break;
    }
    default:
      break;
  }
}

void Transport::close_conn(Conn* c, const std::string& err) {
  if (c->phase == Conn::CLOSED) return;
  const bool was_open = c->phase == Conn::OPEN;
  c->phase = Conn::CLOSED;
  if (c->fd >= 0) {
    epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
    c->fd = -1;
  }
  if (c->shared) c->shared->open.store(false);
  {
    std::lock_guard<std::mutex> g(shared_mu_);
    shared_.erase(c->id);
  }
  // connections that never opened are reported only if locally initiated (connect errors)
  if (was_open || c->initiator) {
    Event e;
    e.kind = Event::CLOSE;
    e.conn = c->id;
    e.data = err;
    e.initiator = c->initiator;
    e.host = c->host;
    e.port = c->port;
    push_event(std::move(e));
  }
}

}  // namespace symnet
