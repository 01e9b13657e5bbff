// Encrypted, message-framed peer transport driven by one epoll thread.
//
// REF equivalent: udx-native 1.10.3 (reliable UDP streams over libuv) plus the
// framing/encryption of @hyperswarm/secret-stream (package-lock.json:6241,
// :763).  There is no NAT to punch on the MI355X boxes,
// so streams run over TCP; everything above the socket -- Noise XX
// authentication with ed25519 identities, per-message secretstream AEAD,
// uint24 length framing (one write == one message, as the provider's JSON
// protocol assumes: src/provider.ts:113-115), keep-alives, idle timeouts and
// write back-pressure with a 'drain' signal (src/provider.ts:250-252) -- is
// done here, off the Python thread.
//
// Frames: [u24 LE length][payload]
//   handshake: the three Noise XX messages
//   header:    32-byte stream id (BLAKE2b(handshake hash, role)) || 24-byte secretstream header
//   data:      secretstream push(message); an empty message is a keep-alive
#pragma once
#include <atomic>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "noise.h"

namespace symnet {

struct Event {
  enum Kind { OPEN = 0, DATA = 1, DRAIN = 2, CLOSE = 3, LISTEN_ERROR = 4 };
  Kind kind;
  uint64_t conn = 0;
  std::string data;  // DATA: plaintext message; CLOSE: error text ("" = clean close)
  std::string remote_pk;
  std::string handshake_hash;
  std::string host;
  int port = 0;
  bool initiator = false;
};

struct ConnShared {
  std::atomic<size_t> queued{0};
  std::atomic<bool> open{true};
  std::atomic<bool> above{false};
  std::atomic<uint64_t> bytes_out{0}, bytes_in{0};
};

class Transport {
 public:
  Transport(const KeyPair& kp, int keepalive_ms, int timeout_ms, size_t high_watermark);
  ~Transport();
  Transport(const Transport&) = delete;

  int listen(const std::string& host, int port);  // returns the bound port
  uint64_t connect(const std::string& host, int port);
  bool write(uint64_t id, std::string data);  // false: above the high watermark (message still queued)
  void end(uint64_t id);                     // flush queued messages, then close
  void destroy(uint64_t id);                 // close now
  // Fault injection (tests): mode 0 appends `data` raw to the socket stream (bypassing
  // framing and encryption); mode 1 frames + encrypts `data`, then flips one ciphertext bit.
  void inject_fault(uint64_t id, int mode, std::string data);
  int fileno() const { return event_fd_; }
  std::vector<Event> poll();
  void close();
  size_t queued(uint64_t id);
  std::string public_key() const { return std::string((const char*)kp_.pk, 32); }

 private:
  struct Conn;
  struct Cmd {
    enum Kind { CONNECT, WRITE, END, DESTROY, FAULT } kind;
    uint64_t id;
    std::string data;
    std::string host;
    int port;
  };
  void loop();
  void wake();
  void push_event(Event&& e);
  void handle_cmds();
  void on_accept(int lfd);
  void on_io(Conn* c, uint32_t events);
  bool flush(Conn* c);
  void send_frame(Conn* c, const uint8_t* p, size_t n);
  void process_frames(Conn* c);
  void handle_frame(Conn* c, const uint8_t* p, size_t n);
  void start_handshake(Conn* c);
  void after_handshake(Conn* c);
  void close_conn(Conn* c, const std::string& err);
  void update_interest(Conn* c);
  void ticks();

  KeyPair kp_;
  int keepalive_ms_, timeout_ms_;
  size_t hwm_;
  int epfd_ = -1, event_fd_ = -1, cmd_fd_ = -1;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> next_id_{1};
  std::thread thread_;
  std::mutex cmd_mu_, ev_mu_, shared_mu_, lst_mu_;
  std::deque<Cmd> cmds_;
  std::deque<Event> events_;
  std::unordered_map<uint64_t, std::shared_ptr<ConnShared>> shared_;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns_;  // loop thread only
  std::vector<int> listeners_;
};

}  // namespace symnet
