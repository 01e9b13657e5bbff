// Host-side self-test of the P2P plane, built with AddressSanitizer + UndefinedBehaviorSanitizer
// (SURVEY.md §5.2): `python -m symmetry_amd._build selftest` -> build/net_selftest_asan, run by
// tests/test_native_sanitizers.py.  Exercises every code path that parses attacker-controlled bytes
// (Noise messages, secretstream frames, transport framing) plus known-answer vectors, so a heap
// overflow / use-after-free / UB in the C++ transport fails the CPU test suite.
#include <poll.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "crypto.h"
#include "noise.h"
#include "transport.h"

using namespace symnet;

static int g_fail = 0;
#define CHECK(cond)                                                   \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

static Bytes unhex(const char* s) {
  Bytes b;
  for (size_t i = 0; s[i] && s[i + 1]; i += 2) {
    unsigned v;
    std::sscanf(s + i, "%2x", &v);
    b.push_back((uint8_t)v);
  }
  return b;
}

static void known_answers() {
  // BLAKE2b-512("abc"), RFC 7693 appendix A
  uint8_t out[64];
  blake2b(out, 64, (const uint8_t*)"abc", 3);
  Bytes want = unhex(
      "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d17d87c5392aab792dc252d5de4533cc9518d38aa8db"
      "f1925ab92386edd4009923");
  CHECK(std::memcmp(out, want.data(), 64) == 0);
  // Poly1305, RFC 8439 §2.5.2
  Bytes key = unhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b");
  const char* msg = "Cryptographic Forum Research Group";
  Poly1305 p(key.data());
  p.update((const uint8_t*)msg, std::strlen(msg));
  uint8_t mac[16];
  p.finish(mac);
  Bytes tag = unhex("a8061dc1305136c6c22b8baf0c0127a9");
  CHECK(std::memcmp(mac, tag.data(), 16) == 0);
}

static void aead_fuzz(std::mt19937& rng) {
  for (int it = 0; it < 200; ++it) {
    uint8_t key[32], nonce[24];
    for (auto& b : key) b = rng();
    for (auto& b : nonce) b = rng();
    Bytes pt(rng() % 3000), ad(rng() % 64);
    for (auto& b : pt) b = rng();
    for (auto& b : ad) b = rng();
    Bytes ct = aead_xchacha20poly1305_encrypt(key, nonce, ad.data(), ad.size(), pt.data(), pt.size());
    Bytes back;
    CHECK(aead_xchacha20poly1305_decrypt(key, nonce, ad.data(), ad.size(), ct.data(), ct.size(), back));
    CHECK(back == pt);
    ct[rng() % ct.size()] ^= (uint8_t)(1 + rng() % 255);
    CHECK(!aead_xchacha20poly1305_decrypt(key, nonce, ad.data(), ad.size(), ct.data(), ct.size(), back));
    // truncated ciphertexts of every short length must be rejected, never over-read
    for (size_t n = 0; n < 17 && n < ct.size(); ++n)
      CHECK(!aead_xchacha20poly1305_decrypt(key, nonce, nullptr, 0, ct.data(), n, back));
  }
}

static void noise_and_stream(std::mt19937& rng) {
  for (int it = 0; it < 30; ++it) {
    KeyPair a = keypair_random(), b = keypair_random();
    NoiseXX i(true, a), r(false, b);
    Bytes m1 = i.write_message(nullptr, 0);
    r.read_message(m1.data(), m1.size());
    Bytes m2 = r.write_message((const uint8_t*)"hi", 2);
    Bytes p2 = i.read_message(m2.data(), m2.size());
    CHECK(p2.size() == 2);
    Bytes m3 = i.write_message(nullptr, 0);
    r.read_message(m3.data(), m3.size());
    CHECK(i.complete() && r.complete());
    CHECK(std::memcmp(i.handshake_hash(), r.handshake_hash(), 64) == 0);
    CHECK(std::memcmp(i.remote_static(), b.pk, 32) == 0);
    uint8_t itx[32], irx[32], rtx[32], rrx[32];
    i.split(itx, irx);
    r.split(rtx, rrx);
    CHECK(std::memcmp(itx, rrx, 32) == 0);
    // a corrupted handshake message must throw, not crash
    NoiseXX i2(true, a), r2(false, b);
    Bytes x1 = i2.write_message(nullptr, 0);
    r2.read_message(x1.data(), x1.size());
    Bytes x2 = r2.write_message(nullptr, 0);
    x2[rng() % x2.size()] ^= 0x80;
    bool threw = false;
    try {
      i2.read_message(x2.data(), x2.size());
    } catch (const CryptoError&) {
      threw = true;
    }
    CHECK(threw);
    // secretstream: random sizes, tags, rekeys, tampering and truncation
    SecretStream tx, rx;
    uint8_t hdr[24];
    tx.init_push(itx, hdr);
    rx.init_pull(itx, hdr);
    for (int k = 0; k < 100; ++k) {
      Bytes m(rng() % 2000);
      for (auto& c : m) c = rng();
      const uint8_t tag = (rng() % 10 == 0) ? SecretStream::TAG_REKEY : SecretStream::TAG_MESSAGE;
      Bytes c = tx.push(m.data(), m.size(), tag);
      Bytes out;
      uint8_t t = 0;
      if (rng() % 7 == 0) {  // tampered copy is rejected and does not advance the state
        Bytes bad = c;
        bad[rng() % bad.size()] ^= 1;
        CHECK(!rx.pull(bad.data(), bad.size(), out, t));
        CHECK(!rx.pull(c.data(), rng() % SecretStream::ABYTES, out, t));
      }
      CHECK(rx.pull(c.data(), c.size(), out, t));
      CHECK(out == m && t == tag);
    }
  }
}

static std::vector<Event> wait_events(Transport& t, int ms) {
  pollfd pfd{t.fileno(), POLLIN, 0};
  ::poll(&pfd, 1, ms);
  return t.poll();
}

static void transport_loopback(std::mt19937& rng) {
  Transport server(keypair_random(), 1000, 10000, 1 << 20);
  Transport client(keypair_random(), 1000, 10000, 1 << 20);
  const int port = server.listen("127.0.0.1", 0);
  const uint64_t cid = client.connect("127.0.0.1", port);
  std::vector<std::string> sent;
  for (int k = 0; k < 300; ++k) {
    std::string m(rng() % 5000, '\0');
    for (auto& c : m) c = (char)rng();
    sent.push_back(m);
    client.write(cid, m);  // queued until the stream opens
  }
  size_t got = 0;
  uint64_t sid = 0;
  bool server_open = false;
  auto t0 = std::chrono::steady_clock::now();
  while (got < sent.size() && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(20)) {
    for (auto& e : wait_events(server, 50)) {
      if (e.kind == Event::OPEN) {
        server_open = true;
        sid = e.conn;
      } else if (e.kind == Event::DATA) {
        CHECK(e.data == sent[got]);
        ++got;
      }
    }
    client.poll();
  }
  CHECK(server_open);
  CHECK(got == sent.size());
  // unframed garbage and an oversized length header close only that connection
  const uint64_t bad = client.connect("127.0.0.1", port);
  client.write(bad, "x");
  bool closed_bad = false;
  bool opened_bad = false;
  t0 = std::chrono::steady_clock::now();
  while (!closed_bad && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(20)) {
    for (auto& e : wait_events(client, 50)) {
      if (e.kind == Event::OPEN && e.conn == bad && !opened_bad) {
        opened_bad = true;
        client.inject_fault(bad, 0, std::string("\xff\xff\xff garbage", 11));
      }
      if (e.kind == Event::CLOSE && e.conn == bad) closed_bad = true;
    }
    server.poll();
  }
  CHECK(closed_bad);
  client.write(cid, "still alive");
  bool alive = false;
  t0 = std::chrono::steady_clock::now();
  while (!alive && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10)) {
    for (auto& e : wait_events(server, 50))
      if (e.kind == Event::DATA && e.conn == sid && e.data == "still alive") alive = true;
    client.poll();
  }
  CHECK(alive);
  client.end(cid);
  client.close();
  server.close();
}

int main() {
  std::mt19937 rng(12345);
  known_answers();
  aead_fuzz(rng);
  noise_and_stream(rng);
  transport_loopback(rng);
  if (g_fail) {
    std::fprintf(stderr, "net selftest: %d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("net selftest: OK\n");
  return 0;
}
