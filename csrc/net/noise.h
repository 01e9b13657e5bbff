// Noise_XX_25519_ChaChaPoly_BLAKE2b with ed25519 static identities, and the
// secretstream (XChaCha20-Poly1305 stream with rekeying) that carries data
// after the handshake.
//
// REF equivalent: @hyperswarm/secret-stream 6.6.1 -> noise-handshake 3.1.0 +
// noise-curve-ed 2.0.1 (XX pattern, DH on ed25519 keys converted to x25519)
// and sodium-secretstream 1.1.0 (libsodium crypto_secretstream_xchacha20poly1305)
// (package-lock.json:763, :4939, :4929, :5734).
// Behaviour-compatible (same identities, authentication and AEAD
// construction), not wire-compatible with the JS stack.
#pragma once
#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "crypto.h"

namespace symnet {

struct KeyPair {
  uint8_t pk[32];  // ed25519 public key (the peer identity)
  uint8_t sk[64];  // libsodium layout: seed || pk
};

KeyPair keypair_from_seed(const uint8_t seed[32]);
KeyPair keypair_random();

class CipherState {
 public:
  bool has_key = false;
  uint8_t k[32];
  uint64_t n = 0;
  void init(const uint8_t key[32]);
  Bytes encrypt(const uint8_t* ad, size_t adlen, const uint8_t* pt, size_t n);
  bool decrypt(const uint8_t* ad, size_t adlen, const uint8_t* ct, size_t n, Bytes& out);
};

class NoiseXX {
 public:
  NoiseXX(bool initiator, const KeyPair& s, const Bytes& prologue = {});
  // Message i (0-based) is written by the initiator for i even, by the responder for i odd.
  Bytes write_message(const uint8_t* payload, size_t len);
  Bytes read_message(const uint8_t* msg, size_t len);  // returns payload; throws CryptoError on failure
  bool complete() const { return step_ == 3; }
  bool my_turn() const { return (step_ % 2 == 0) == initiator_; }
  // After completion: transport keys and the handshake hash (channel binding).
  void split(uint8_t tx[32], uint8_t rx[32]) const;
  const uint8_t* handshake_hash() const { return h_; }
  const uint8_t* remote_static() const { return rs_; }
  bool initiator() const { return initiator_; }

 private:
  void mix_hash(const uint8_t* d, size_t n);
  void mix_key(const uint8_t* ikm, size_t n);
  Bytes encrypt_and_hash(const uint8_t* pt, size_t n);
  Bytes decrypt_and_hash(const uint8_t* ct, size_t n);
  void dh(const KeyPair& local, const uint8_t remote[32], uint8_t out[32]) const;

  bool initiator_;
  int step_ = 0;
  KeyPair s_, e_;
  uint8_t rs_[32] = {0}, re_[32] = {0};
  uint8_t h_[64], ck_[64];
  CipherState cs_;
};

void hmac_blake2b(const uint8_t* key, size_t keylen, const uint8_t* data, size_t n, uint8_t out[64]);
void hkdf2(const uint8_t ck[64], const uint8_t* ikm, size_t n, uint8_t out1[64], uint8_t out2[64]);

// libsodium crypto_secretstream_xchacha20poly1305 construction.
class SecretStream {
 public:
  static constexpr size_t HEADERBYTES = 24;
  static constexpr size_t ABYTES = 17;
  static constexpr uint8_t TAG_MESSAGE = 0, TAG_PUSH = 1, TAG_REKEY = 2, TAG_FINAL = 3;

  // push side: generates a random header
  void init_push(const uint8_t key[32], uint8_t header[24]);
  void init_pull(const uint8_t key[32], const uint8_t header[24]);
  Bytes push(const uint8_t* m, size_t mlen, uint8_t tag = TAG_MESSAGE, const uint8_t* ad = nullptr, size_t adlen = 0);
  bool pull(const uint8_t* c, size_t clen, Bytes& m, uint8_t& tag, const uint8_t* ad = nullptr, size_t adlen = 0);
  void rekey();

 private:
  uint8_t k_[32];
  uint8_t nonce_[12];  // counter (4, LE) || inonce (8)
  void counter_reset();
  void after_message(const uint8_t mac[16], uint8_t tag);
};

}  // namespace symnet
