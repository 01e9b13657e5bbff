// Crypto primitives of the P2P plane, over OpenSSL 3 libcrypto plus small
// self-contained pieces OpenSSL does not expose in the needed form.
//
// REF equivalent: sodium-native 4.1.1 (libsodium via N-API), used through
// hypercore-crypto / noise-handshake / sodium-secretstream
// (package-lock.json:5725, :3397, :4939, :5734).
//
//   ed25519      keypair-from-seed, detached sign / verify   (crypto_sign_*)
//   x25519       scalar multiplication                        (crypto_scalarmult)
//   ed->x25519   key conversion for Noise DH with ed25519 identities (noise-curve-ed)
//   BLAKE2b      RFC 7693, keyed, 1..64-byte output           (crypto_generichash)
//   ChaCha20     RFC 8439 block function with 32-bit counter  (crypto_stream_chacha20_ietf)
//   HChaCha20    XChaCha subkey derivation                     (crypto_core_hchacha20)
//   Poly1305     RFC 8439 one-time MAC                         (crypto_onetimeauth)
//   ChaCha20-Poly1305 IETF AEAD, XChaCha20-Poly1305 AEAD
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace symnet {

using Bytes = std::vector<uint8_t>;

struct CryptoError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void random_bytes(uint8_t* out, size_t n);
Bytes random_bytes(size_t n);

// ---- ed25519 ------------------------------------------------------------------------------------
// secret key in libsodium layout: seed (32) || public key (32)
void ed25519_keypair_from_seed(const uint8_t seed[32], uint8_t pk[32], uint8_t sk[64]);
void ed25519_sign(const uint8_t* msg, size_t len, const uint8_t sk[64], uint8_t sig[64]);
bool ed25519_verify(const uint8_t* msg, size_t len, const uint8_t sig[64], const uint8_t pk[32]);

// ---- x25519 --------------------------------------------------------------------------------------
void x25519_public(const uint8_t sk[32], uint8_t pk[32]);
bool x25519(const uint8_t sk[32], const uint8_t pk[32], uint8_t out[32]);  // false on all-zero output
bool ed25519_pk_to_x25519(const uint8_t ed_pk[32], uint8_t x_pk[32]);
void ed25519_sk_to_x25519(const uint8_t ed_sk[64], uint8_t x_sk[32]);

// ---- BLAKE2b (RFC 7693) -------------------------------------------------------------------------
struct Blake2b {
  uint64_t h[8], t[2];
  uint8_t buf[128];
  size_t c, outlen;
  Blake2b(size_t outlen = 64, const uint8_t* key = nullptr, size_t keylen = 0);
  void update(const uint8_t* in, size_t n);
  void final(uint8_t* out);
};
void blake2b(uint8_t* out, size_t outlen, const uint8_t* in, size_t inlen, const uint8_t* key = nullptr,
             size_t keylen = 0);

// ---- ChaCha20 / HChaCha20 / Poly1305 ---------------------------------------------------------
void chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]);
void chacha20_xor(uint8_t* out, const uint8_t* in, size_t n, const uint8_t key[32], const uint8_t nonce[12],
                  uint32_t counter);
void hchacha20(uint8_t out[32], const uint8_t in[16], const uint8_t key[32]);

struct Poly1305 {
  uint32_t r[5], h[5], pad[4];
  uint8_t buf[16];
  size_t leftover;
  bool final_block;
  explicit Poly1305(const uint8_t key[32]);
  void update(const uint8_t* m, size_t n);
  void finish(uint8_t mac[16]);

 private:
  void blocks(const uint8_t* m, size_t n);
};

// ---- AEADs --------------------------------------------------------------------------------------
// ChaCha20-Poly1305 (RFC 8439); out = ciphertext || tag(16)
Bytes aead_chacha20poly1305_encrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* ad, size_t adlen,
                                    const uint8_t* pt, size_t ptlen);
bool aead_chacha20poly1305_decrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* ad, size_t adlen,
                                   const uint8_t* ct, size_t ctlen, Bytes& pt);
Bytes aead_xchacha20poly1305_encrypt(const uint8_t key[32], const uint8_t nonce[24], const uint8_t* ad, size_t adlen,
                                     const uint8_t* pt, size_t ptlen);
bool aead_xchacha20poly1305_decrypt(const uint8_t key[32], const uint8_t nonce[24], const uint8_t* ad, size_t adlen,
                                    const uint8_t* ct, size_t ctlen, Bytes& pt);

bool ct_equal(const uint8_t* a, const uint8_t* b, size_t n);
void wipe(void* p, size_t n);

// ---- hypercore-crypto semantics -----------------------------------------------------------------
// discoveryKey(pk) = BLAKE2b-256(message = "hypercore", key = pk)
void discovery_key(const uint8_t* key, size_t keylen, uint8_t out[32]);

}  // namespace symnet
