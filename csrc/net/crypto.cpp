// Crypto primitives (see crypto.h).  ed25519 / x25519 / SHA-512 / CSPRNG come
// from OpenSSL 3 libcrypto; BLAKE2b (RFC 7693), ChaCha20 / HChaCha20
// (RFC 8439, draft-irtf-cfrg-xchacha) and Poly1305 (RFC 8439, 26-bit-limb
// form) are implemented here because the Noise / secretstream constructions
// need their raw block-level forms (counter-addressed keystream, streaming
// one-time MAC) rather than OpenSSL's AEAD wrapper.
#include "crypto.h"

#include <openssl/bn.h>
#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <openssl/rand.h>
#include <openssl/sha.h>

#include <cstring>
#include <memory>

namespace symnet {

namespace {

inline uint32_t ld32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline void st32(uint8_t* p, uint32_t v) {
  p[0] = v;
  p[1] = v >> 8;
  p[2] = v >> 16;
  p[3] = v >> 24;
}
inline uint64_t ld64(const uint8_t* p) { return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32); }
inline void st64(uint8_t* p, uint64_t v) {
  st32(p, (uint32_t)v);
  st32(p + 4, (uint32_t)(v >> 32));
}
inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

struct PkeyDel {
  void operator()(EVP_PKEY* p) const { EVP_PKEY_free(p); }
};
struct MdCtxDel {
  void operator()(EVP_MD_CTX* p) const { EVP_MD_CTX_free(p); }
};
struct PkCtxDel {
  void operator()(EVP_PKEY_CTX* p) const { EVP_PKEY_CTX_free(p); }
};
using PkeyPtr = std::unique_ptr<EVP_PKEY, PkeyDel>;

}  // namespace

void random_bytes(uint8_t* out, size_t n) {
  if (n && RAND_bytes(out, (int)n) != 1) throw CryptoError("RAND_bytes failed");
}

Bytes random_bytes(size_t n) {
  Bytes b(n);
  random_bytes(b.data(), n);
  return b;
}

bool ct_equal(const uint8_t* a, const uint8_t* b, size_t n) { return CRYPTO_memcmp(a, b, n) == 0; }
void wipe(void* p, size_t n) { OPENSSL_cleanse(p, n); }

// ---- ed25519 ------------------------------------------------------------------------------------
void ed25519_keypair_from_seed(const uint8_t seed[32], uint8_t pk[32], uint8_t sk[64]) {
  PkeyPtr key(EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, seed, 32));
  if (!key) throw CryptoError("ed25519 key from seed failed");
  size_t len = 32;
  if (EVP_PKEY_get_raw_public_key(key.get(), pk, &len) != 1 || len != 32) throw CryptoError("ed25519 pk failed");
  std::memcpy(sk, seed, 32);
  std::memcpy(sk + 32, pk, 32);
}

void ed25519_sign(const uint8_t* msg, size_t len, const uint8_t sk[64], uint8_t sig[64]) {
  PkeyPtr key(EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, sk, 32));
  std::unique_ptr<EVP_MD_CTX, MdCtxDel> ctx(EVP_MD_CTX_new());
  size_t siglen = 64;
  if (!key || !ctx || EVP_DigestSignInit(ctx.get(), nullptr, nullptr, nullptr, key.get()) != 1 ||
      EVP_DigestSign(ctx.get(), sig, &siglen, msg, len) != 1 || siglen != 64)
    throw CryptoError("ed25519 sign failed");
}

bool ed25519_verify(const uint8_t* msg, size_t len, const uint8_t sig[64], const uint8_t pk[32]) {
  PkeyPtr key(EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, nullptr, pk, 32));
  if (!key) return false;
  std::unique_ptr<EVP_MD_CTX, MdCtxDel> ctx(EVP_MD_CTX_new());
  if (!ctx || EVP_DigestVerifyInit(ctx.get(), nullptr, nullptr, nullptr, key.get()) != 1) return false;
  return EVP_DigestVerify(ctx.get(), sig, 64, msg, len) == 1;
}

// ---- x25519 --------------------------------------------------------------------------------------
void x25519_public(const uint8_t sk[32], uint8_t pk[32]) {
  PkeyPtr key(EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, nullptr, sk, 32));
  size_t len = 32;
  if (!key || EVP_PKEY_get_raw_public_key(key.get(), pk, &len) != 1) throw CryptoError("x25519 pk failed");
}

bool x25519(const uint8_t sk[32], const uint8_t pk[32], uint8_t out[32]) {
  PkeyPtr key(EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, nullptr, sk, 32));
  PkeyPtr peer(EVP_PKEY_new_raw_public_key(EVP_PKEY_X25519, nullptr, pk, 32));
  if (!key || !peer) return false;
  std::unique_ptr<EVP_PKEY_CTX, PkCtxDel> ctx(EVP_PKEY_CTX_new(key.get(), nullptr));
  size_t len = 32;
  if (!ctx || EVP_PKEY_derive_init(ctx.get()) != 1 || EVP_PKEY_derive_set_peer(ctx.get(), peer.get()) != 1 ||
      EVP_PKEY_derive(ctx.get(), out, &len) != 1 || len != 32)
    return false;
  uint8_t acc = 0;
  for (int i = 0; i < 32; ++i) acc |= out[i];
  return acc != 0;
}

// Edwards y -> Montgomery u = (1 + y) / (1 - y) mod p, p = 2^255 - 19.
bool ed25519_pk_to_x25519(const uint8_t ed_pk[32], uint8_t x_pk[32]) {
  uint8_t be[32];
  for (int i = 0; i < 32; ++i) be[i] = ed_pk[31 - i];
  be[0] &= 0x7f;  // drop the sign bit of x
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *p = BN_new(), *y = BN_bin2bn(be, 32, nullptr), *one = BN_new(), *num = BN_new(), *den = BN_new(),
         *u = BN_new();
  bool ok = ctx && p && y && one && num && den && u;
  if (ok) {
    BN_one(one);
    BN_set_bit(p, 255);
    BN_sub_word(p, 19);
    ok = BN_cmp(y, p) < 0 && BN_mod_add(num, one, y, p, ctx) && BN_mod_sub(den, one, y, p, ctx) && !BN_is_zero(den) &&
         BN_mod_inverse(den, den, p, ctx) != nullptr && BN_mod_mul(u, num, den, p, ctx);
    if (ok) {
      uint8_t ube[32];
      ok = BN_bn2binpad(u, ube, 32) == 32;
      for (int i = 0; i < 32; ++i) x_pk[i] = ube[31 - i];
    }
  }
  BN_free(p);
  BN_free(y);
  BN_free(one);
  BN_free(num);
  BN_free(den);
  BN_free(u);
  BN_CTX_free(ctx);
  return ok;
}

void ed25519_sk_to_x25519(const uint8_t ed_sk[64], uint8_t x_sk[32]) {
  uint8_t h[64];
  SHA512(ed_sk, 32, h);
  h[0] &= 248;
  h[31] &= 127;
  h[31] |= 64;
  std::memcpy(x_sk, h, 32);
  wipe(h, sizeof h);
}

// ---- BLAKE2b ------------------------------------------------------------------------------------
namespace {
const uint64_t B2_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                           0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                           0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
const uint8_t B2_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

void b2_compress(Blake2b& s, bool last) {
  uint64_t v[16], m[16];
  for (int i = 0; i < 8; ++i) {
    v[i] = s.h[i];
    v[i + 8] = B2_IV[i];
  }
  v[12] ^= s.t[0];
  v[13] ^= s.t[1];
  if (last) v[14] = ~v[14];
  for (int i = 0; i < 16; ++i) m[i] = ld64(s.buf + 8 * i);
#define B2G(a, b, c, d, x, y)    \
  v[a] = v[a] + v[b] + (x);      \
  v[d] = rotr64(v[d] ^ v[a], 32); \
  v[c] = v[c] + v[d];            \
  v[b] = rotr64(v[b] ^ v[c], 24); \
  v[a] = v[a] + v[b] + (y);      \
  v[d] = rotr64(v[d] ^ v[a], 16); \
  v[c] = v[c] + v[d];            \
  v[b] = rotr64(v[b] ^ v[c], 63);
  for (int r = 0; r < 12; ++r) {
    const uint8_t* sg = B2_SIGMA[r];
    B2G(0, 4, 8, 12, m[sg[0]], m[sg[1]]);
    B2G(1, 5, 9, 13, m[sg[2]], m[sg[3]]);
    B2G(2, 6, 10, 14, m[sg[4]], m[sg[5]]);
    B2G(3, 7, 11, 15, m[sg[6]], m[sg[7]]);
    B2G(0, 5, 10, 15, m[sg[8]], m[sg[9]]);
    B2G(1, 6, 11, 12, m[sg[10]], m[sg[11]]);
    B2G(2, 7, 8, 13, m[sg[12]], m[sg[13]]);
    B2G(3, 4, 9, 14, m[sg[14]], m[sg[15]]);
  }
#undef B2G
  for (int i = 0; i < 8; ++i) s.h[i] ^= v[i] ^ v[i + 8];
}
}  // namespace

Blake2b::Blake2b(size_t outlen_, const uint8_t* key, size_t keylen) : c(0), outlen(outlen_) {
  if (outlen == 0 || outlen > 64 || keylen > 64) throw CryptoError("blake2b: bad outlen/keylen");
  for (int i = 0; i < 8; ++i) h[i] = B2_IV[i];
  h[0] ^= 0x01010000ULL ^ ((uint64_t)keylen << 8) ^ outlen;
  t[0] = t[1] = 0;
  std::memset(buf, 0, sizeof buf);
  if (keylen) {
    update(key, keylen);
    c = 128;
  }
}

void Blake2b::update(const uint8_t* in, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    if (c == 128) {
      t[0] += c;
      if (t[0] < c) t[1]++;
      b2_compress(*this, false);
      c = 0;
    }
    buf[c++] = in[i];
  }
}

void Blake2b::final(uint8_t* out) {
  t[0] += c;
  if (t[0] < c) t[1]++;
  while (c < 128) buf[c++] = 0;
  b2_compress(*this, true);
  uint8_t full[64];
  for (int i = 0; i < 8; ++i) st64(full + 8 * i, h[i]);
  std::memcpy(out, full, outlen);
}

void blake2b(uint8_t* out, size_t outlen, const uint8_t* in, size_t inlen, const uint8_t* key, size_t keylen) {
  Blake2b s(outlen, key, keylen);
  s.update(in, inlen);
  s.final(out);
}

void discovery_key(const uint8_t* key, size_t keylen, uint8_t out[32]) {
  static const uint8_t kHypercore[] = {'h', 'y', 'p', 'e', 'r', 'c', 'o', 'r', 'e'};
  blake2b(out, 32, kHypercore, sizeof kHypercore, key, keylen);
}

// ---- ChaCha20 -------------------------------------------------------------------------------------
namespace {
inline void qr(uint32_t* x, int a, int b, int c, int d) {
  x[a] += x[b];
  x[d] = rotl32(x[d] ^ x[a], 16);
  x[c] += x[d];
  x[b] = rotl32(x[b] ^ x[c], 12);
  x[a] += x[b];
  x[d] = rotl32(x[d] ^ x[a], 8);
  x[c] += x[d];
  x[b] = rotl32(x[b] ^ x[c], 7);
}

void chacha_rounds(uint32_t* x) {
  for (int i = 0; i < 10; ++i) {
    qr(x, 0, 4, 8, 12);
    qr(x, 1, 5, 9, 13);
    qr(x, 2, 6, 10, 14);
    qr(x, 3, 7, 11, 15);
    qr(x, 0, 5, 10, 15);
    qr(x, 1, 6, 11, 12);
    qr(x, 2, 7, 8, 13);
    qr(x, 3, 4, 9, 14);
  }
}

void chacha_init(uint32_t* s, const uint8_t key[32]) {
  s[0] = 0x61707865;
  s[1] = 0x3320646e;
  s[2] = 0x79622d32;
  s[3] = 0x6b206574;
  for (int i = 0; i < 8; ++i) s[4 + i] = ld32(key + 4 * i);
}
}  // namespace

void chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]) {
  uint32_t s[16], x[16];
  chacha_init(s, key);
  s[12] = counter;
  s[13] = ld32(nonce);
  s[14] = ld32(nonce + 4);
  s[15] = ld32(nonce + 8);
  std::memcpy(x, s, sizeof s);
  chacha_rounds(x);
  for (int i = 0; i < 16; ++i) st32(out + 4 * i, x[i] + s[i]);
}

void chacha20_xor(uint8_t* out, const uint8_t* in, size_t n, const uint8_t key[32], const uint8_t nonce[12],
                  uint32_t counter) {
  uint8_t ks[64];
  for (size_t off = 0; off < n; off += 64, ++counter) {
    chacha20_block(key, counter, nonce, ks);
    const size_t m = n - off < 64 ? n - off : 64;
    for (size_t i = 0; i < m; ++i) out[off + i] = in[off + i] ^ ks[i];
  }
  wipe(ks, sizeof ks);
}

void hchacha20(uint8_t out[32], const uint8_t in[16], const uint8_t key[32]) {
  uint32_t x[16];
  chacha_init(x, key);
  for (int i = 0; i < 4; ++i) x[12 + i] = ld32(in + 4 * i);
  chacha_rounds(x);
  for (int i = 0; i < 4; ++i) {
    st32(out + 4 * i, x[i]);
    st32(out + 16 + 4 * i, x[12 + i]);
  }
}

// ---- Poly1305 (26-bit limbs) ----------------------------------------------------------------------
Poly1305::Poly1305(const uint8_t key[32]) : leftover(0), final_block(false) {
  r[0] = ld32(key + 0) & 0x3ffffff;
  r[1] = (ld32(key + 3) >> 2) & 0x3ffff03;
  r[2] = (ld32(key + 6) >> 4) & 0x3ffc0ff;
  r[3] = (ld32(key + 9) >> 6) & 0x3f03fff;
  r[4] = (ld32(key + 12) >> 8) & 0x00fffff;
  for (int i = 0; i < 5; ++i) h[i] = 0;
  for (int i = 0; i < 4; ++i) pad[i] = ld32(key + 16 + 4 * i);
}

void Poly1305::blocks(const uint8_t* m, size_t n) {
  const uint32_t hibit = final_block ? 0 : (1u << 24);
  const uint32_t r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
  const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
  uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
  while (n >= 16) {
    h0 += ld32(m + 0) & 0x3ffffff;
    h1 += (ld32(m + 3) >> 2) & 0x3ffffff;
    h2 += (ld32(m + 6) >> 4) & 0x3ffffff;
    h3 += (ld32(m + 9) >> 6) & 0x3ffffff;
    h4 += (ld32(m + 12) >> 8) | hibit;
    uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
    uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
    uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
    uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
    uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
    uint32_t c = (uint32_t)(d0 >> 26);
    h0 = (uint32_t)d0 & 0x3ffffff;
    d1 += c;
    c = (uint32_t)(d1 >> 26);
    h1 = (uint32_t)d1 & 0x3ffffff;
    d2 += c;
    c = (uint32_t)(d2 >> 26);
    h2 = (uint32_t)d2 & 0x3ffffff;
    d3 += c;
    c = (uint32_t)(d3 >> 26);
    h3 = (uint32_t)d3 & 0x3ffffff;
    d4 += c;
    c = (uint32_t)(d4 >> 26);
    h4 = (uint32_t)d4 & 0x3ffffff;
    h0 += c * 5;
    c = h0 >> 26;
    h0 &= 0x3ffffff;
    h1 += c;
    m += 16;
    n -= 16;
  }
  h[0] = h0;
  h[1] = h1;
  h[2] = h2;
  h[3] = h3;
  h[4] = h4;
}

void Poly1305::update(const uint8_t* m, size_t n) {
  if (leftover) {
    size_t want = 16 - leftover;
    if (want > n) want = n;
    std::memcpy(buf + leftover, m, want);
    n -= want;
    m += want;
    leftover += want;
    if (leftover < 16) return;
    blocks(buf, 16);
    leftover = 0;
  }
  if (n >= 16) {
    const size_t want = n & ~(size_t)15;
    blocks(m, want);
    m += want;
    n -= want;
  }
  if (n) {
    std::memcpy(buf, m, n);
    leftover = n;
  }
}

void Poly1305::finish(uint8_t mac[16]) {
  if (leftover) {
    buf[leftover++] = 1;
    while (leftover < 16) buf[leftover++] = 0;
    final_block = true;
    blocks(buf, 16);
  }
  uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4], c;
  c = h1 >> 26; h1 &= 0x3ffffff; h2 += c;
  c = h2 >> 26; h2 &= 0x3ffffff; h3 += c;
  c = h3 >> 26; h3 &= 0x3ffffff; h4 += c;
  c = h4 >> 26; h4 &= 0x3ffffff; h0 += c * 5;
  c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
  uint32_t g4 = h4 + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1;
  g0 &= mask; g1 &= mask; g2 &= mask; g3 &= mask; g4 &= mask;
  mask = ~mask;
  h0 = (h0 & mask) | g0;
  h1 = (h1 & mask) | g1;
  h2 = (h2 & mask) | g2;
  h3 = (h3 & mask) | g3;
  h4 = (h4 & mask) | g4;
  h0 = (h0 | (h1 << 26));
  h1 = ((h1 >> 6) | (h2 << 20));
  h2 = ((h2 >> 12) | (h3 << 14));
  h3 = ((h3 >> 18) | (h4 << 8));
  uint64_t f = (uint64_t)h0 + pad[0];
  h0 = (uint32_t)f;
  f = (uint64_t)h1 + pad[1] + (f >> 32);
  h1 = (uint32_t)f;
  f = (uint64_t)h2 + pad[2] + (f >> 32);
  h2 = (uint32_t)f;
  f = (uint64_t)h3 + pad[3] + (f >> 32);
  h3 = (uint32_t)f;
  st32(mac + 0, h0);
  st32(mac + 4, h1);
  st32(mac + 8, h2);
  st32(mac + 12, h3);
  wipe(r, sizeof r);
  wipe(pad, sizeof pad);
}

// ---- AEAD ----------------------------------------------------------------------------------------
namespace {
void pad16(Poly1305& p, size_t n) {
  static const uint8_t zeros[16] = {0};
  if (n % 16) p.update(zeros, 16 - n % 16);
}

void aead_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* ad, size_t adlen, const uint8_t* ct,
              size_t ctlen, uint8_t tag[16]) {
  uint8_t block0[64];
  chacha20_block(key, 0, nonce, block0);
  Poly1305 p(block0);
  wipe(block0, sizeof block0);
  p.update(ad, adlen);
  pad16(p, adlen);
  p.update(ct, ctlen);
  pad16(p, ctlen);
  uint8_t lens[16];
  st64(lens, adlen);
  st64(lens + 8, ctlen);
  p.update(lens, 16);
  p.finish(tag);
}
}  // namespace

Bytes aead_chacha20poly1305_encrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* ad, size_t adlen,
                                    const uint8_t* pt, size_t ptlen) {
  Bytes out(ptlen + 16);
  chacha20_xor(out.data(), pt, ptlen, key, nonce, 1);
  aead_tag(key, nonce, ad, adlen, out.data(), ptlen, out.data() + ptlen);
  return out;
}

bool aead_chacha20poly1305_decrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* ad, size_t adlen,
                                   const uint8_t* ct, size_t ctlen, Bytes& pt) {
  if (ctlen < 16) return false;
  const size_t n = ctlen - 16;
  uint8_t tag[16];
  aead_tag(key, nonce, ad, adlen, ct, n, tag);
  if (!ct_equal(tag, ct + n, 16)) return false;
  pt.resize(n);
  chacha20_xor(pt.data(), ct, n, key, nonce, 1);
  return true;
}

Bytes aead_xchacha20poly1305_encrypt(const uint8_t key[32], const uint8_t nonce[24], const uint8_t* ad, size_t adlen,
                                     const uint8_t* pt, size_t ptlen) {
  uint8_t sub[32], n12[12] = {0};
  hchacha20(sub, nonce, key);
  std::memcpy(n12 + 4, nonce + 16, 8);
  Bytes out = aead_chacha20poly1305_encrypt(sub, n12, ad, adlen, pt, ptlen);
  wipe(sub, sizeof sub);
  return out;
}

bool aead_xchacha20poly1305_decrypt(const uint8_t key[32], const uint8_t nonce[24], const uint8_t* ad, size_t adlen,
                                    const uint8_t* ct, size_t ctlen, Bytes& pt) {
  uint8_t sub[32], n12[12] = {0};
  hchacha20(sub, nonce, key);
  std::memcpy(n12 + 4, nonce + 16, 8);
  const bool ok = aead_chacha20poly1305_decrypt(sub, n12, ad, adlen, ct, ctlen, pt);
  wipe(sub, sizeof sub);
  return ok;
}

}  // namespace symnet
