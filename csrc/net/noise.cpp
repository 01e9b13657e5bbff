// Noise XX (Noise Protocol Framework rev. 34, §5 processing rules, §7.5 XX)
// over x25519-from-ed25519 DH, ChaCha20-Poly1305 and BLAKE2b; plus the
// libsodium secretstream construction.  See noise.h.
#include "noise.h"

#include <cstring>

namespace symnet {

namespace {
const char kProtocolName[] = "Noise_XX_25519_ChaChaPoly_BLAKE2b";

void le64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
}  // namespace

KeyPair keypair_from_seed(const uint8_t seed[32]) {
  KeyPair kp;
  ed25519_keypair_from_seed(seed, kp.pk, kp.sk);
  return kp;
}

KeyPair keypair_random() {
  uint8_t seed[32];
  random_bytes(seed, 32);
  KeyPair kp = keypair_from_seed(seed);
  wipe(seed, sizeof seed);
  return kp;
}

// ---- CipherState ---------------------------------------------------------------------------------
void CipherState::init(const uint8_t key[32]) {
  std::memcpy(k, key, 32);
  n = 0;
  has_key = true;
}

Bytes CipherState::encrypt(const uint8_t* ad, size_t adlen, const uint8_t* pt, size_t len) {
  if (!has_key) return Bytes(pt, pt + len);
  uint8_t nonce[12] = {0};
  le64(nonce + 4, n++);
  return aead_chacha20poly1305_encrypt(k, nonce, ad, adlen, pt, len);
}

bool CipherState::decrypt(const uint8_t* ad, size_t adlen, const uint8_t* ct, size_t len, Bytes& out) {
  if (!has_key) {
    out.assign(ct, ct + len);
    return true;
  }
  uint8_t nonce[12] = {0};
  le64(nonce + 4, n);
  if (!aead_chacha20poly1305_decrypt(k, nonce, ad, adlen, ct, len, out)) return false;
  ++n;
  return true;
}

// ---- HMAC / HKDF over BLAKE2b (HASHLEN 64, BLOCKLEN 128) --------------------------------------
void hmac_blake2b(const uint8_t* key, size_t keylen, const uint8_t* data, size_t n, uint8_t out[64]) {
  uint8_t k0[128] = {0};
  if (keylen > 128) {
    blake2b(k0, 64, key, keylen);
  } else {
    std::memcpy(k0, key, keylen);
  }
  uint8_t ipad[128], opad[128];
  for (int i = 0; i < 128; ++i) {
    ipad[i] = k0[i] ^ 0x36;
    opad[i] = k0[i] ^ 0x5c;
  }
  uint8_t inner[64];
  Blake2b a(64);
  a.update(ipad, 128);
  a.update(data, n);
  a.final(inner);
  Blake2b b(64);
  b.update(opad, 128);
  b.update(inner, 64);
  b.final(out);
  wipe(k0, sizeof k0);
}

void hkdf2(const uint8_t ck[64], const uint8_t* ikm, size_t n, uint8_t out1[64], uint8_t out2[64]) {
  uint8_t temp[64];
  hmac_blake2b(ck, 64, ikm, n, temp);
  const uint8_t one = 1;
  hmac_blake2b(temp, 64, &one, 1, out1);
  uint8_t buf[65];
  std::memcpy(buf, out1, 64);
  buf[64] = 2;
  hmac_blake2b(temp, 64, buf, 65, out2);
  wipe(temp, sizeof temp);
}

// ---- Handshake -------------------------------------------------------------------------------------
NoiseXX::NoiseXX(bool initiator, const KeyPair& s, const Bytes& prologue) : initiator_(initiator), s_(s) {
  std::memset(h_, 0, 64);
  std::memcpy(h_, kProtocolName, sizeof(kProtocolName) - 1);  // name <= HASHLEN: zero padded
  std::memcpy(ck_, h_, 64);
  mix_hash(prologue.data(), prologue.size());
}

void NoiseXX::mix_hash(const uint8_t* d, size_t n) {
  Blake2b b(64);
  b.update(h_, 64);
  b.update(d, n);
  b.final(h_);
}

void NoiseXX::mix_key(const uint8_t* ikm, size_t n) {
  uint8_t k[64];
  hkdf2(ck_, ikm, n, ck_, k);
  cs_.init(k);
  wipe(k, sizeof k);
}

Bytes NoiseXX::encrypt_and_hash(const uint8_t* pt, size_t n) {
  Bytes ct = cs_.encrypt(h_, 64, pt, n);
  mix_hash(ct.data(), ct.size());
  return ct;
}

Bytes NoiseXX::decrypt_and_hash(const uint8_t* ct, size_t n) {
  Bytes pt;
  uint8_t hcopy[64];
  std::memcpy(hcopy, h_, 64);
  if (!cs_.decrypt(hcopy, 64, ct, n, pt)) throw CryptoError("noise: decryption failed");
  mix_hash(ct, n);
  return pt;
}

void NoiseXX::dh(const KeyPair& local, const uint8_t remote[32], uint8_t out[32]) const {
  uint8_t xs[32], xp[32];
  ed25519_sk_to_x25519(local.sk, xs);
  if (!ed25519_pk_to_x25519(remote, xp) || !x25519(xs, xp, out)) {
    wipe(xs, sizeof xs);
    throw CryptoError("noise: invalid remote key");
  }
  wipe(xs, sizeof xs);
}

Bytes NoiseXX::write_message(const uint8_t* payload, size_t len) {
  if (complete() || !my_turn()) throw CryptoError("noise: not our turn to write");
  Bytes out;
  uint8_t shared[32];
  if (step_ == 0) {  // -> e
    e_ = keypair_random();
    out.insert(out.end(), e_.pk, e_.pk + 32);
    mix_hash(e_.pk, 32);
  } else if (step_ == 1) {  // <- e, ee, s, es
    e_ = keypair_random();
    out.insert(out.end(), e_.pk, e_.pk + 32);
    mix_hash(e_.pk, 32);
    dh(e_, re_, shared);
    mix_key(shared, 32);
    Bytes c = encrypt_and_hash(s_.pk, 32);
    out.insert(out.end(), c.begin(), c.end());
    dh(s_, re_, shared);
    mix_key(shared, 32);
  } else {  // -> s, se
    Bytes c = encrypt_and_hash(s_.pk, 32);
    out.insert(out.end(), c.begin(), c.end());
    dh(s_, re_, shared);
    mix_key(shared, 32);
  }
  wipe(shared, sizeof shared);
  Bytes c = encrypt_and_hash(payload, len);
  out.insert(out.end(), c.begin(), c.end());
  ++step_;
  return out;
}

Bytes NoiseXX::read_message(const uint8_t* msg, size_t len) {
  if (complete() || my_turn()) throw CryptoError("noise: not our turn to read");
  uint8_t shared[32];
  size_t off = 0;
  auto need = [&](size_t n) {
    if (len - off < n) throw CryptoError("noise: short message");
  };
  if (step_ == 0) {  // responder reads -> e
    need(32);
    std::memcpy(re_, msg, 32);
    mix_hash(re_, 32);
    off = 32;
  } else if (step_ == 1) {  // initiator reads <- e, ee, s, es
    need(32);
    std::memcpy(re_, msg, 32);
    mix_hash(re_, 32);
    off = 32;
    dh(e_, re_, shared);
    mix_key(shared, 32);
    need(48);
    Bytes s = decrypt_and_hash(msg + off, 48);
    off += 48;
    std::memcpy(rs_, s.data(), 32);
    dh(e_, rs_, shared);
    mix_key(shared, 32);
  } else {  // responder reads -> s, se
    need(48);
    Bytes s = decrypt_and_hash(msg + off, 48);
    off += 48;
    std::memcpy(rs_, s.data(), 32);
    dh(e_, rs_, shared);
    mix_key(shared, 32);
  }
  wipe(shared, sizeof shared);
  Bytes payload = decrypt_and_hash(msg + off, len - off);
  ++step_;
  return payload;
}

void NoiseXX::split(uint8_t tx[32], uint8_t rx[32]) const {
  if (!complete()) throw CryptoError("noise: handshake incomplete");
  uint8_t k1[64], k2[64];
  hkdf2(ck_, nullptr, 0, k1, k2);
  if (initiator_) {
    std::memcpy(tx, k1, 32);
    std::memcpy(rx, k2, 32);
  } else {
    std::memcpy(tx, k2, 32);
    std::memcpy(rx, k1, 32);
  }
  wipe(k1, sizeof k1);
  wipe(k2, sizeof k2);
}

// ---- secretstream -------------------------------------------------------------------------------------
void SecretStream::counter_reset() {
  std::memset(nonce_, 0, 4);
  nonce_[0] = 1;
}

void SecretStream::init_push(const uint8_t key[32], uint8_t header[24]) {
  random_bytes(header, 24);
  init_pull(key, header);
}

void SecretStream::init_pull(const uint8_t key[32], const uint8_t header[24]) {
  hchacha20(k_, header, key);
  counter_reset();
  std::memcpy(nonce_ + 4, header + 16, 8);
}

void SecretStream::rekey() {
  uint8_t buf[40];
  std::memcpy(buf, k_, 32);
  std::memcpy(buf + 32, nonce_ + 4, 8);
  chacha20_xor(buf, buf, 40, k_, nonce_, 0);
  std::memcpy(k_, buf, 32);
  std::memcpy(nonce_ + 4, buf + 32, 8);
  wipe(buf, sizeof buf);
  counter_reset();
}

void SecretStream::after_message(const uint8_t mac[16], uint8_t tag) {
  for (int i = 0; i < 8; ++i) nonce_[4 + i] ^= mac[i];
  // little-endian increment of the 32-bit counter
  uint16_t c = 1;
  for (int i = 0; i < 4; ++i) {
    c += nonce_[i];
    nonce_[i] = (uint8_t)c;
    c >>= 8;
  }
  const bool zero = (nonce_[0] | nonce_[1] | nonce_[2] | nonce_[3]) == 0;
  if ((tag & TAG_REKEY) || zero) rekey();
}

namespace {
void ss_pad(Poly1305& p, size_t n) {
  static const uint8_t zeros[16] = {0};
  const size_t r = (0x10 - n) & 0xf;
  if (r) p.update(zeros, r);
}
}  // namespace

Bytes SecretStream::push(const uint8_t* m, size_t mlen, uint8_t tag, const uint8_t* ad, size_t adlen) {
  Bytes out(1 + mlen + 16);
  uint8_t block[64];
  chacha20_block(k_, 0, nonce_, block);
  Poly1305 p(block);
  p.update(ad, adlen);
  ss_pad(p, adlen);
  std::memset(block, 0, 64);
  block[0] = tag;
  chacha20_xor(block, block, 64, k_, nonce_, 1);
  p.update(block, 64);
  out[0] = block[0];
  uint8_t* c = out.data() + 1;
  chacha20_xor(c, m, mlen, k_, nonce_, 2);
  p.update(c, mlen);
  ss_pad(p, 64 + mlen);
  uint8_t slen[8];
  le64(slen, adlen);
  p.update(slen, 8);
  le64(slen, 64 + mlen);
  p.update(slen, 8);
  uint8_t* mac = c + mlen;
  p.finish(mac);
  wipe(block, sizeof block);
  after_message(mac, tag);
  return out;
}

bool SecretStream::pull(const uint8_t* c, size_t clen, Bytes& m, uint8_t& tag, const uint8_t* ad, size_t adlen) {
  if (clen < ABYTES) return false;
  const size_t mlen = clen - ABYTES;
  uint8_t block[64];
  chacha20_block(k_, 0, nonce_, block);
  Poly1305 p(block);
  p.update(ad, adlen);
  ss_pad(p, adlen);
  std::memset(block, 0, 64);
  block[0] = c[0];
  chacha20_xor(block, block, 64, k_, nonce_, 1);
  const uint8_t t = block[0];
  block[0] = c[0];
  p.update(block, 64);
  const uint8_t* body = c + 1;
  p.update(body, mlen);
  ss_pad(p, 64 + mlen);
  uint8_t slen[8];
  le64(slen, adlen);
  p.update(slen, 8);
  le64(slen, 64 + mlen);
  p.update(slen, 8);
  uint8_t mac[16];
  p.finish(mac);
  wipe(block, sizeof block);
  if (!ct_equal(mac, body + mlen, 16)) return false;
  m.resize(mlen);
  chacha20_xor(m.data(), body, mlen, k_, nonce_, 2);
  tag = t;
  after_message(mac, t);
  return true;
}

}  // namespace symnet
