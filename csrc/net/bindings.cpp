// pybind11 module symmetry_amd.net._native: crypto primitives, Noise XX,
// secretstream and the epoll transport.  Long-running work never holds the
// GIL: the transport thread is pure C++ and Python only drains its event queue.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "crypto.h"
#include "noise.h"
#include "transport.h"

namespace py = pybind11;
using namespace symnet;

namespace {

std::string need(const py::bytes& b, size_t n, const char* what) {
  std::string s = b;
  if (s.size() != n) throw py::value_error(std::string(what) + " must be " + std::to_string(n) + " bytes");
  return s;
}

const uint8_t* u8(const std::string& s) { return reinterpret_cast<const uint8_t*>(s.data()); }
py::bytes pyb(const uint8_t* p, size_t n) { return py::bytes(reinterpret_cast<const char*>(p), n); }
py::bytes pyb(const Bytes& b) { return pyb(b.data(), b.size()); }

KeyPair kp_from(const py::bytes& pk, const py::bytes& sk) {
  KeyPair kp;
  std::string p = need(pk, 32, "public key"), s = need(sk, 64, "secret key");
  std::memcpy(kp.pk, p.data(), 32);
  std::memcpy(kp.sk, s.data(), 64);
  return kp;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "symmetry_amd P2P plane: crypto, Noise XX, secretstream, epoll transport";

  // ---- crypto ----------------------------------------------------------------------------------
  m.def("random_bytes", [](size_t n) { return pyb(random_bytes(n)); });
  m.def("keypair", [](py::bytes seed) {
    std::string s = need(seed, 32, "seed");
    KeyPair kp = keypair_from_seed(u8(s));
    return py::make_tuple(pyb(kp.pk, 32), pyb(kp.sk, 64));
  });
  m.def("sign", [](py::bytes msg, py::bytes sk) {
    std::string mm = msg, s = need(sk, 64, "secret key");
    uint8_t sig[64];
    ed25519_sign(u8(mm), mm.size(), u8(s), sig);
    return pyb(sig, 64);
  });
  m.def("verify", [](py::bytes msg, py::bytes sig, py::bytes pk) {
    std::string mm = msg, sg = sig, p = pk;
    if (sg.size() != 64 || p.size() != 32) return false;
    return ed25519_verify(u8(mm), mm.size(), u8(sg), u8(p));
  });
  m.def("discovery_key", [](py::bytes key) {
    std::string k = key;
    if (k.empty() || k.size() > 64) throw py::value_error("key must be 1..64 bytes");
    uint8_t out[32];
    discovery_key(u8(k), k.size(), out);
    return pyb(out, 32);
  });
  m.def(
      "blake2b",
      [](py::bytes data, size_t outlen, py::bytes key) {
        std::string d = data, k = key;
        uint8_t out[64];
        blake2b(out, outlen, u8(d), d.size(), k.empty() ? nullptr : u8(k), k.size());
        return pyb(out, outlen);
      },
      py::arg("data"), py::arg("outlen") = 64, py::arg("key") = py::bytes());
  m.def("x25519_public", [](py::bytes sk) {
    std::string s = need(sk, 32, "secret key");
    uint8_t pk[32];
    x25519_public(u8(s), pk);
    return pyb(pk, 32);
  });
  m.def("x25519", [](py::bytes sk, py::bytes pk) -> py::object {
    std::string s = need(sk, 32, "secret key"), p = need(pk, 32, "public key");
    uint8_t out[32];
    if (!x25519(u8(s), u8(p), out)) return py::none();
    return pyb(out, 32);
  });
  m.def("ed25519_pk_to_x25519", [](py::bytes pk) -> py::object {
    std::string p = need(pk, 32, "public key");
    uint8_t out[32];
    if (!ed25519_pk_to_x25519(u8(p), out)) return py::none();
    return pyb(out, 32);
  });
  m.def("ed25519_sk_to_x25519", [](py::bytes sk) {
    std::string s = need(sk, 64, "secret key");
    uint8_t out[32];
    ed25519_sk_to_x25519(u8(s), out);
    return pyb(out, 32);
  });
  m.def("hchacha20", [](py::bytes in, py::bytes key) {
    std::string i = need(in, 16, "input"), k = need(key, 32, "key");
    uint8_t out[32];
    hchacha20(out, u8(i), u8(k));
    return pyb(out, 32);
  });
  m.def("chacha20_block", [](py::bytes key, uint32_t counter, py::bytes nonce) {
    std::string k = need(key, 32, "key"), n = need(nonce, 12, "nonce");
    uint8_t out[64];
    chacha20_block(u8(k), counter, u8(n), out);
    return pyb(out, 64);
  });
  m.def("poly1305", [](py::bytes key, py::bytes msg) {
    std::string k = need(key, 32, "key"), mm = msg;
    Poly1305 p(u8(k));
    p.update(u8(mm), mm.size());
    uint8_t mac[16];
    p.finish(mac);
    return pyb(mac, 16);
  });
  m.def("aead_encrypt", [](py::bytes key, py::bytes nonce, py::bytes ad, py::bytes pt) {
    std::string k = need(key, 32, "key"), n = need(nonce, 12, "nonce"), a = ad, p = pt;
    return pyb(aead_chacha20poly1305_encrypt(u8(k), u8(n), u8(a), a.size(), u8(p), p.size()));
  });
  m.def("aead_decrypt", [](py::bytes key, py::bytes nonce, py::bytes ad, py::bytes ct) -> py::object {
    std::string k = need(key, 32, "key"), n = need(nonce, 12, "nonce"), a = ad, c = ct;
    Bytes out;
    if (!aead_chacha20poly1305_decrypt(u8(k), u8(n), u8(a), a.size(), u8(c), c.size(), out)) return py::none();
    return pyb(out);
  });
  m.def("xaead_encrypt", [](py::bytes key, py::bytes nonce, py::bytes ad, py::bytes pt) {
    std::string k = need(key, 32, "key"), n = need(nonce, 24, "nonce"), a = ad, p = pt;
    return pyb(aead_xchacha20poly1305_encrypt(u8(k), u8(n), u8(a), a.size(), u8(p), p.size()));
  });
  m.def("xaead_decrypt", [](py::bytes key, py::bytes nonce, py::bytes ad, py::bytes ct) -> py::object {
    std::string k = need(key, 32, "key"), n = need(nonce, 24, "nonce"), a = ad, c = ct;
    Bytes out;
    if (!aead_xchacha20poly1305_decrypt(u8(k), u8(n), u8(a), a.size(), u8(c), c.size(), out)) return py::none();
    return pyb(out);
  });

  // ---- Noise XX ---------------------------------------------------------------------------------
  py::class_<NoiseXX>(m, "NoiseXX")
      .def(py::init([](bool initiator, py::bytes pk, py::bytes sk, py::bytes prologue) {
             std::string pr = prologue;
             return new NoiseXX(initiator, kp_from(pk, sk), Bytes(pr.begin(), pr.end()));
           }),
           py::arg("initiator"), py::arg("public_key"), py::arg("secret_key"), py::arg("prologue") = py::bytes())
      .def("write_message",
           [](NoiseXX& h, py::bytes payload) {
             std::string p = payload;
             return pyb(h.write_message(u8(p), p.size()));
           },
           py::arg("payload") = py::bytes())
      .def("read_message",
           [](NoiseXX& h, py::bytes msg) {
             std::string mm = msg;
             try {
               return pyb(h.read_message(u8(mm), mm.size()));
             } catch (const CryptoError& e) {
               throw py::value_error(e.what());
             }
           })
      .def_property_readonly("complete", &NoiseXX::complete)
      .def_property_readonly("handshake_hash", [](NoiseXX& h) { return pyb(h.handshake_hash(), 64); })
      .def_property_readonly("remote_public_key", [](NoiseXX& h) { return pyb(h.remote_static(), 32); })
      .def("split", [](NoiseXX& h) {
        uint8_t tx[32], rx[32];
        h.split(tx, rx);
        return py::make_tuple(pyb(tx, 32), pyb(rx, 32));
      });

  // ---- secretstream ----------------------------------------------------------------------------
  py::class_<SecretStream>(m, "SecretStream")
      .def_static("push_init",
                  [](py::bytes key) {
                    std::string k = need(key, 32, "key");
                    auto* s = new SecretStream();
                    uint8_t header[24];
                    s->init_push(u8(k), header);
                    return py::make_tuple(py::cast(s, py::return_value_policy::take_ownership), pyb(header, 24));
                  })
      .def_static("pull_init",
                  [](py::bytes key, py::bytes header) {
                    std::string k = need(key, 32, "key"), h = need(header, 24, "header");
                    auto* s = new SecretStream();
                    s->init_pull(u8(k), u8(h));
                    return s;
                  },
                  py::return_value_policy::take_ownership)
      .def("push",
           [](SecretStream& s, py::bytes msg, uint8_t tag, py::bytes ad) {
             std::string mm = msg, a = ad;
             return pyb(s.push(u8(mm), mm.size(), tag, u8(a), a.size()));
           },
           py::arg("msg"), py::arg("tag") = 0, py::arg("ad") = py::bytes())
      .def("pull",
           [](SecretStream& s, py::bytes ct, py::bytes ad) {
             std::string c = ct, a = ad;
             Bytes out;
             uint8_t tag = 0;
             if (!s.pull(u8(c), c.size(), out, tag, u8(a), a.size()))
               throw py::value_error("secretstream: authentication failed");
             return py::make_tuple(pyb(out), tag);
           },
           py::arg("ct"), py::arg("ad") = py::bytes())
      .def("rekey", &SecretStream::rekey);

  // ---- transport -------------------------------------------------------------------------------
  py::class_<Transport>(m, "Transport")
      .def(py::init([](py::bytes pk, py::bytes sk, int keepalive_ms, int timeout_ms, size_t hwm) {
             return new Transport(kp_from(pk, sk), keepalive_ms, timeout_ms, hwm);
           }),
           py::arg("public_key"), py::arg("secret_key"), py::arg("keepalive_ms") = 5000,
           py::arg("timeout_ms") = 20000, py::arg("high_watermark") = 1 << 20)
      .def("listen", &Transport::listen, py::arg("host") = "127.0.0.1", py::arg("port") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("connect", &Transport::connect, py::call_guard<py::gil_scoped_release>())
      .def("write",
           [](Transport& t, uint64_t id, py::bytes data) {
             std::string d = data;
             py::gil_scoped_release rel;
             return t.write(id, std::move(d));
           })
      .def("end", &Transport::end, py::call_guard<py::gil_scoped_release>())
      .def("inject_fault",
           [](Transport& t, uint64_t id, int mode, py::bytes data) { t.inject_fault(id, mode, std::string(data)); })
      .def("destroy", &Transport::destroy, py::call_guard<py::gil_scoped_release>())
      .def("queued", &Transport::queued)
      .def("fileno", &Transport::fileno)
      .def_property_readonly("public_key", [](Transport& t) { return py::bytes(t.public_key()); })
      .def("close", &Transport::close, py::call_guard<py::gil_scoped_release>())
      .def("poll", [](Transport& t) {
        std::vector<Event> evs;
        {
          py::gil_scoped_release rel;
          evs = t.poll();
        }
        py::list out;
        for (auto& e : evs) {
          static const char* kinds[] = {"open", "data", "drain", "close", "listen_error"};
          py::dict d;
          d["kind"] = kinds[e.kind];
          d["conn"] = e.conn;
          if (e.kind == Event::DATA) {
            d["data"] = py::bytes(e.data);
          } else if (e.kind == Event::CLOSE) {
            d["error"] = e.data;
          } else if (e.kind == Event::OPEN) {
            d["remote_public_key"] = py::bytes(e.remote_pk);
            d["handshake_hash"] = py::bytes(e.handshake_hash);
          }
          d["host"] = e.host;
          d["port"] = e.port;
          d["initiator"] = e.initiator;
          out.append(d);
        }
        return out;
      });
}
