"""Identities and topics (hypercore-crypto semantics, REF ``global.d.ts:38-51``).

* ``key_pair(seed)``     ed25519 keypair from a 32-byte seed (crypto_sign_seed_keypair)
* ``discovery_key(pk)``  BLAKE2b-256(message="hypercore", key=pk) (crypto_generichash)
* ``verify/sign``        ed25519 detached
* ``seed_from_name``     ``Buffer.alloc(32).fill(name)`` -- the provider identity seed
  (``src/provider.ts:41-43``): the UTF-8 bytes of ``name`` repeated and
  truncated to 32 bytes; an empty or missing name gives an all-zero seed.
* ``server_topic``       ``discoveryKey(Buffer.from(serverKey))`` -- the UTF-8
  bytes of the 64-char hex string, NOT hex-decoded (``src/provider.ts:85-86``).
* ``server_public_key``  the hex-decoded 32-byte ed25519 key used to verify the
  server's signature (``src/provider.ts:133-141``).
"""
from __future__ import annotations

from dataclasses import dataclass

from . import _native


@dataclass(frozen=True)
class KeyPair:
    public_key: bytes
    secret_key: bytes  # libsodium layout: seed || public key


def key_pair(seed: bytes | None = None) -> KeyPair:
    if seed is None:
        seed = _native.random_bytes(32)
    if len(seed) != 32:
        raise ValueError("seed must be 32 bytes")
    pk, sk = _native.keypair(bytes(seed))
    return KeyPair(pk, sk)


def seed_from_name(name) -> bytes:
    if name is None or name == "":
        return bytes(32)
    raw = str(name).encode("utf-8")
    return (raw * (32 // len(raw) + 1))[:32]


def discovery_key(key: bytes) -> bytes:
    return _native.discovery_key(bytes(key))


def random_bytes(n: int = 32) -> bytes:
    return _native.random_bytes(n)


def sign(message: bytes, secret_key: bytes) -> bytes:
    return _native.sign(bytes(message), bytes(secret_key))


def verify(message: bytes, signature: bytes, public_key: bytes) -> bool:
    return bool(_native.verify(bytes(message), bytes(signature), bytes(public_key)))


def server_topic(server_key_hex: str) -> bytes:
    return discovery_key(str(server_key_hex).encode("utf-8"))


def server_public_key(server_key_hex: str) -> bytes:
    pk = bytes.fromhex(server_key_hex)
    if len(pk) != 32:
        raise ValueError(f"Expected a 32-byte public key, but got {len(pk)} bytes")
    return pk
