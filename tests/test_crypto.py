"""Known-answer tests for the C++ crypto core (csrc/net/crypto.cpp) and the
hypercore-crypto semantics built on it (SURVEY.md §4.2 'Unit: crypto/native')."""
import hashlib

import pytest

from symmetry_amd.net import _native as n
from symmetry_amd.net import identity

H = bytes.fromhex


def test_ed25519_rfc8032_test1():
    seed = H("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    pk, sk = n.keypair(seed)
    assert pk == H("d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a")
    assert sk == seed + pk
    sig = n.sign(b"", sk)
    assert sig == H("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b"
                    "46bd25bf5f0595bbe24655141438e7a100b")
    assert n.verify(b"", sig, pk)
    assert not n.verify(b"x", sig, pk)
    bad = bytearray(sig)
    bad[0] ^= 1
    assert not n.verify(b"", bytes(bad), pk)


def test_ed25519_libsodium_seed_vector():
    pk, _ = n.keypair(b"\x01" * 32)
    assert pk.hex() == "8a88e3dd7409f195fd52db2d3cba5d72ca6709bf1d94121bf3748801b40f6f5c"


def test_x25519_rfc7748():
    k = H("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4")
    u = H("e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c")
    assert n.x25519(k, u) == H("c3da55379de9c6908e94ea4df28d084f32eccf03491c71f754b4075577a28552")
    a = H("77076d0a7318a57d3c16c17251b26645df4c2f87ebc0992ab177fba51db92c2a")
    assert n.x25519_public(a) == H("8520f0098930a754748b7ddcb43ef75a0dbf3a0d26381af4eba4a98eaa9b4e6a")


def test_ed_to_x25519_conversion_is_consistent():
    for i in range(5):
        pk, sk = n.keypair(bytes([i + 7]) * 32)
        assert n.x25519_public(n.ed25519_sk_to_x25519(sk)) == n.ed25519_pk_to_x25519(pk)
    # DH agreement through converted identities (what Noise with ed25519 static keys relies on)
    pa, sa = n.keypair(b"a" * 32)
    pb, sb = n.keypair(b"b" * 32)
    s1 = n.x25519(n.ed25519_sk_to_x25519(sa), n.ed25519_pk_to_x25519(pb))
    s2 = n.x25519(n.ed25519_sk_to_x25519(sb), n.ed25519_pk_to_x25519(pa))
    assert s1 == s2 and s1 is not None


def test_blake2b_rfc7693_and_hashlib():
    assert n.blake2b(b"abc").hex() == (
        "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d17d87c5392aab792dc252d5de4533cc9518d38aa8"
        "dbf1925ab92386edd4009923")
    for size in (0, 1, 127, 128, 129, 1000):
        data = bytes(range(256)) * 4
        data = data[:size]
        for outlen in (16, 32, 64):
            for key in (b"", b"k", bytes(range(64))):
                assert n.blake2b(data, outlen, key) == hashlib.blake2b(data, digest_size=outlen, key=key).digest()


def test_discovery_key_is_keyed_blake2b_of_hypercore():
    pk = bytes(range(32))
    assert identity.discovery_key(pk) == hashlib.blake2b(b"hypercore", digest_size=32, key=pk).digest()
    # the server topic keys BLAKE2b with the 64 UTF-8 bytes of the hex string (src/provider.ts:85-86)
    sk_hex = "4b4a9cc325d134dee6679e9407420023531fd7e96c563f6c5d00fd5549b77435"
    assert identity.server_topic(sk_hex) == hashlib.blake2b(b"hypercore", digest_size=32,
                                                              key=sk_hex.encode()).digest()
    assert identity.server_public_key(sk_hex) == H(sk_hex)
    with pytest.raises(ValueError, match="Expected a 32-byte public key"):
        identity.server_public_key("abcd")


def test_seed_from_name_matches_buffer_fill():
    assert identity.seed_from_name("ab") == b"ab" * 16
    assert identity.seed_from_name("twinnydotdev") == (b"twinnydotdev" * 3)[:32]
    assert identity.seed_from_name("") == bytes(32)
    assert identity.seed_from_name(None) == bytes(32)
    assert identity.seed_from_name("é") == ("é".encode() * 16)[:32]
    assert len(identity.seed_from_name("x" * 100)) == 32


def test_chacha20_block_rfc8439():
    key = bytes(range(32))
    out = n.chacha20_block(key, 1, H("000000090000004a00000000"))
    assert out.hex().startswith("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e")


def test_poly1305_rfc8439():
    key = H("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    assert n.poly1305(key, b"Cryptographic Forum Research Group") == H("a8061dc1305136c6c22b8baf0c0127a9")


SUNSCREEN = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, "
             b"sunscreen would be it.")


def test_aead_chacha20poly1305_rfc8439():
    key = bytes(range(0x80, 0xa0))
    nonce = H("070000004041424344454647")
    ad = H("50515253c0c1c2c3c4c5c6c7")
    ct = n.aead_encrypt(key, nonce, ad, SUNSCREEN)
    assert ct[:16] == H("d31a8d34648e60db7b86afbc53ef7ec2")
    assert ct[-16:] == H("1ae10b594f09e26a7e902ecbd0600691")
    assert n.aead_decrypt(key, nonce, ad, ct) == SUNSCREEN
    tampered = bytearray(ct)
    tampered[3] ^= 0x40
    assert n.aead_decrypt(key, nonce, ad, bytes(tampered)) is None


def test_hchacha20_and_xchacha_draft_vectors():
    key = bytes(range(32))
    assert n.hchacha20(H("000000090000004a0000000031415927"), key) == H(
        "82413b4227b27bfed30e42508a877d73a0f9e4d58a74a853c12ec41326d3ecdc")
    key = bytes(range(0x80, 0xa0))
    nonce = bytes(range(0x40, 0x58))
    ad = H("50515253c0c1c2c3c4c5c6c7")
    ct = n.xaead_encrypt(key, nonce, ad, SUNSCREEN)
    assert ct[:16] == H("bd6d179d3e83d43b9576579493c0e939")
    assert ct[-16:] == H("c0875924c1c7987947deafd8780acf49")
    assert n.xaead_decrypt(key, nonce, ad, ct) == SUNSCREEN


def test_sign_verify_roundtrip_identity_module():
    kp = identity.key_pair(identity.seed_from_name("provider"))
    msg = identity.random_bytes(32)
    assert identity.verify(msg, identity.sign(msg, kp.secret_key), kp.public_key)
    assert not identity.verify(msg, bytes(64), kp.public_key)
