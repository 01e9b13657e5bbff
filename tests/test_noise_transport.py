"""Noise XX handshake, secretstream and the epoll transport / swarm (C++ data plane)."""
import asyncio

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from symmetry_amd.net import DiscoveryServer, Swarm, discovery_key, identity
from symmetry_amd.net import _native as n


def _pair():
    a = identity.key_pair(b"A" * 32)
    b = identity.key_pair(b"B" * 32)
    return a, b


def _handshake(prologue=b""):
    a, b = _pair()
    i = n.NoiseXX(True, a.public_key, a.secret_key, prologue)
    r = n.NoiseXX(False, b.public_key, b.secret_key, prologue)
    m1 = i.write_message(b"")
    assert r.read_message(m1) == b""
    m2 = r.write_message(b"resp-payload")
    assert i.read_message(m2) == b"resp-payload"
    m3 = i.write_message(b"init-payload")
    assert r.read_message(m3) == b"init-payload"
    return a, b, i, r, (m1, m2, m3)


def test_noise_xx_roundtrip_and_identities():
    a, b, i, r, msgs = _handshake()
    assert i.complete and r.complete
    assert i.remote_public_key == b.public_key
    assert r.remote_public_key == a.public_key
    assert i.handshake_hash == r.handshake_hash
    itx, irx = i.split()
    rtx, rrx = r.split()
    assert itx == rrx and irx == rtx and itx != irx
    # message sizes of the XX pattern: e | e,enc(s),enc(payload) | enc(s),enc(payload)
    assert len(msgs[0]) == 32
    assert len(msgs[1]) == 32 + 48 + len(b"resp-payload") + 16


def test_noise_rejects_tampering_and_prologue_mismatch():
    a, b = _pair()
    i = n.NoiseXX(True, a.public_key, a.secret_key)
    r = n.NoiseXX(False, b.public_key, b.secret_key)
    r.read_message(i.write_message(b""))
    m2 = bytearray(r.write_message(b""))
    m2[40] ^= 1
    with pytest.raises(ValueError):
        i.read_message(bytes(m2))
    i = n.NoiseXX(True, a.public_key, a.secret_key, b"p1")
    r = n.NoiseXX(False, b.public_key, b.secret_key, b"p2")
    r.read_message(i.write_message(b""))
    with pytest.raises(ValueError):
        i.read_message(r.write_message(b""))


def test_secretstream_roundtrip_tags_rekey_and_tamper():
    key = n.random_bytes(32)
    push, header = n.SecretStream.push_init(key)
    pull = n.SecretStream.pull_init(key, header)
    for i in range(50):
        msg = bytes([i]) * i
        tag = 2 if i == 20 else 0  # explicit REKEY in the middle
        ct = push.push(msg, tag)
        assert len(ct) == len(msg) + 17
        assert pull.pull(ct) == (msg, tag)
    ct = push.push(b"final", 3)
    bad = bytearray(ct)
    bad[-1] ^= 1
    with pytest.raises(ValueError):
        pull.pull(bytes(bad))
    # replay / reorder is rejected: the state advanced
    c1, c2 = push.push(b"one"), push.push(b"two")
    with pytest.raises(ValueError):
        pull.pull(c2)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.binary(max_size=300), max_size=20), st.binary(max_size=16))
def test_secretstream_fuzz(msgs, ad):
    key = n.random_bytes(32)
    push, header = n.SecretStream.push_init(key)
    pull = n.SecretStream.pull_init(key, header)
    for m in msgs:
        assert pull.pull(push.push(m, 0, ad), ad)[0] == m


async def _swarm_pair(**kw):
    ds = DiscoveryServer()
    await ds.start()
    a = Swarm(bootstrap=[ds.address], **kw)
    b = Swarm(bootstrap=[ds.address], **kw)
    return ds, a, b


def test_swarm_messages_preserve_boundaries_and_backpressure():
    async def main():
        ds, a, b = await _swarm_pair(high_watermark=1 << 16)
        topic = discovery_key(b"t" * 32)
        got = asyncio.Queue()
        a.on("connection", lambda c, i: c.on("data", lambda d: c.write(d)))
        conns = []

        def on_b(c, i):
            conns.append(c)
            c.on("data", got.put_nowait)

        b.on("connection", on_b)
        await a.join(topic, server=True, client=False).flushed()
        await b.join(topic, server=False, client=True).flushed()
        for _ in range(50):
            if conns:
                break
            await asyncio.sleep(0.05)
        c = conns[0]
        assert c.remote_public_key == a.key_pair.public_key
        assert c.raw_stream.remote_host == "127.0.0.1"
        sizes = [0, 1, 100, 65535, 70000, 1 << 20]
        saw_false = False
        for s in sizes:
            ok = c.write(bytes([s % 251]) * s)
            if not ok:
                saw_false = True
                await c.drain()
        assert saw_false  # 1 MiB > 64 KiB high-water mark
        for s in sizes:
            if s == 0:
                continue  # empty writes are keep-alives on the wire: never delivered
            d = await asyncio.wait_for(got.get(), 10)
            assert len(d) == s and d == bytes([s % 251]) * s
        await a.destroy()
        await b.destroy()
        await ds.stop()

    asyncio.run(main())


def test_swarm_firewall_and_max_connections():
    async def main():
        ds = DiscoveryServer()
        await ds.start()
        topic = discovery_key(b"f" * 32)
        server = Swarm(bootstrap=[ds.address], max_connections=1)
        seen = []
        server.on("connection", lambda c, i: seen.append(c))
        await server.join(topic, server=True, client=False).flushed()
        clients = [Swarm(bootstrap=[ds.address]) for _ in range(3)]
        for cl in clients:
            await cl.join(topic, server=False, client=True).flushed()
        await asyncio.sleep(0.5)
        assert len(server.peers) == 1 and len(seen) == 1
        # firewall rejects a specific key
        blocked = identity.key_pair(b"Z" * 32)
        fw = Swarm(bootstrap=[ds.address], firewall=lambda pk: pk == blocked.public_key)
        await fw.join(discovery_key(b"g" * 32), server=True, client=False).flushed()
        bad = Swarm(blocked, bootstrap=[ds.address])
        await bad.join(discovery_key(b"g" * 32), server=False, client=True).flushed()
        await asyncio.sleep(0.3)
        assert not fw.peers
        for s in clients + [server, fw, bad]:
            await s.destroy()
        await ds.stop()

    asyncio.run(main())


def test_swarm_reconnects_after_drop():
    async def main():
        ds, a, b = await _swarm_pair()
        b.refresh_interval = 0.2
        topic = discovery_key(b"r" * 32)
        opened = []
        b.on("connection", lambda c, i: opened.append(c))
        await a.join(topic, server=True, client=False).flushed()
        await b.join(topic, server=False, client=True).flushed()
        for _ in range(40):
            if opened:
                break
            await asyncio.sleep(0.05)
        assert len(opened) == 1
        for c in list(a.connections):
            c.destroy()
        for _ in range(80):
            if len(opened) >= 2:
                break
            await asyncio.sleep(0.05)
        assert len(opened) >= 2 and opened[-1].writable
        await a.destroy()
        await b.destroy()
        await ds.stop()

    asyncio.run(main())
