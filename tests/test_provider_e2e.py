"""BASELINE config 1 end-to-end on CPU (SURVEY.md §4.2 'Integration'): discovery node +
Symmetry server + provider (proxy and native backends) + mock Ollama + client, all over the
encrypted swarm on 127.0.0.1."""
import asyncio
import json
import os

import pytest
import yaml

from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
from symmetry_amd.net import DiscoveryServer
from symmetry_amd.provider.node import SymmetryProvider
from symmetry_amd.testing.mock_client import SymmetryClient
from symmetry_amd.testing.mock_ollama import MockOllama
from symmetry_amd.testing.mock_server import SymmetryServer


def _cfg(tmp_path, server_key, **over):
    cfg = {"apiHostname": "127.0.0.1", "apiKey": "sk-secret", "apiPath": "/v1/chat/completions", "apiPort": 11434,
           "apiProtocol": "http", "apiProvider": "ollama", "dataCollectionEnabled": True, "maxConnections": 10,
           "modelName": "llama3:8b", "name": "tester", "path": str(tmp_path / "data"), "public": True,
           "serverKey": server_key}
    cfg.update(over)
    p = tmp_path / "provider.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return str(p)


class Harness:
    def __init__(self, tmp_path, backend=None, ollama_kw=None, server_kw=None, **cfg_over):
        self.tmp_path, self.backend = tmp_path, backend
        self.ollama_kw, self.server_kw, self.cfg_over = ollama_kw or {}, server_kw or {}, cfg_over

    async def __aenter__(self):
        self.ds = DiscoveryServer()
        await self.ds.start()
        self.boot = [self.ds.address]
        self.server = SymmetryServer(bootstrap=self.boot, ping_interval=0.2, **self.server_kw)
        await self.server.start()
        self.ollama = MockOllama(**self.ollama_kw)
        port = await self.ollama.start()
        over = dict(self.cfg_over)
        over.setdefault("apiPort", port)
        self.cfg_path = _cfg(self.tmp_path, self.server.server_key, **over)
        self.provider = SymmetryProvider(self.cfg_path, backend=self.backend, bootstrap=self.boot)
        await self.provider.init()
        for _ in range(100):
            if self.server.providers():
                break
            await asyncio.sleep(0.05)
        self.clients = []
        return self

    async def client(self):
        c = SymmetryClient(self.boot, self.server.server_key)
        await c.start()
        self.clients.append(c)
        return c

    async def connect(self):
        c = await self.client()
        det = await c.request_provider("llama3:8b")
        return c, await c.connect_provider(det["discoveryKey"])

    async def __aexit__(self, *a):
        for c in self.clients:
            await c.stop()
        await self.provider.destroy()
        await self.server.stop()
        await self.ollama.stop()
        await self.ds.stop()


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


def test_registration_auth_and_join_payload(tmp_path):
    async def main():
        async with Harness(tmp_path) as h:
            assert h.provider._server_verified is True
            join = h.server.joins[-1]
            assert join["discoveryKey"] == h.provider.discovery_key.hex()
            assert join["modelName"] == "llama3:8b" and join["name"] == "tester"
            assert join["apiKey"] is None  # redacted
            await asyncio.sleep(0.5)
            assert h.server.pongs >= 1  # ping -> pong liveness
            rows = h.server.providers("llama3:8b")
            assert rows and rows[0]["discovery_key"] == h.provider.discovery_key.hex()

    run(main())


def test_forged_server_signature_is_detected(tmp_path):
    async def main():
        async with Harness(tmp_path, server_kw={"sign_bad": True}, strictServerAuth=True) as h:
            for _ in range(40):
                if h.provider._server_verified is not None:
                    break
                await asyncio.sleep(0.05)
            assert h.provider._server_verified is False

    run(main())


def test_proxy_stream_order_and_data_collection(tmp_path):
    async def main():
        async with Harness(tmp_path) as h:
            c, conn = await h.connect()
            msgs = [{"role": "user", "content": "hello world"}]
            r = await c.chat(conn, msgs)
            assert r.header == {"symmetryEmitterKey": "inference"}
            assert r.ended and r.ended_key == "inference"
            assert r.text == "Echo from mock ollama: hello world"
            body = h.ollama.requests[-1]
            assert body == {"model": "llama3:8b", "messages": msgs, "stream": True}
            assert h.ollama.headers[-1]["Authorization"] == "Bearer sk-secret"
            await asyncio.sleep(0.3)
            name = f"{h.provider.key_pair.public_key.hex()}-1.json"
            path = os.path.join(tmp_path, "data", name)
            saved = json.loads(open(path).read())
            assert saved == msgs + [{"role": "assistant", "content": r.text}]
            # a different emitter key streams but is not collected
            r2 = await c.chat(conn, msgs, emitter_key="chat-42", new_conversation=True)
            assert r2.ended_key == "chat-42"
            await asyncio.sleep(0.2)
            assert not os.path.exists(os.path.join(tmp_path, "data", f"{h.provider.key_pair.public_key.hex()}-2.json"))

    run(main())


def test_upstream_error_sends_error_event_and_inference_ended(tmp_path):
    async def main():
        async with Harness(tmp_path, ollama_kw={"status": 500}) as h:
            c, conn = await h.connect()
            r = await c.chat(conn, [{"role": "user", "content": "x"}])
            assert r.ended and r.error is not None and "500" in r.error

    run(main())


def _tiny_engine(max_num_seqs=4):
    return LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=max_num_seqs, max_model_len=512,
                                  block_size=32, default_max_tokens=12))


def test_native_backend_streams_one_event_per_token(tmp_path):
    from symmetry_amd.backends.native import NativeBackend

    async def main():
        eng = _tiny_engine()
        backend = NativeBackend({"modelName": "tiny-llama"}, engine=eng)
        async with Harness(tmp_path, backend=backend, apiProvider="native", modelName="llama3:8b") as h:
            c, conn = await h.connect()
            msgs = [{"role": "user", "content": "hi"}]
            r = await c.chat(conn, msgs, extra={"max_tokens": 9, "ignore_eos": True})
            assert r.ended and r.header == {"symmetryEmitterKey": "inference"}
            # chunk k is one SSE event; tokens = content events; plus the final [DONE] event
            assert r.chunks[-1] == b"data: [DONE]\n\n"
            assert all(ch.startswith(b"data: ") and ch.count(b"data:") == 1 for ch in r.chunks)
            assert len(r.chunks) >= 9
            from symmetry_amd.engine.sequence import SamplingParams

            other = _tiny_engine()  # same seed -> same weights; the served engine's thread stays untouched
            ref = other.generate(other.tokenizer.apply_chat_template(msgs),
                                 SamplingParams(max_tokens=9, ignore_eos=True))
            assert r.text == other.tokenizer.decode(ref)

    run(main())


def test_client_disconnect_aborts_generation(tmp_path):
    from symmetry_amd.backends.native import NativeBackend

    async def main():
        eng = _tiny_engine()
        backend = NativeBackend({"modelName": "tiny-llama"}, engine=eng)
        async with Harness(tmp_path, backend=backend, apiProvider="native") as h:
            c, conn = await h.connect()
            await c.chat(conn, [{"role": "user", "content": "x"}], extra={"max_tokens": 400, "ignore_eos": True},
                         disconnect_after=3)
            for _ in range(100):
                if not eng.scheduler.has_work():
                    break
                await asyncio.sleep(0.05)
            assert not eng.scheduler.has_work()
            assert eng.blocks.num_free == eng.blocks.num_blocks - eng.blocks.reserved

    run(main())


def test_max_connections_is_enforced(tmp_path):
    async def main():
        async with Harness(tmp_path, maxConnections=1) as h:
            c1, conn1 = await h.connect()
            c2 = await h.client()
            det = await c2.request_provider("llama3:8b")
            try:
                conn2 = await c2.connect_provider(det["discoveryKey"], timeout=1.5)
            except asyncio.TimeoutError:
                conn2 = None
            # the provider admits the authenticated stream only while under maxConnections: the
            # second peer is dropped right after its handshake
            for _ in range(40):
                if conn2 is None or not conn2.writable:
                    break
                await asyncio.sleep(0.05)
            assert conn2 is None or not conn2.writable
            assert len(h.provider._provider_swarm.peers) == 1
            r = await c1.chat(conn1, [{"role": "user", "content": "still served"}])
            assert r.ended

    run(main())


def test_concurrent_clients(tmp_path):
    async def main():
        async with Harness(tmp_path, ollama_kw={"delay_s": 0.01}) as h:
            pairs = [await h.connect() for _ in range(3)]
            res = await asyncio.gather(*(c.chat(conn, [{"role": "user", "content": f"q{i}"}])
                                         for i, (c, conn) in enumerate(pairs)))
            assert [r.text for r in res] == [f"Echo from mock ollama: q{i}" for i in range(3)]

    run(main())
