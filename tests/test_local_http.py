"""Local OpenAI-compatible endpoint of the native engine (``serveHttp``; SURVEY.md §2.3 apiHostname /
apiPort / apiPath in native mode): streaming and non-streaming chat, models, auth, and sharing the engine
with swarm peers (the proxy backend of a second provider can even relay to it, Ollama-style)."""
import asyncio
import json

import aiohttp

from test_provider_e2e import Harness, _tiny_engine, run


def test_native_engine_serves_openai_http_and_swarm_together(tmp_path):
    from symmetry_amd.backends.native import NativeBackend

    async def main():
        eng = _tiny_engine()
        backend = NativeBackend({"modelName": "tiny-llama"}, engine=eng)
        async with Harness(tmp_path, backend=backend, apiProvider="native", apiPort=0, serveHttp=True,
                           apiKey="local-secret") as h:
            base = f"http://{h.provider.http.host}:{h.provider.http.port}"
            hdr = {"Authorization": "Bearer local-secret"}
            body = {"model": "tiny-llama", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 6,
                    "ignore_eos": True}
            async with aiohttp.ClientSession() as s:
                async with s.get(base + "/v1/models") as r:
                    assert (await r.json())["data"][0]["id"] == "llama3:8b"
                async with s.post(base + "/v1/chat/completions", json=body) as r:
                    assert r.status == 401
                async with s.post(base + "/v1/chat/completions", json=body, headers=hdr) as r:
                    full = await r.json()
                msg = full["choices"][0]["message"]
                assert msg["role"] == "assistant" and full["choices"][0]["finish_reason"] == "length"
                async with s.post(base + "/v1/chat/completions", json=dict(body, stream=True), headers=hdr) as r:
                    raw = (await r.read()).decode()
                events = [e[6:] for e in raw.split("\n\n") if e.startswith("data: ")]
                assert events[-1] == "[DONE]"
                streamed = "".join((json.loads(e)["choices"][0]["delta"].get("content") or "") for e in events[:-1])
                assert streamed == msg["content"]  # greedy: stream and non-stream agree
                # a swarm client is served by the same engine concurrently
                c, conn = await h.connect()
                r_swarm, _ = await asyncio.gather(
                    c.chat(conn, [{"role": "user", "content": "hi"}], extra={"max_tokens": 6, "ignore_eos": True}),
                    s.post(base + "/v1/chat/completions", json=body, headers=hdr))
                assert r_swarm.ended and r_swarm.text == msg["content"]
                async with s.get(base + "/metrics") as r:
                    assert (await r.json())["requests"] >= 3

    run(main())
