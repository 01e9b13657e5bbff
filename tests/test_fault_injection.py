"""Fault injection over the real encrypted swarm: corrupt / unframed bytes on a client
stream, a stalled reader, the server dropping every provider link, and a backend fault mid-stream.
The provider must drop only the faulty peer, keep serving everyone else, free engine resources, and
re-register with the server by itself."""
import asyncio

from test_provider_e2e import Harness, _tiny_engine, run


def _peers(h):
    return len(h.provider._provider_swarm.peers)


async def _wait(pred, tries=100, dt=0.05):
    for _ in range(tries):
        if pred():
            return True
        await asyncio.sleep(dt)
    return pred()


def test_corrupt_and_unframed_bytes_drop_only_that_peer(tmp_path):
    async def main():
        async with Harness(tmp_path) as h:
            good_c, good = await h.connect()
            for kind in ("corrupt", "raw"):
                bad_c, bad = await h.connect()
                assert await _wait(lambda: _peers(h) == 2)
                bad.inject_fault(kind, b"\xff" * 64)
                # the provider fails authentication on that stream and closes it
                assert await _wait(lambda: _peers(h) == 1), kind
            r = await good_c.chat(good, [{"role": "user", "content": "after the faults"}])
            assert r.ended and r.text == "Echo from mock ollama: after the faults"

    run(main())


def test_stalled_consumer_is_cancelled_without_blocking_others():
    """A consumer that stops pulling outputs (stalled reader / stuck socket) is aborted once it is
    queue_limit outputs behind; the engine thread never blocks and other requests finish."""
    from symmetry_amd.engine.llm_engine import AsyncEngine
    from symmetry_amd.engine.sequence import SamplingParams

    async def main():
        eng = _tiny_engine()
        ae = AsyncEngine(eng, queue_limit=4)
        try:
            slow = ae.generate("slow", prompt_ids=[5, 6, 7], params=SamplingParams(max_tokens=300, ignore_eos=True))
            first = await slow.__anext__()  # then stall: never pull again until the fast request is done
            assert not first.finished
            outs = [o async for o in ae.generate("fast", prompt_ids=[9, 8],
                                                 params=SamplingParams(max_tokens=6, ignore_eos=True))]
            assert outs[-1].finished and outs[-1].error is None and sum(len(o.token_ids) for o in outs) == 6
            rest = [o async for o in slow]
            assert rest[-1].finished and rest[-1].error and "too slow" in rest[-1].error
            assert sum(len(o.token_ids) for o in rest) < 300
            assert await _wait(lambda: not eng.scheduler.has_work())
            assert eng.blocks.num_free == eng.blocks.num_blocks - eng.blocks.reserved
        finally:
            ae.stop()

    run(main())


def test_provider_reregisters_after_server_drops_links(tmp_path):
    async def main():
        async with Harness(tmp_path) as h:
            assert h.server.providers()
            first = h.server.providers()[0]["peer_key"]
            h.server.drop_providers()
            assert await _wait(lambda: not h.server.providers(), tries=40)
            # swarm reconnect with backoff -> challenge + join again -> registered and verified
            assert await _wait(lambda: bool(h.server.providers()), tries=200)
            assert h.server.providers()[0]["peer_key"] == first
            c, conn = await h.connect()
            r = await c.chat(conn, [{"role": "user", "content": "back"}])
            assert r.ended

    run(main())


def test_backend_fault_mid_stream_sends_error_and_keeps_serving(tmp_path):
    async def main():
        async with Harness(tmp_path, ollama_kw={"fail_after": 2}) as h:
            c, conn = await h.connect()
            r = await c.chat(conn, [{"role": "user", "content": "one two three four five"}])
            assert r.ended and r.error is not None
            c2, conn2 = await h.connect()  # the provider is still up and answers the next client
            r2 = await c2.chat(conn2, [{"role": "user", "content": "again"}])
            assert r2.ended

    run(main())


def test_direct_stream_congested_and_vanished_peers():
    """The callback streaming path (NativeBackend.stream_direct, used by the provider node): a peer that
    stays congested for maxBacklog outputs has its request aborted with BackendError; a peer that is gone
    aborts its request at once; a healthy one gets role, one event per token, finish_reason and [DONE]."""
    import json

    from symmetry_amd.backends.base import BackendError
    from symmetry_amd.backends.native import NativeBackend

    async def main():
        eng = _tiny_engine()
        be = NativeBackend({"modelName": "tiny-llama", "maxBacklog": 3}, engine=eng)
        await be.start()
        try:
            req = {"messages": [{"role": "user", "content": "hi"}], "max_tokens": 40, "ignore_eos": True}
            congested = []
            try:
                await be.stream_direct(req, lambda raw, d: congested.append(raw) or False)
                raise AssertionError("expected a slow-consumer abort")
            except BackendError as exc:
                assert "too slow" in str(exc)
            assert 3 < len(congested) < 40
            gone = []
            await be.stream_direct(req, lambda raw, d: gone.append(raw) and None)
            assert len(gone) == 1
            ok = []
            await be.stream_direct(req, lambda raw, d: ok.append(raw) or True)
            events = [r.decode() for r in ok]
            assert events[-1] == "data: [DONE]\n\n"
            objs = [json.loads(e[len("data: "):]) for e in events[:-1]]
            assert objs[0]["choices"][0]["delta"].get("role") == "assistant"
            assert objs[-1]["choices"][0]["finish_reason"] == "length"
            assert 2 <= len(objs) <= 40  # tokens that complete no UTF-8 text carry no event
            assert await _wait(lambda: not eng.has_unfinished())
        finally:
            await be.stop()

    run(main())
