"""BASELINE config 4 shape on the CPU: a tensor-parallel provider launched exactly like the GPU one
(`torchrun --nproc-per-node 2 -m symmetry_amd.cli -c provider.yaml`, gloo instead of RCCL), registered
with a local server and streaming a chat to a client over the encrypted swarm.  Rank 0 serves the swarm,
rank 1 mirrors every engine step through the metadata broadcast."""
import asyncio
import os
import signal
import socket
import subprocess
import sys

import pytest
import yaml

from symmetry_amd.net import DiscoveryServer
from symmetry_amd.testing.mock_client import SymmetryClient
from symmetry_amd.testing.mock_server import SymmetryServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("launch", ["torchrun", "plain"])
def test_tp2_provider_over_torchrun_streams_like_tp1(tmp_path, launch):
    """``plain``: ``symmetry-cli -c provider.yaml`` with tensorParallelSize 2 starts the torchrun ranks itself."""
    async def main():
        ds = DiscoveryServer()
        await ds.start()
        boot = [ds.address]
        server = SymmetryServer(bootstrap=boot, ping_interval=1.0)
        await server.start()
        cfg = {"apiHostname": "127.0.0.1", "apiPath": "/v1/chat/completions", "apiPort": 0, "apiProtocol": "http",
               "apiProvider": "native", "dataCollectionEnabled": False, "maxConnections": 4,
               "modelName": "tiny-llama", "name": "tp-provider", "path": str(tmp_path / "data"), "public": True,
               "serverKey": server.server_key, "tensorParallelSize": 2, "device": "cpu", "maxModelLen": 256,
               "metricsInterval": 0}
        path = tmp_path / "provider.yaml"
        path.write_text(yaml.safe_dump(cfg))
        env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "symmetry_amd.cli", "-c",
               str(path), "--bootstrap", f"{boot[0][0]}:{boot[0][1]}"]
        if launch == "plain":
            cmd = [sys.executable, "-m", "symmetry_amd.cli", "-c", str(path), "--bootstrap", f"{boot[0][0]}:{boot[0][1]}"]
        proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                start_new_session=True)
        try:
            for _ in range(600):
                if server.providers("tiny-llama") or proc.poll() is not None:
                    break
                await asyncio.sleep(0.1)
            assert proc.poll() is None, proc.stderr.read().decode()[-3000:]
            assert server.providers("tiny-llama")
            c = SymmetryClient(boot, server.server_key)
            await c.start()
            det = await c.request_provider("tiny-llama")
            conn = await c.connect_provider(det["discoveryKey"])
            msgs = [{"role": "user", "content": "tensor parallel"}]
            r = await c.chat(conn, msgs, extra={"max_tokens": 8, "ignore_eos": True}, timeout=120)
            await c.stop()
            assert r.ended and r.error is None and r.content_events >= 1
            return r.text
        finally:
            os.killpg(proc.pid, signal.SIGTERM)  # exactly the process group started above
            try:
                proc.wait(20)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
            await server.stop()
            await ds.stop()

    text = asyncio.run(main())
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine
    from symmetry_amd.engine.sequence import SamplingParams

    ref = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=4, max_model_len=256,
                                 weight_init="full"))
    ids = ref.generate(ref.tokenizer.apply_chat_template([{"role": "user", "content": "tensor parallel"}]),
                       SamplingParams(max_tokens=8, ignore_eos=True))
    # same weights (seeded full init), same greedy decode: TP=2 over gloo reproduces the TP=1 text
    assert text == ref.tokenizer.decode(ids), (text, ref.tokenizer.decode(ids))


def test_tp_config_fails_at_startup_without_gpus(tmp_path):
    """tensorParallelSize 2 on a box with fewer GPUs: symmetry-cli exits non-zero before announcing."""
    from symmetry_amd import cli

    cfg = {"apiHostname": "127.0.0.1", "apiPath": "/v1/chat/completions", "apiPort": 0, "apiProtocol": "http",
           "apiProvider": "native", "modelName": "tiny-llama", "name": "tp", "path": str(tmp_path),
           "public": True, "serverKey": "00" * 32, "tensorParallelSize": 2}
    path = tmp_path / "provider.yaml"
    path.write_text(yaml.safe_dump(cfg))
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has the GPUs")
    assert cli.main(["-c", str(path)]) == 1
    plan = cli.tp_launch_plan(cfg, str(path), None)
    assert "--nproc-per-node=2" in plan and plan[-2:] == ["-c", str(path)]


def test_engine_refuses_tp_without_communicator():
    from symmetry_amd.engine.llm_engine import EngineConfig, LLMEngine

    with pytest.raises(ValueError, match="communicator"):
        LLMEngine(EngineConfig(model="tiny-llama", device="cpu", tp_size=2, max_model_len=128))


def test_tp2_worker_killed_mid_stream_fails_fast_and_leaves(tmp_path):
    """Fault containment: SIGKILL rank 1 of a streaming TP=2 provider.  Rank 0's health monitor sees
    the worker gone on the metadata ring's back-channel; the client's stream ends with the OpenAI error event +
    ``inferenceEnded`` within seconds, the provider sends ``leave`` to the server and exits non-zero (no hang,
    no half-alive provider answering pings)."""
    import time

    import psutil

    async def main():
        ds = DiscoveryServer()
        await ds.start()
        boot = [ds.address]
        server = SymmetryServer(bootstrap=boot, ping_interval=1.0)
        await server.start()
        cfg = {"apiHostname": "127.0.0.1", "apiPath": "/v1/chat/completions", "apiPort": 0, "apiProtocol": "http",
               "apiProvider": "native", "dataCollectionEnabled": False, "maxConnections": 4,
               "modelName": "tiny-llama", "name": "tp-fault", "path": str(tmp_path / "data"), "public": True,
               "serverKey": server.server_key, "tensorParallelSize": 2, "device": "cpu", "maxModelLen": 4096,
               "metricsInterval": 0}
        path = tmp_path / "provider.yaml"
        path.write_text(yaml.safe_dump(cfg))
        env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "symmetry_amd.cli", "-c",
               str(path), "--bootstrap", f"{boot[0][0]}:{boot[0][1]}"]
        proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                start_new_session=True)
        try:
            for _ in range(600):
                if server.providers("tiny-llama") or proc.poll() is not None:
                    break
                await asyncio.sleep(0.1)
            assert proc.poll() is None, proc.stderr.read().decode()[-3000:]
            ranks = {}
            for ch in psutil.Process(proc.pid).children(recursive=True):
                try:
                    r = ch.environ().get("RANK")
                except psutil.Error:
                    continue
                if r is not None and "symmetry_amd.cli" in " ".join(ch.cmdline()):
                    ranks[r] = ch.pid
            assert set(ranks) == {"0", "1"}, ranks
            c = SymmetryClient(boot, server.server_key)
            await c.start()
            det = await c.request_provider("tiny-llama")
            conn = await c.connect_provider(det["discoveryKey"])
            streaming = asyncio.Event()
            msgs = [{"role": "user", "content": "kill a worker"}]
            chat = asyncio.ensure_future(c.chat(conn, msgs, extra={"max_tokens": 3000, "ignore_eos": True},
                                                timeout=60, on_chunk=lambda r: r.content_events >= 5
                                                and streaming.set()))
            await asyncio.wait_for(streaming.wait(), 120)
            os.kill(ranks["1"], signal.SIGKILL)  # exactly the worker rank found above
            t_kill = time.perf_counter()
            r = await chat
            t_ended = time.perf_counter() - t_kill
            await c.stop()
            assert r.ended and r.error is not None, (r.ended, r.error, r.content_events)
            assert r.content_events < 3000 and t_ended < 15, (r.content_events, t_ended)
            for _ in range(150):
                if server.leaves:
                    break
                await asyncio.sleep(0.1)
            assert server.leaves and not server.providers("tiny-llama"), server.leaves
            code = await asyncio.to_thread(proc.wait, 60)
            assert code != 0
            print(f"stream ended {t_ended:.2f} s after the kill, {r.content_events} tokens, exit code {code}: "
                  f"{r.error[:120]}")
            return t_ended
        finally:
            if proc.poll() is None:
                os.killpg(proc.pid, signal.SIGKILL)  # exactly the process group started above
                proc.wait(20)
            await server.stop()
            await ds.stop()

    asyncio.run(main())
