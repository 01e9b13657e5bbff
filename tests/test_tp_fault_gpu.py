"""GPU-side fault containment of a tensor-parallel provider (What's weak #8).

Two ranks of a TP=2 provider share the one MI355X (``SYMMETRY_TP_COMM=gloo`` for the host-staged fallback) with
the xGMI kernels ON between the processes: every decode step is a replayed hipGraph whose row-parallel
projections are fused GEMM + peer-memory all-reduce launches (``SYMMETRY_XGMI_FUSED=force``) that SPIN on the
other rank's granules.  SIGKILL of rank 1 mid-stream must end rank 0's spinning graph through the error word
(set by rank 0's health monitor, ``parallel/health.py``), not the kernel's wait limit; then the client's stream
ends with the OpenAI error event + ``inferenceEnded``, the provider sends ``leave`` and exits non-zero
(``/root/reference/src/provider.ts:124-126`` liveness, ``:270-274`` error path; the reference has no TP).
"""
import asyncio
import os
import signal
import socket
import subprocess
import sys
import time

import pytest
import yaml

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_tp2_worker_killed_while_graphs_spin_on_xgmi(gpu, tmp_path):
    import psutil

    from symmetry_amd.net import DiscoveryServer
    from symmetry_amd.testing.mock_client import SymmetryClient
    from symmetry_amd.testing.mock_server import SymmetryServer

    async def main():
        ds = DiscoveryServer()
        await ds.start()
        boot = [ds.address]
        server = SymmetryServer(bootstrap=boot, ping_interval=1.0)
        await server.start()
        cfg = {"apiHostname": "127.0.0.1", "apiPath": "/v1/chat/completions", "apiPort": 0, "apiProtocol": "http",
               "apiProvider": "native", "dataCollectionEnabled": False, "maxConnections": 4,
               "modelName": "small-llama", "name": "tp-gpu-fault", "path": str(tmp_path / "data"), "public": True,
               "serverKey": server.server_key, "tensorParallelSize": 2, "maxModelLen": 4096, "metricsInterval": 0}
        path = tmp_path / "provider.yaml"
        path.write_text(yaml.safe_dump(cfg))
        env = dict(os.environ, PYTHONPATH=ROOT, SYMMETRY_TP_COMM="gloo", SYMMETRY_XGMI="1",
                   SYMMETRY_XGMI_GRAPHS="1", SYMMETRY_XGMI_FUSED="force")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "symmetry_amd.cli", "-c",
               str(path), "--bootstrap", f"{boot[0][0]}:{boot[0][1]}"]
        log = open(tmp_path / "provider.log", "w+")
        proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT,
                                start_new_session=True)
        try:
            for _ in range(900):
                if server.providers("small-llama") or proc.poll() is not None:
                    break
                await asyncio.sleep(0.1)
            log.seek(0)
            assert proc.poll() is None and server.providers("small-llama"), log.read()[-3000:]
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
            det = await c.request_provider("small-llama")
            conn = await c.connect_provider(det["discoveryKey"])
            streaming = asyncio.Event()
            chat = asyncio.ensure_future(c.chat(conn, [{"role": "user", "content": "kill a worker"}],
                                                extra={"max_tokens": 3000, "ignore_eos": True}, timeout=60,
                                                on_chunk=lambda r: r.content_events >= 20 and streaming.set()))
            await asyncio.wait_for(streaming.wait(), 60)
            os.kill(ranks["1"], signal.SIGKILL)  # exactly the worker rank found above
            t_kill = time.perf_counter()
            r = await chat
            t_ended = time.perf_counter() - t_kill
            await c.stop()
            assert r.ended and r.error is not None, (r.ended, r.error, r.content_events)
            # well inside the one-shot kernels' own wait limit: the error word ended the spinning graph
            assert r.content_events < 3000 and t_ended < 10, (r.content_events, t_ended)
            for _ in range(150):
                if server.leaves:
                    break
                await asyncio.sleep(0.1)
            assert server.leaves and not server.providers("small-llama"), server.leaves
            code = await asyncio.to_thread(proc.wait, 60)
            assert code != 0
            log.seek(0)
            text = log.read()
            print(f"stream ended {t_ended:.2f} s after the kill, {r.content_events} tokens, exit code {code}: "
                  f"{r.error[:120]}")
            return text
        finally:
            if proc.poll() is None:
                os.killpg(proc.pid, signal.SIGKILL)  # exactly the process group started above
                proc.wait(20)
            log.close()
            await server.stop()
            await ds.stop()

    asyncio.run(main())
