"""Data-parallel replicas on one node (``symmetry-cli --replicas N``): the launch plan gives every replica
its own identity, ports, metrics file and GPU slice (a torchrun group when tensorParallelSize > 1), and a
real 2-replica launch registers two providers with the server, both serving chats over the swarm."""
import asyncio
import os
import signal
import subprocess
import sys

import pytest

from symmetry_amd.cli import REPLICA_ENV, replica_plan
from symmetry_amd.net import DiscoveryServer
from symmetry_amd.testing.mock_client import SymmetryClient
from symmetry_amd.testing.mock_ollama import MockOllama
from symmetry_amd.testing.mock_server import SymmetryServer
from test_provider_e2e import _cfg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_replica_plan_slices_gpus_and_identities():
    cfg = {"name": "node", "apiProvider": "native", "tensorParallelSize": 4, "listenPort": 7000,
           "serveHttp": True, "apiPort": 8000, "metricsFile": "/tmp/m.json"}
    plan = replica_plan(cfg, "p.yaml", 2, "127.0.0.1:1")
    (a0, e0), (a1, e1) = plan
    assert e0["HIP_VISIBLE_DEVICES"] == "0,1,2,3" and e1["HIP_VISIBLE_DEVICES"] == "4,5,6,7"
    assert (e0["SYMMETRY_NAME"], e1["SYMMETRY_NAME"]) == ("node-0", "node-1")
    assert (e0["SYMMETRY_LISTENPORT"], e1["SYMMETRY_LISTENPORT"]) == ("7000", "7001")
    assert (e0["SYMMETRY_APIPORT"], e1["SYMMETRY_APIPORT"]) == ("8000", "8001")
    assert e1["SYMMETRY_METRICSFILE"] == "/tmp/m-1.json" and e1[REPLICA_ENV] == "1"
    assert "torch.distributed.run" in a0 and "--nproc-per-node=4" in a0 and "--master-port=29601" in a1
    assert a0[-4:] == ["-c", "p.yaml", "--bootstrap", "127.0.0.1:1"]
    # a restricted launcher hands out slices of its own visible devices; tp 1 runs the CLI directly
    plan = replica_plan({"name": "n", "apiProvider": "native"}, "p.yaml", 3, visible="4,5,6")
    assert [e["HIP_VISIBLE_DEVICES"] for _, e in plan] == ["4", "5", "6"]
    assert plan[0][0][1:3] == ["-m", "symmetry_amd.cli"]
    with pytest.raises(ValueError):
        replica_plan({"apiProvider": "native", "tensorParallelSize": 2}, "p.yaml", 2, visible="0,1,2")


def test_two_replicas_register_and_serve(tmp_path):
    async def main():
        ds = DiscoveryServer()
        await ds.start()
        server = SymmetryServer(bootstrap=[ds.address], ping_interval=0.2)
        await server.start()
        ollama = MockOllama()
        port = await ollama.start()
        cfg = _cfg(tmp_path, server.server_key, apiPort=port, name="node")
        env = {k: v for k, v in os.environ.items() if not k.startswith("SYMMETRY_")}
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        host, p = ds.address
        launcher = subprocess.Popen([sys.executable, "-m", "symmetry_amd.cli", "-c", cfg, "--replicas", "2",
                                     "--bootstrap", f"{host}:{p}"], env=env, cwd=ROOT)
        try:
            for _ in range(600):
                names = sorted(j.get("name") for j in server.joins)
                if len(set(names)) >= 2:
                    break
                await asyncio.sleep(0.05)
            assert sorted(set(j.get("name") for j in server.joins)) == ["node-0", "node-1"]
            keys = {j["discoveryKey"] for j in server.joins}
            assert len(keys) == 2  # two identities, two topics
            for key in keys:
                c = SymmetryClient([ds.address], server.server_key)
                await c.start()
                try:
                    conn = await c.connect_provider(key)
                    r = await c.chat(conn, [{"role": "user", "content": "replica"}])
                    assert r.ended and r.text == "Echo from mock ollama: replica"
                finally:
                    await c.stop()
        finally:
            launcher.send_signal(signal.SIGINT)
            try:
                launcher.wait(timeout=30)
            except subprocess.TimeoutExpired:
                launcher.kill()
                launcher.wait()
            await server.stop()
            await ollama.stop()
            await ds.stop()

    asyncio.run(asyncio.wait_for(main(), 90))
