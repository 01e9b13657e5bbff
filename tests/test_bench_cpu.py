"""bench.py contract (driver-facing): one JSON line from rank 0 with the BASELINE metric, whole-job value,
max-over-ranks timing; single process and a 2-rank torchrun (gloo on CPU, tiny model)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "tiny-llama", "--steps", "3", "--warmup", "1", "--clients", "2", "--prompt-len", "16",
        "--max-model-len", "128"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _check(r, n):
    assert r["metric"].startswith("streamed tokens/sec + p50 TTFT per client")
    assert r["n_gpus"] == n and r["steps"] == 3 and r["warmup"] == 1
    assert r["higher_is_better"] is True and r["scaling"] == "weak" and r["dtype"] == "bf16"
    assert r["config"]["parallelism"] == f"dp{n}" and r["config"]["global_batch"] == 2 * n
    assert r["value"] > 0 and r["ms_per_step"] > 0 and r["p50_ttft_ms"] > 0
    assert 0 < r["mean_ttft_ms"] <= r["max_ttft_ms"] and r["p50_ttft_ms"] <= r["max_ttft_ms"]
    # whole-job aggregate = world * clients * (1000 / ms_per_step)
    assert abs(r["value"] - n * 2 * 1e3 / r["ms_per_step"]) / r["value"] < 0.01


def test_bench_single_process():
    _check(_run([sys.executable, "bench.py", "--gpus", "1"] + ARGS), 1)


def test_bench_torchrun_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2"] + ARGS
    _check(_run(cmd), 2)
