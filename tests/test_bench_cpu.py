"""bench.py contract (driver-facing): one JSON line from rank 0 with the BASELINE metric, the per-client value,
max-over-ranks timing; single process, a 2-rank torchrun in the default tensor-parallel mode (one provider
over both ranks, strong scaling) and in data-parallel mode (gloo on CPU, tiny model)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "tiny-llama", "--steps", "3", "--warmup", "1", "--clients", "2", "--prompt-len", "32",
        "--max-model-len", "128", "--client-tokens", "8"]


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


def _check(r, n, mode):
    assert r["metric"].startswith("streamed tokens/sec + p50 TTFT per client")
    assert r["n_gpus"] == n and r["steps"] == 3 and r["warmup"] == 1
    assert r["higher_is_better"] is True and r["dtype"] == "bf16"
    assert r["scaling"] == ("strong" if mode == "tp" and n > 1 else "weak")
    clients = 2 * n if mode == "dp" else 2
    assert r["config"]["parallelism"] == f"{mode}{n}" and r["config"]["global_batch"] == clients
    assert r["value"] > 0 and r["ms_per_step"] > 0
    assert 0 < r["engine_mean_ttft_ms"] <= r["engine_max_ttft_ms"]
    assert r["engine_p50_ttft_ms"] <= r["engine_max_ttft_ms"]
    # engine-side whole-job aggregate = clients * (1000 / ms_per_step); per client = 1000 / ms_per_step
    assert abs(r["aggregate_tokens_per_s"] - clients * 1e3 / r["ms_per_step"]) / r["aggregate_tokens_per_s"] < 0.01
    assert abs(r["engine_per_client_tokens_per_s"] - 1e3 / r["ms_per_step"]) < 0.01 * r["engine_per_client_tokens_per_s"]
    assert len(r["per_rank_ms_per_step"]) == n and max(r["per_rank_ms_per_step"]) == r["ms_per_step"]
    # the client-end run: every client streamed over the swarm and got its inferenceEnded; its per-client
    # socket-measured median is the headline value (the metric's unit)
    ce = r["client_end"]
    assert ce["all_ended"] and ce["clients"] == 2 and ce["p50_ttft_ms"] > 0, ce
    assert r["p50_ttft_ms"] == ce["p50_ttft_ms"] and r["client_end_per_client_tokens_per_s"] > 0
    assert r["unit"] == "tokens/s per client" and r["value"] == ce["per_client_tokens_per_s_median"]
    assert r["value_source"].startswith("client_end")
    # every token the first two clients were streamed agrees with the fp32 oracle of the same weights (under TP the
    # oracle runs sharded over the ranks and sums / gathers like the engine)
    v = r["verified"]
    assert v["clients"] == 2 and v["tokens"] >= 2 * 3 and v["mismatches"] == 0, v


def test_bench_single_process():
    _check(_run([sys.executable, "bench.py", "--gpus", "1"] + ARGS), 1, "dp")


def test_bench_torchrun_two_ranks_tp():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2"] + ARGS
    _check(_run(cmd), 2, "tp")


def test_bench_torchrun_two_ranks_dp():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--parallel", "dp"] + ARGS
    _check(_run(cmd), 2, "dp")


def test_bench_plain_gpus_two_launches_its_ranks_tp():
    """``python bench.py --gpus 2`` with no launcher starts its own 2-rank torchrun child (the driver's BENCH
    form must not silently time one GPU)."""
    _check(_run([sys.executable, "bench.py", "--gpus", "2"] + ARGS), 2, "tp")


def test_bench_plain_gpus_two_launches_its_ranks_dp():
    _check(_run([sys.executable, "bench.py", "--gpus", "2", "--parallel", "dp"] + ARGS), 2, "dp")


def test_bench_world_size_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2"] + ARGS, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert "error" in line and line["value"] is None and line["n_gpus"] == 2


def test_bench_too_few_gpus_is_an_error(monkeypatch, capsys):
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv(bench.SHARED_GPU_ENV, raising=False)
    monkeypatch.setattr(bench, "visible_gpus", lambda: 1)
    args = type("A", (), {"gpus": 8, "steps": 3, "warmup": 1})()
    assert bench._self_launch(args) == 2
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert "8 GPUs, 1 visible" in line["error"] and line["value"] is None
    plan = bench.launch_plan(["--gpus", "8"], 8, 29555)
    assert "--nproc-per-node=8" in plan and "--master-addr" in plan and "127.0.0.1" in plan


def test_ep_rehearsal_reports_bytes_per_mode():
    """bench/ep_rehearsal.py (the EP operating-point sweep) on gloo with tiny-mixtral: one JSON line per prompt total
    and mode; the owner exchange pushes fewer bytes per layer than the fp32 all-reduce combine at world 2."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = {}
    for mode in ("a2a", "allreduce"):
        p = subprocess.run([sys.executable, "bench/ep_rehearsal.py", "--world", "2", "--mode", mode, "--model",
                            "tiny-mixtral", "--tokens", "256", "--reps", "1", "--device", "cpu", "--kv-blocks", "64"],
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-3000:]
        rows = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(rows) == 1 and rows[0]["mode"] == mode and rows[0]["tokens"] == 256, rows
        out[mode] = rows[0]
    assert out["a2a"]["moe_calls"]["a2a"] > 0 and out["allreduce"]["moe_calls"]["allreduce"] > 0
    d = 256  # tiny-mixtral hidden size
    assert out["allreduce"]["bytes_per_layer_rank0"] == 2 * (2 - 1) * 256 * d * 4 // 2
    assert 0 < out["a2a"]["bytes_per_layer_rank0"] < out["allreduce"]["bytes_per_layer_rank0"]
