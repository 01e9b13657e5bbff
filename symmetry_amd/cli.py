"""Command-line entry points.

``symmetry-cli [-c, --config <path>]`` (REF ``src/symmetry.ts:1-23``): default
config ``~/.config/symmetry/provider.yaml``, ``--version`` prints ``1.0.0``
(the reference's own string, ``src/symmetry.ts:11``).  Added flags:
``--bootstrap host:port`` (discovery nodes; also ``bootstrap:`` in the YAML),
``--init`` (write the install script's default provider.yaml).

Multi-GPU native providers (``tensorParallelSize > 1``) run one process per
GPU: plain ``symmetry-cli -c provider.yaml`` checks the visible GPUs and
starts them as one ``torchrun`` child (or launch ``torchrun --nproc-per-node 8
-m symmetry_amd.cli -c provider.yaml`` yourself): rank 0 runs the provider
node and the scheduler, the other ranks mirror its forward passes (SURVEY.md
§3.6).  A mismatch fails at start-up, before the provider announces itself.

Data-parallel replicas on one node (SURVEY.md §2.5 "one provider process per
GPU group"): ``symmetry-cli -c provider.yaml --replicas N`` (or ``replicas: N``
in the YAML) starts N independent providers, replica i on GPUs
[i*tp, (i+1)*tp) (``tp = tensorParallelSize``; each replica a ``torchrun``
group when tp > 1), named ``<name>-<i>`` so each has its own identity and
topic; the server spreads clients over them like over any set of providers.
8 GPUs: ``--replicas 8`` for Llama-3-8B, ``tensorParallelSize: 8`` for 70B,
``--replicas 2`` + ``tensorParallelSize: 4`` in between.

Also: ``symmetry-server`` (registry/assignment server), ``symmetry-dht``
(discovery node), ``symmetry-client`` (a chat client over the swarm).
"""
from __future__ import annotations

import argparse
import asyncio
import getpass
import json
import os
import sys

from .config import DEFAULT_CONFIG_PATH, ConfigManager, default_config_text

VERSION = "1.0.0"


def _init_config(path: str, native: bool) -> int:
    d = os.path.dirname(path)
    os.makedirs(d, exist_ok=True)
    if os.path.exists(path):
        print(f"provider.yaml already exists at {path}")
        return 0
    try:
        user = getpass.getuser()
    except Exception:
        user = "provider"
    with open(path, "w") as f:
        f.write(default_config_text(user, d, native=native))
    print(f"provider.yaml created successfully at {path}")
    return 0


async def _run_provider(cfg: ConfigManager, bootstrap, engine=None) -> int:
    from .backends.native import NativeBackend
    from .provider.node import SymmetryProvider

    backend = NativeBackend(cfg.get_all(), engine=engine) if engine is not None else None
    prov = SymmetryProvider(cfg, backend=backend, bootstrap=bootstrap, install_signal_handlers=True)
    await prov.init()
    await prov.wait_closed()
    return prov.exit_code


def _distributed_engine(cfg: ConfigManager):
    """torchrun launch: build this rank's TP shard; rank 0 returns the engine, others serve forever."""
    from .engine.llm_engine import EngineConfig
    from .parallel.launch import init_tp_engine

    tp = int(cfg.get("tensorParallelSize") or 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if tp > 1 and tp != world:
        raise SystemExit(f"Error: tensorParallelSize {tp} but the launcher started {world} ranks")
    ecfg = EngineConfig.from_provider(cfg.get_all())
    engine, rank = init_tp_engine(ecfg)
    _exit_when_orphaned()
    if rank != 0:
        try:
            engine.runner.worker_loop()  # reports a failure to rank 0 over the metadata ring before raising
        except BaseException:
            import traceback

            traceback.print_exc()
            _hard_exit(1)
        sys.exit(0)
    return engine


def _hard_exit(code: int) -> None:
    """Leave without interpreter teardown: the process-group / communicator destructors can block forever on a
    peer that is gone (fault containment: the supervisor restarts the ranks)."""
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


def _exit_when_orphaned(period_s: float = 1.0) -> None:
    """A torchrun rank whose launcher (the elastic agent) is gone leaves at once: its peers are gone too, so
    worker ranks would block in the metadata broadcast and rank 0's shutdown in its stop broadcast forever."""
    import threading
    import time

    parent = os.getppid()

    def watch():
        while True:
            time.sleep(period_s)
            if os.getppid() != parent:
                os._exit(0)

    threading.Thread(target=watch, name="symmetry-orphan-watch", daemon=True).start()


REPLICA_ENV = "SYMMETRY_REPLICA_INDEX"


def replica_plan(cfg: dict, config_path: str, replicas: int, bootstrap: str | None = None,
                 visible: str | None = None, port_base: int = 29600) -> list[tuple[list, dict]]:
    """(argv, env overrides) of every replica process: its own name (identity, topic), listen / local HTTP
    port and metrics file, and its GPUs as HIP_VISIBLE_DEVICES (a slice of ``visible`` when the launcher
    itself was restricted)."""
    tp = int(cfg.get("tensorParallelSize") or 1)
    devs = [d.strip() for d in visible.split(",")] if visible else [str(d) for d in range(replicas * tp)]
    if len(devs) < replicas * tp:
        raise ValueError(f"{replicas} replicas x tensorParallelSize {tp} need {replicas * tp} GPUs, "
                         f"{len(devs)} visible")
    base = [sys.executable, "-m", "symmetry_amd.cli", "-c", config_path]
    if bootstrap:
        base += ["--bootstrap", bootstrap]
    plan = []
    for i in range(replicas):
        env = {REPLICA_ENV: str(i), "SYMMETRY_NAME": f"{cfg.get('name') or 'provider'}-{i}"}
        if cfg.get("listenPort"):
            env["SYMMETRY_LISTENPORT"] = str(int(cfg["listenPort"]) + i)
        if cfg.get("serveHttp"):
            env["SYMMETRY_APIPORT"] = str(int(cfg["apiPort"]) + i)
        if cfg.get("metricsFile"):
            root, ext = os.path.splitext(str(cfg["metricsFile"]))
            env["SYMMETRY_METRICSFILE"] = f"{root}-{i}{ext}"
        if str(cfg.get("apiProvider", "")).lower() == "native":
            env["HIP_VISIBLE_DEVICES"] = ",".join(devs[i * tp:(i + 1) * tp])
        argv = base
        if tp > 1:
            argv = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={tp}",
                    "--master-addr", "127.0.0.1", f"--master-port={port_base + i}", "-m", "symmetry_amd.cli",
                    *base[3:]]
        plan.append((argv, env))
    return plan


def _launch_replicas(cfg: ConfigManager, config_path: str, replicas: int, bootstrap: str | None) -> int:
    """Run the replica providers as child processes (never an exec of this process) until they exit or
    the launcher is interrupted; then stop exactly those children."""
    import signal
    import subprocess

    visible = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if visible is None and cfg.is_native and str(cfg.get("device", "auto")) != "cpu":
        import torch  # device_count() does not initialise the GPU runtime on this stack

        n = torch.cuda.device_count()
        if n:
            visible = ",".join(str(d) for d in range(n))
    plan = replica_plan(cfg.get_all(), config_path, replicas, bootstrap, visible)
    procs = [subprocess.Popen(argv, env={**os.environ, **env}) for argv, env in plan]

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGINT)

    signal.signal(signal.SIGTERM, stop)
    try:
        codes = [p.wait() for p in procs]
    except KeyboardInterrupt:
        stop()
        codes = []
        for p in procs:
            try:
                codes.append(p.wait(timeout=30))
            except subprocess.TimeoutExpired:
                p.kill()
                codes.append(p.wait())
    return max((abs(c) for c in codes), default=0)


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def tp_launch_plan(cfg: dict, config_path: str, bootstrap: str | None, port: int | None = None) -> list:
    """argv of the torchrun child that runs a ``tensorParallelSize > 1`` provider started as a plain
    ``symmetry-cli`` (one rank per GPU; rank 0 announces itself only once every shard is built)."""
    tp = int(cfg.get("tensorParallelSize") or 1)
    argv = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={tp}",
            "--master-addr", "127.0.0.1", f"--master-port={port or _free_port()}", "-m", "symmetry_amd.cli",
            "-c", config_path]
    if bootstrap:
        argv += ["--bootstrap", bootstrap]
    return argv


def _launch_tp(cfg: ConfigManager, config_path: str, bootstrap: str | None) -> int:
    """``tensorParallelSize > 1`` outside torchrun: check the GPUs at start-up (the reference validates its
    config before it goes online, ``src/config.ts:19-45``), then run the ranks as ONE torchrun child --
    started before this process touches the GPU, never an exec -- and exit with its code."""
    import subprocess

    tp = int(cfg.get("tensorParallelSize") or 1)
    if str(cfg.get("device", "auto")) != "cpu":
        import torch  # device_count() does not initialise the GPU runtime on this stack

        n = torch.cuda.device_count()
        if n < tp:
            print(f"Error: tensorParallelSize {tp} needs {tp} GPUs, {n} visible", file=sys.stderr)
            return 1
    p = subprocess.Popen(tp_launch_plan(cfg.get_all(), config_path, bootstrap))
    try:
        return abs(p.wait())
    except KeyboardInterrupt:
        import signal

        p.send_signal(signal.SIGINT)
        try:
            return abs(p.wait(timeout=30))
        except subprocess.TimeoutExpired:
            p.kill()
            return abs(p.wait())


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="symmetry-cli", description="symmetry cli")
    ap.add_argument("-c", "--config", default=DEFAULT_CONFIG_PATH, help="Path to config file")
    ap.add_argument("-V", "--version", action="version", version=VERSION)
    ap.add_argument("--bootstrap", default=None, help="discovery node(s) host:port[,host:port]")
    ap.add_argument("--init", action="store_true", help="write a default provider.yaml and exit")
    ap.add_argument("--native", action="store_true", help="with --init: apiProvider native")
    ap.add_argument("--replicas", type=int, default=None,
                    help="data-parallel providers on this node, one per GPU group of tensorParallelSize GPUs")
    args = ap.parse_args(argv)
    if args.init:
        return _init_config(args.config, args.native)
    try:
        cfg = ConfigManager(args.config)
    except Exception as exc:
        print(f"Error: {exc}", file=sys.stderr)
        return 1
    replicas = int(args.replicas or cfg.get("replicas") or 1)
    if replicas > 1 and REPLICA_ENV not in os.environ:
        return _launch_replicas(cfg, args.config, replicas, args.bootstrap)
    engine = None
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and cfg.is_native and int(cfg.get("tensorParallelSize") or 1) > 1:
        return _launch_tp(cfg, args.config, args.bootstrap)
    if world > 1 and cfg.is_native:
        engine = _distributed_engine(cfg)
    code = 0
    try:
        code = asyncio.run(_run_provider(cfg, args.bootstrap, engine)) or 0
    except KeyboardInterrupt:
        pass
    if engine is not None and (code or engine.fatal is not None):
        _hard_exit(code or 1)  # a TP peer is gone: do not wait on its collectives / process group at teardown
    return code


def server_main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="symmetry-server")
    ap.add_argument("--bootstrap", default="127.0.0.1:49737")
    ap.add_argument("--seed-hex", default=None, help="32-byte hex seed of the server identity")
    args = ap.parse_args(argv)

    async def run():
        from .provider.node import parse_bootstrap
        from .testing.mock_server import SymmetryServer

        srv = SymmetryServer(seed=bytes.fromhex(args.seed_hex) if args.seed_hex else None,
                             bootstrap=parse_bootstrap(args.bootstrap))
        await srv.start()
        print(f"symmetry server key: {srv.server_key}", flush=True)
        await asyncio.Event().wait()

    try:
        asyncio.run(run())
    except KeyboardInterrupt:
        pass
    return 0


def client_main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="symmetry-client")
    ap.add_argument("--bootstrap", default="127.0.0.1:49737")
    ap.add_argument("--server-key", required=True)
    ap.add_argument("--model", default="llama3:8b")
    ap.add_argument("--prompt", default="Hello!")
    ap.add_argument("--max-tokens", type=int, default=None)
    args = ap.parse_args(argv)

    async def run():
        from .provider.node import parse_bootstrap
        from .testing.mock_client import SymmetryClient

        cl = SymmetryClient(parse_bootstrap(args.bootstrap), args.server_key)
        await cl.start()
        det = await cl.request_provider(args.model)
        if "discoveryKey" not in det:
            print(json.dumps(det))
            return
        conn = await cl.connect_provider(det["discoveryKey"])
        extra = {"max_tokens": args.max_tokens} if args.max_tokens else None
        res = await cl.chat(conn, [{"role": "user", "content": args.prompt}], extra=extra)
        print(res.text)
        print(json.dumps({"ttft_ms": None if res.ttft_s is None else res.ttft_s * 1e3,
                          "tokens_per_s": res.tokens_per_s, "events": res.content_events}), file=sys.stderr)
        await cl.stop()

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
