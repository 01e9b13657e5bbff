"""Command-line entry points.

``symmetry-cli [-c, --config <path>]`` (REF ``src/symmetry.ts:1-23``): default
config ``~/.config/symmetry/provider.yaml``, ``--version`` prints ``1.0.0``
(the reference's own string, ``src/symmetry.ts:11``).  Added flags:
``--bootstrap host:port`` (discovery nodes; also ``bootstrap:`` in the YAML),
``--init`` (write the install script's default provider.yaml).

Multi-GPU native providers (``tensorParallelSize > 1``) are launched one
process per GPU, e.g. ``torchrun --nproc-per-node 8 -m symmetry_amd.cli -c
provider.yaml``: rank 0 runs the provider node and the scheduler, the other
ranks mirror its forward passes over RCCL.

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


async def _run_provider(cfg: ConfigManager, bootstrap, engine=None) -> None:
    from .backends.native import NativeBackend
    from .provider.node import SymmetryProvider

    backend = NativeBackend(cfg.get_all(), engine=engine) if engine is not None else None
    prov = SymmetryProvider(cfg, backend=backend, bootstrap=bootstrap, install_signal_handlers=True)
    await prov.init()
    await prov.wait_closed()


def _distributed_engine(cfg: ConfigManager):
    """torchrun launch: build this rank's TP shard; rank 0 returns the engine, others serve forever."""
    from .engine.llm_engine import EngineConfig
    from .parallel.launch import init_tp_engine

    ecfg = EngineConfig.from_provider(cfg.get_all())
    engine, rank = init_tp_engine(ecfg)
    if rank != 0:
        engine.runner.worker_loop()
        sys.exit(0)
    return engine


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="symmetry-cli", description="symmetry cli")
    ap.add_argument("-c", "--config", default=DEFAULT_CONFIG_PATH, help="Path to config file")
    ap.add_argument("-V", "--version", action="version", version=VERSION)
    ap.add_argument("--bootstrap", default=None, help="discovery node(s) host:port[,host:port]")
    ap.add_argument("--init", action="store_true", help="write a default provider.yaml and exit")
    ap.add_argument("--native", action="store_true", help="with --init: apiProvider native")
    args = ap.parse_args(argv)
    if args.init:
        return _init_config(args.config, args.native)
    try:
        cfg = ConfigManager(args.config)
    except Exception as exc:
        print(f"Error: {exc}", file=sys.stderr)
        return 1
    engine = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and cfg.is_native:
        engine = _distributed_engine(cfg)
    try:
        asyncio.run(_run_provider(cfg, args.bootstrap, engine))
    except KeyboardInterrupt:
        pass
    return 0


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
