"""Alternating A/B runs of bench.py (run on the GPU box; each arm is its own child process).

usage: python tools/ab_bench.py OUT.jsonl --reps 3 --arm NAME 'ENV=V ...' 'bench args' [--arm ...]

Arms run interleaved (A B A B ...) so drift hits both; every run appends one JSON line
{"arm", "rep", "env", "args", "result"} and the script ends with a summary line per arm
(mean / min / max of ms_per_step and p50 TTFT).  A run that fails or times out stops the script
(no retries: a failing GPU step is read, not repeated).
"""
from __future__ import annotations

import json
import os
import shlex
import statistics
import subprocess
import sys


def main() -> int:
    argv = sys.argv[1:]
    out = argv.pop(0)
    reps, timeout = 3, 240
    arms = []
    while argv:
        a = argv.pop(0)
        if a == "--reps":
            reps = int(argv.pop(0))
        elif a == "--timeout":
            timeout = int(argv.pop(0))
        elif a == "--arm":
            arms.append((argv.pop(0), argv.pop(0), argv.pop(0)))
        else:
            raise SystemExit(f"unknown argument {a}")
    res = {name: [] for name, _, _ in arms}
    with open(out, "a") as f:
        for rep in range(reps):
            for name, env_s, args_s in arms:
                env = dict(os.environ)
                for kv in shlex.split(env_s):
                    k, v = kv.split("=", 1)
                    env[k] = v
                cmd = ["timeout", "-k", "10", str(timeout), sys.executable, "bench.py"] + shlex.split(args_s)
                p = subprocess.run(cmd, env=env, capture_output=True, text=True)
                line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
                if p.returncode != 0 or not line:
                    sys.stderr.write(p.stderr[-4000:])
                    f.write(json.dumps({"arm": name, "rep": rep, "env": env_s, "args": args_s,
                                        "rc": p.returncode}) + "\n")
                    return 1
                r = json.loads(line[-1])
                res[name].append(r)
                f.write(json.dumps({"arm": name, "rep": rep, "env": env_s, "args": args_s, "result": r}) + "\n")
                f.flush()
                print(name, rep, r["ms_per_step"], r["p50_ttft_ms"], flush=True)
        for name, env_s, args_s in arms:
            ms = [r["ms_per_step"] for r in res[name]]
            tt = [r["p50_ttft_ms"] for r in res[name]]
            summ = {"arm": name, "env": env_s, "args": args_s, "summary": {
                "ms_per_step_mean": round(statistics.mean(ms), 4), "ms_per_step_min": min(ms),
                "ms_per_step_max": max(ms), "p50_ttft_mean": round(statistics.mean(tt), 2),
                "p50_ttft_min": min(tt), "p50_ttft_max": max(tt), "n": len(ms)}}
            f.write(json.dumps(summ) + "\n")
            print(json.dumps(summ), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
