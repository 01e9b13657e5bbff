"""Alternating A/B runs of a benchmark script (run on the GPU box; each arm is its own child process).

usage: python tools/ab_bench.py OUT.jsonl [--script bench/prefill.py] --reps 3 --arm NAME 'ENV=V ...' 'args' [--arm ...]

The script (default bench.py; e.g. bench/prefill.py, bench/host/prefill_step.py, bench/e2e.py) must print its
result as a JSON line; the last one is kept.  Examples of the single-purpose wrappers this replaces:
  Mixtral w2 streaming:  --script bench/prefill.py --arm tile '' '--model mixtral:8x7b --clients 4'
                         --arm stream 'SYMMETRY_MOE_PRE_ROWS=176' '--model mixtral:8x7b --clients 4'
  prefill GEMM path:     --script bench/prefill.py --arm lib 'SYMMETRY_PGEMM=0' '--clients 6' --arm pg '' '--clients 6'

Arms run interleaved (A B A B ...) so drift hits both; every run appends one JSON line
{"arm", "rep", "env", "args", "result"} and the script ends with a summary line per arm
(mean / min / max of every numeric timing key the script reports: ms_per_step, p50_ttft_ms, ttft_ms).  A run that fails or times out stops the script
(no retries: a failing GPU step is read, not repeated).
"""
from __future__ import annotations

import json
import os
import shlex
import statistics
import subprocess
import sys


KEYS = ("ms_per_step", "p50_ttft_ms", "ttft_ms", "value")


def main() -> int:
    argv = sys.argv[1:]
    out = argv.pop(0)
    reps, timeout, script = 3, 240, "bench.py"
    arms = []
    while argv:
        a = argv.pop(0)
        if a == "--reps":
            reps = int(argv.pop(0))
        elif a == "--timeout":
            timeout = int(argv.pop(0))
        elif a == "--script":
            script = argv.pop(0)
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
                cmd = ["timeout", "-k", "10", str(timeout), sys.executable, script] + shlex.split(args_s)
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
                print(name, rep, {k: r[k] for k in KEYS if k in r}, flush=True)
        for name, env_s, args_s in arms:
            summ = {"arm": name, "env": env_s, "args": args_s, "summary": {"n": len(res[name])}}
            for k in KEYS:
                vals = [r[k] for r in res[name] if isinstance(r.get(k), (int, float))]
                if vals:
                    summ["summary"].update({k + "_mean": round(statistics.mean(vals), 4), k + "_min": min(vals),
                                            k + "_max": max(vals)})
            f.write(json.dumps(summ) + "\n")
            print(json.dumps(summ), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
