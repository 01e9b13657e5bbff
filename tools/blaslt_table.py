"""Turn a `tools/blaslt_tune.sh` sweep (JSON lines) into the runtime table `symmetry_amd/ops/blaslt_table.json`.

    python tools/blaslt_table.py gpurun_out/blaslt_tune.jsonl [--min-gain 0.03]

Keeps, per "N,K" projection, the M rows whose best solution beats the library heuristic by >= min-gain (others
map to -1: the heuristic); `ops.linear` picks the entry nearest to a step's M.
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("sweep")
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--out", default=os.path.join(ROOT, "symmetry_amd", "ops", "blaslt_table.json"))
    args = ap.parse_args()
    table: dict = {}
    for line in open(args.sweep):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        gain = d["default_us"] / d["us"] - 1 if d["us"] > 0 else 0.0
        key = f'{d["N"]},{d["K"]}'
        table.setdefault(key, {})[str(d["M"])] = {
            "index": d["index"] if gain >= args.min_gain else -1,
            "us": d["us"], "default_us": d["default_us"]}
    with open(args.out, "w") as f:
        json.dump({"note": "hipBLASLt solution per (N,K) projection and M rows; -1 = library heuristic "
                           "(bench/kernels/blaslt_tune.cpp on MI355X, this ROCm build)", "table": table}, f, indent=1)
    print(f"{args.out}: {sum(len(v) for v in table.values())} entries over {len(table)} shapes")


if __name__ == "__main__":
    main()
