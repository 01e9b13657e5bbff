#!/bin/bash
# rocprofv3 kernel trace of one TP-shard decode run (bench/tp_shard.py) with the per-layer launches and with the
# decode-step engine; per-kernel stats CSVs under gpurun_out/prof_tp_shard_e{0,1}/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODEL=${1:-llama3:8b}
TP=${2:-8}
C=${3:-10}
for e in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tp_shard_e$e -o run -- \
    python3 bench/tp_shard.py --model $MODEL --tp $TP --clients $C --engine $e --steps 32 --warmup 4 \
    > gpurun_out/prof_tp_shard_e$e.log 2>&1 || exit $?
  grep '^{' gpurun_out/prof_tp_shard_e$e.log | cut -c1-200
done
