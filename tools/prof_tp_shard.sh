#!/bin/bash
# rocprofv3 kernel trace of one TP rank's decode shard on one GPU (bench/tp_shard.py) -> per-kernel CSV.
#   TP=8 TAG=tp8 bash tools/prof_tp_shard.sh
set -o pipefail
tag=${TAG:-tp${TP:-8}}
root=$(pwd)
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof_$tag -o run -- \
  python3 "$root/bench/tp_shard.py" --tp ${TP:-8} --clients ${CLIENTS:-10} --model ${MODEL:-llama3:8b} > "$root/gpurun_out/prof_$tag.log" 2>&1 || exit $?
db=$(ls /tmp/prof_$tag/*/*.db /tmp/prof_$tag/*.db 2>/dev/null | head -1)
cd "$root" && python3 tools/prof_summary.py "$db" "gpurun_out/prof_$tag.csv" --last-ms ${LAST_MS:-30} > "gpurun_out/prof_$tag.txt"
