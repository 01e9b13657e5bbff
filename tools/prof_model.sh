#!/bin/bash
# rocprofv3 kernel trace of a steady-state bench.py decode window for MODEL / CLIENTS -> gpurun_out/prof_$TAG.csv
set -o pipefail
tag=${TAG:-model}
root=$(pwd)
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof_$tag -o run -- \
  python3 "$root/bench.py" --model ${MODEL:-llama3:8b} --clients ${CLIENTS:-4} --steps 24 --warmup 4 --client-end 0 \
  --max-model-len 1024 --profile-steps 8 --verify-clients 0 > "$root/gpurun_out/prof_$tag.log" 2>&1 || exit $?
db=$(ls /tmp/prof_$tag/*/*.db /tmp/prof_$tag/*.db 2>/dev/null | head -1)
cd "$root" && python3 tools/prof_summary.py "$db" "gpurun_out/prof_$tag.csv" --last-ms ${LAST_MS:-60} > "gpurun_out/prof_$tag.txt"
