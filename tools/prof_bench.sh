#!/bin/bash
# rocprofv3 kernel trace of a steady-state bench.py decode window -> per-kernel CSV under gpurun_out/.
#   TAG=name CLIENTS=64 [ENVS="SYMMETRY_MG_FUSED=0"] bash tools/prof_bench.sh
set -o pipefail
tag=${TAG:-prof}
root=$(pwd)
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for kv in $ENVS; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof_$tag -o run -- \
  python3 "$root/bench.py" --clients ${CLIENTS:-10} --steps 48 --warmup 8 --client-end 0 --max-model-len 1024 --verify-clients 0 \
  --profile-steps 16 > "$root/gpurun_out/prof_$tag.log" 2>&1 || exit $?
db=$(ls /tmp/prof_$tag/*/*.db /tmp/prof_$tag/*.db 2>/dev/null | head -1)
cd "$root" && python3 tools/prof_summary.py "$db" "gpurun_out/prof_$tag.csv" --last-ms ${LAST_MS:-40} > "gpurun_out/prof_$tag.txt"
