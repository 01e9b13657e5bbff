#!/bin/bash
# rocprofv3 kernel trace of the bench's first prefill step (C prompts of L tokens in one step) ->
# per-kernel CSV of the final LAST_MS of the trace (the last rep's step).
#   TAG=name [MODEL=llama3:8b] CLIENTS=6 PLEN=128 [LAST_MS=16] bash tools/prof_prefill.sh
set -o pipefail
tag=${TAG:-prefill}
root=$(pwd)
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof_$tag -o run -- \
  python3 "$root/bench/prefill.py" --model ${MODEL:-llama3:8b} --clients ${CLIENTS:-6} --prompt-len ${PLEN:-128} --reps 3 \
  > "$root/gpurun_out/prof_$tag.log" 2>&1 || exit $?
db=$(ls /tmp/prof_$tag/*/*.db /tmp/prof_$tag/*.db 2>/dev/null | head -1)
cd "$root" && python3 tools/prof_summary.py "$db" "gpurun_out/prof_$tag.csv" --last-ms ${LAST_MS:-16} \
  > "gpurun_out/prof_$tag.txt"
