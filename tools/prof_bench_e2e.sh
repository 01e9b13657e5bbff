#!/bin/bash
# rocprofv3 kernel trace of a whole bench.py run (engine steps + client-end run) -> prefill step spans / gaps
set -o pipefail
root=$(pwd)
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof_e2e -o run -- \
  python3 "$root/bench.py" --steps 16 --warmup 4 > "$root/gpurun_out/prof_e2e.log" 2>&1 || exit $?
db=$(ls /tmp/prof_e2e/*/*.db /tmp/prof_e2e/*.db 2>/dev/null | head -1)
cd "$root" && python3 tools/prefill_gaps.py "$db" --detail ${SERIES:+--series "$SERIES"} > gpurun_out/prefill_gaps.txt
