#!/bin/bash
# Short-prefill timing (bench/host/prefill_step.py) (graphs on / off) + a rocprofv3 kernel trace of TOKENS-token prefills -> gpurun_out/pf_*
set -o pipefail
tok=${TOKENS:-128}
root=$(pwd)
mkdir -p "$root/gpurun_out"
timeout -k 10 300 python -u bench/host/prefill_step.py --tokens $tok --reps 20 > gpurun_out/pf_time_on.json 2> gpurun_out/pf_time_on.err || exit $?
timeout -k 10 300 python -u bench/host/prefill_step.py --tokens $tok --reps 20 --no-graphs > gpurun_out/pf_time_off.json 2> gpurun_out/pf_time_off.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof_pf -o run -- \
  python3 "$root/bench/host/prefill_step.py" --tokens $tok --reps 10 > "$root/gpurun_out/pf_prof.log" 2>&1 || exit $?
db=$(ls /tmp/prof_pf/*/*.db /tmp/prof_pf/*.db 2>/dev/null | head -1)
cd "$root" && python3 tools/prof_summary.py "$db" "gpurun_out/pf_prof.csv" --last-ms ${LAST_MS:-150} --top 60 > "gpurun_out/pf_prof.txt"
