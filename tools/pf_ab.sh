#!/bin/bash
# Short-prefill A/B (bench/host/prefill_step.py, graphs on): each ENV=VAL setting, alternating, for each token count.
# usage: tools/pf_ab.sh "SYMMETRY_MG_GU_WIDE=0" "SYMMETRY_MG_GU_WIDE=1" -- 128 512
set -o pipefail
mkdir -p gpurun_out
arms=()
while [ "$1" != "--" ] && [ -n "$1" ]; do arms+=("$1"); shift; done
shift
for tok in "$@"; do
  for rep in 1 2; do
    for arm in "${arms[@]}"; do
      out=$(env $arm timeout -k 10 300 python -u bench/host/prefill_step.py --tokens $tok --reps 20 2>>gpurun_out/pf_ab.err | grep '^{') || exit 1
      echo "{\"arm\": \"$arm\", \"tokens\": $tok, \"rep\": $rep, \"result\": $out}" | tee -a gpurun_out/pf_ab.jsonl
    done
  done
done
