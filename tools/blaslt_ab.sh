#!/bin/bash
# Tuned hipBLASLt solutions (SYMMETRY_BLASLT_TUNED=1) vs the library heuristic (0): kernel test, then alternating
# prefill timings -> gpurun_out/blaslt_ab.jsonl
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k blaslt \
  > gpurun_out/blaslt_ab_tests.log 2>&1 || exit $?
for arm in ${ARMS:-1 0}; do
  for cfg in ${CFGS:-10:128 1:2048}; do
    set -- ${cfg/:/ }
    SYMMETRY_BLASLT_TUNED=$arm timeout -k 10 200 python -u bench/prefill.py --clients $1 --prompt-len $2 --reps 5 \
      2>>gpurun_out/blaslt_ab.err | grep '^{' | sed "s/^{/{\"tuned\": $arm, /" >> gpurun_out/blaslt_ab.jsonl || exit $?
  done
  SYMMETRY_BLASLT_TUNED=$arm timeout -k 10 200 python -u bench/host/prefill_step.py --tokens 128 --reps 20 \
    2>>gpurun_out/blaslt_ab.err | grep '^{' | sed "s/^{/{\"tuned\": $arm, /" >> gpurun_out/blaslt_ab.jsonl || exit $?
done
