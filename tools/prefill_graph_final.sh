#!/bin/bash
# Prefill graphs captured at start-up: GPU test, multi-turn TTFT on/off, config 2 e2e on -> gpurun_out/pgf_*
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  -k "prefill_graphs or llama3_8b_shapes or prefix_cache" > gpurun_out/pgf_tests.log 2>&1 || exit $?
bash tools/multiturn_pg_ab.sh || exit $?
timeout -k 10 240 python -u bench/e2e.py --model llama3:8b --clients 1 > gpurun_out/pgf_c2.json 2> gpurun_out/pgf_c2.err || exit $?
