#!/bin/bash
# Prefill hipGraph buckets: GPU tests, then config 2 (one client, Llama-3-8B, e2e over the swarm) with the
# buckets on / off -> gpurun_out/pg_*.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  -k "prefill_graphs or llama3_8b_shapes or top_k_one or staggered or prefix_cache" > gpurun_out/pg_tests.log 2>&1 || exit $?
timeout -k 10 240 python -u bench/e2e.py --model llama3:8b --clients 1 > gpurun_out/pg_c2_on.json 2> gpurun_out/pg_c2_on.err || exit $?
SYMMETRY_PREFILL_GRAPH_TOKENS=0 timeout -k 10 240 python -u bench/e2e.py --model llama3:8b --clients 1 \
  > gpurun_out/pg_c2_off.json 2> gpurun_out/pg_c2_off.err || exit $?
