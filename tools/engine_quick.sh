#!/bin/bash
# Decode-step engine quick loop on one GPU: correctness (tests/test_decode_engine_gpu.py), the phase timeline from
# in-kernel stamps (bench/kernels/bench_engine.py), then the TP-shard step time with / without the engine
# (bench/tp_shard.py).  Output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/engine_tp_shard.jsonl
timeout -k 10 300 python -u -m pytest tests/test_decode_engine_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/engine_tests.log 2>&1
rc=$?; tail -4 gpurun_out/engine_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/kernels/bench_engine.py --tp 8 > gpurun_out/engine_stamps.jsonl \
  2> gpurun_out/bench_engine.err || exit $?
tail -c 1500 gpurun_out/engine_stamps.jsonl
for cfg in "llama3:8b 1 10 0" "llama3:8b 1 10 1" "llama3:8b 2 10 1" "llama3:8b 8 10 0" "llama3:8b 8 10 1" "llama3:8b 4 10 0" "llama3:8b 4 10 1" "llama3:70b 8 4 0" \
           "llama3:70b 8 4 1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench/tp_shard.py --model $1 --tp $2 --clients $3 --engine $4 \
    >> gpurun_out/engine_tp_shard.jsonl 2> gpurun_out/tp_shard.err || exit $?
done
grep '^{' gpurun_out/engine_tp_shard.jsonl | cut -c1-160
