#!/bin/bash
# Decode-step engine (csrc/kernels/decode_layers.hip): correctness on one GPU, then the TP-shard step times with
# and without it (bench/tp_shard.py: one rank's shard, world-1 collectives), then the 2-process TP=2 rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_engine_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/engine_tests.log 2>&1
rc=$?; tail -6 gpurun_out/engine_tests.log; [ $rc -eq 0 ] || exit $rc
for tp in 8 4; do
  for e in 0 1; do
    timeout -k 10 300 python -u bench/tp_shard.py --tp $tp --clients 10 --engine $e >> gpurun_out/engine_tp_shard.jsonl \
      2> gpurun_out/engine_tp_shard_$tp_$e.err || exit $?
  done
done
grep '^{' gpurun_out/engine_tp_shard.jsonl
timeout -k 10 300 python -u -m pytest tests/test_tp_gpu.py -x -v -k engine --timeout 240 --timeout-method thread \
  > gpurun_out/engine_tp2.log 2>&1
rc=$?; tail -4 gpurun_out/engine_tp2.log; exit $rc
