#!/bin/bash
# xGMI collective tests + TP shard timings (TP 2/4/8 on one GPU) + the TP=2 two-process rehearsal.
# Run on the gpurun box: bash tools/tp_check.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py tests/test_tp_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/tp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tp_tests.log; [ $rc -eq 0 ] || exit $rc
for tp in 2 4 8; do
  timeout -k 10 200 python -u bench/tp_shard.py --tp $tp --clients 10 > gpurun_out/tp_shard_$tp.json 2> gpurun_out/tp_shard_$tp.err
  rc=$?; tail -1 gpurun_out/tp_shard_$tp.json; [ $rc -eq 0 ] || exit $rc
done
TP=8 TAG=tp8 bash tools/prof_tp_shard.sh && head -8 gpurun_out/prof_tp8.csv
