#!/bin/bash
# 10-client decode kernel profile (1 GPU) + TP shard timings at TP = 2 / 4 / 8 (XAR on) and 70B TP = 8.
set -o pipefail
TAG=d10 bash tools/prof_bench.sh && head -12 gpurun_out/prof_d10.csv || exit $?
for tp in 2 4 8; do
  timeout -k 10 200 python -u bench/tp_shard.py --tp $tp --clients 10 > gpurun_out/tp_shard_$tp.json 2> gpurun_out/tp_shard_$tp.err
  rc=$?; tail -1 gpurun_out/tp_shard_$tp.json | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench/tp_shard.py --tp 8 --clients 4 --model llama3:70b > gpurun_out/tp_shard_70b.json 2> gpurun_out/tp_shard_70b.err
rc=$?; tail -1 gpurun_out/tp_shard_70b.json | cut -c1-120; exit $rc
