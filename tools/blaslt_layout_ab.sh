#!/bin/bash
# hipBLASLt prefill projections: weights as [N][K] (TN, today) vs transposed [K][N] (NN), heuristic pick and the
# best of up to MAXA supported solutions per shape at each of MS rows -> gpurun_out/blaslt_layout.jsonl
set -o pipefail
mkdir -p gpurun_out
for m in ${MS:-768}; do
  for lay in tn nn; do
    for sh in ${SHAPES:-gate_up down qkv o}; do
      timeout -k 10 240 bench/kernels/blaslt_algos ${MAXA:-300} $sh $m ${OUT:-bf16} $lay >> gpurun_out/blaslt_layout.jsonl \
        2>> gpurun_out/blaslt_layout.err || exit $?
    done
  done
done
