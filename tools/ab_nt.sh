#!/bin/bash
# Non-temporal weight loads in the decode GEMMs (x-resident body now honours them): per-kernel sweep + A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench/kernels/bench_decode_gemm.py --shapes qkv o gate_up down --m 10 \
  --variants 11 111 4 104 --layouts shuf > gpurun_out/nt_kernels.jsonl 2>&1
rc=$?; grep '^{' gpurun_out/nt_kernels.jsonl | cut -c1-140; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/ab_bench.py gpurun_out/nt_ab.jsonl --reps 3 \
  --arm default '' '--client-end 0 --steps 64 --warmup 8 --nt-weights 0' \
  --arm nt '' '--client-end 0 --steps 64 --warmup 8 --nt-weights 1' > gpurun_out/nt_ab.log 2>&1
rc=$?; tail -2 gpurun_out/nt_ab.log; exit $rc
