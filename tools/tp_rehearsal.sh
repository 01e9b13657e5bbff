#!/bin/bash
# TP=2 two-process rehearsal on one GPU (bench.py --gpus 2, host-staged gloo + xGMI kernels + decode graphs):
# step times, per-rank times and rank 0's host-phase breakdown (timed steps and client-end run).
set -o pipefail
bash tools/gpu_suite.sh tp > gpurun_out/tp2_rehearsal.txt 2>&1
rc=$?
grep '^{' gpurun_out/bench_tp2.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); ce=d['client_end']
print(json.dumps({k: d[k] for k in ('value','ms_per_step','per_rank_ms_per_step','host_ms_per_step','p50_ttft_ms')}))
print(json.dumps({'step_phase_ms': ce['engine']['step_phase_ms'], 'runner_host_ms_per_step': ce.get('runner_host_ms_per_step')}))"
exit $rc
