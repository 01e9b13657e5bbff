#!/bin/bash
# TP=4 rehearsal: bench.py --gpus 4 with four ranks on ONE GPU (host-staged gloo for prefill-sized collectives,
# xGMI one-shot kernels between the four processes for decode-sized ones, decode hipGraphs)
set -o pipefail
mkdir -p gpurun_out
SYMMETRY_TP_COMM=gloo SYMMETRY_XGMI=1 SYMMETRY_XGMI_GRAPHS=1 timeout -k 10 500 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 4 --steps 32 --warmup 4 > gpurun_out/bench_tp4.json 2> gpurun_out/bench_tp4.err
rc=$?
grep '^{' gpurun_out/bench_tp4.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); ce=d['client_end']
print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','per_rank_ms_per_step','host_ms_per_step','p50_ttft_ms','tp')}))
print(json.dumps({'all_ended': ce['all_ended'], 'step_phase_ms': ce['engine']['step_phase_ms']}))"
exit $rc
