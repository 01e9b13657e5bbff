#!/bin/bash
# GPU check used during development: GPU tests, the 1-GPU bench, and a 2-rank TP rehearsal on one GPU
# (host-staged gloo communicator + the xGMI kernels between two processes + decode hipGraphs).
# Usage (on the gpurun box): bash tools/gpu_suite.sh [tests|bench|tp|all]...
set -o pipefail
mkdir -p gpurun_out
what="${*:-all}"
run_tests() {
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputests.log 2>&1
  local rc=$?; tail -3 gpurun_out/gputests.log; return $rc
}
run_bench() {
  timeout -k 10 300 python -u bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
  local rc=$?; cat gpurun_out/bench1.json; return $rc
}
run_tp() {
  SYMMETRY_TP_COMM=gloo SYMMETRY_XGMI=1 SYMMETRY_XGMI_GRAPHS=1 timeout -k 10 400 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 2 --steps 32 --warmup 4 > gpurun_out/bench_tp2.json 2> gpurun_out/bench_tp2.err
  local rc=$?; cat gpurun_out/bench_tp2.json; return $rc
}
for w in $what; do
  case $w in
    tests) run_tests || exit $? ;;
    bench) run_bench || exit $? ;;
    tp) run_tp || exit $? ;;
    all) run_tests && run_bench && run_tp || exit $? ;;
  esac
done
