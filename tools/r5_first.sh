set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit $?
cat gpurun_out/bench1.json
SYMMETRY_BENCH_SHARED_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 32 --warmup 4 > gpurun_out/bench_tp2_plain.json 2> gpurun_out/bench_tp2_plain.err || exit $?
cat gpurun_out/bench_tp2_plain.json
