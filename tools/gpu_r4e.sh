set -e
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py tests/test_tp_gpu.py -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python bench/kernels/bench_xgmi.py > $O/bench_xgmi.jsonl 2> $O/bench_xgmi.err
