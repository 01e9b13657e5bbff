set -e
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_xgmi.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 180 --timeout-method thread > $O/pytest_tp.log 2>&1
