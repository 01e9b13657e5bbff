set -e
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
