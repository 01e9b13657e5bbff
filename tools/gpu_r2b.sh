set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b/pytest.log 2>&1
timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/r2b/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b/prof -o run -- python3 bench.py --steps 32 --warmup 8 > gpurun_out/r2b/prof.log 2>&1
