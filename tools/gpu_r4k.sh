set -e
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 1000 python tools/ab_bench.py $O/ab_slab_loads.jsonl --reps 3 \
  --arm c64 '' '--clients 64 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm c32 '' '--clients 32 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm c10 '' '--steps 64 --warmup 8' > $O/ab.log 2>&1
