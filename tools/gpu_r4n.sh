set -e
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
SYMMETRY_NORM_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "norm" > $O/pytest.log 2>&1
timeout -k 10 900 python tools/ab_bench.py $O/ab_norm_wide.jsonl --reps 3 \
  --arm nt256 'SYMMETRY_NORM_WIDE=0' '--clients 64 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm nt512 'SYMMETRY_NORM_WIDE=1' '--clients 64 --max-model-len 1024 --steps 48 --warmup 8' > $O/ab.log 2>&1
