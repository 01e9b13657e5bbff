set -e
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
SYMMETRY_ATTN_PREFETCH=512 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 180 --timeout-method thread > $O/pytest_engine_pf.log 2>&1
timeout -k 10 900 python tools/ab_bench.py $O/ab_prefetch.jsonl --reps 3 \
  --arm off 'SYMMETRY_ATTN_PREFETCH=0' '--steps 64 --warmup 8' \
  --arm pf256 'SYMMETRY_ATTN_PREFETCH=256' '--steps 64 --warmup 8' \
  --arm pf512 'SYMMETRY_ATTN_PREFETCH=512' '--steps 64 --warmup 8' \
  --arm pf1024 'SYMMETRY_ATTN_PREFETCH=1024' '--steps 64 --warmup 8' > $O/ab.log 2>&1
