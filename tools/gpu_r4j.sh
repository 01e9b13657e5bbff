set -e
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 180 --timeout-method thread -k "rope or general_rows or wide" > $O/pytest.log 2>&1
timeout -k 10 1000 python tools/ab_bench.py $O/ab_rope_rows.jsonl --reps 3 \
  --arm grouped 'SYMMETRY_ROPE_DECODE_ROWS=0' '--clients 64 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm rows 'SYMMETRY_ROPE_DECODE_ROWS=1' '--clients 64 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm grouped32 'SYMMETRY_ROPE_DECODE_ROWS=0' '--clients 32 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm rows32 'SYMMETRY_ROPE_DECODE_ROWS=1' '--clients 32 --max-model-len 1024 --steps 48 --warmup 8' > $O/ab.log 2>&1
