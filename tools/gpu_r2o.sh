set -e
export TMPDIR=/tmp
O=gpurun_out/r2o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attn_decode" > $O/pytest_attn.log 2>&1
timeout -k 10 1000 python tools/ab_bench.py $O/stream_ab.jsonl --reps 2 \
  --arm grid1k SYMMETRY_ATTN_STREAM_MIN=0 '--prompt-len 1024 --steps 32 --warmup 4' \
  --arm stream1k SYMMETRY_ATTN_STREAM_MIN=1024 '--prompt-len 1024 --steps 32 --warmup 4' \
  --arm grid2k SYMMETRY_ATTN_STREAM_MIN=0 '--prompt-len 2048 --steps 32 --warmup 4' \
  --arm stream2k SYMMETRY_ATTN_STREAM_MIN=1024 '--prompt-len 2048 --steps 32 --warmup 4' \
  --arm grid7k SYMMETRY_ATTN_STREAM_MIN=0 '--prompt-len 7168 --steps 32 --warmup 4' \
  --arm stream7k SYMMETRY_ATTN_STREAM_MIN=1024 '--prompt-len 7168 --steps 32 --warmup 4' > $O/stream_ab.log 2>&1
