set -e
export TMPDIR=/tmp
O=gpurun_out/r2y
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attn_decode or wide" > $O/pytest.log 2>&1
ARMS=""
for C in 128 256; do
  ARMS="$ARMS --arm def$C SYMMETRY_ATTN_WAVE_UNITS=0 '--clients $C --prompt-len 600 --max-model-len 2048 --steps 32 --warmup 4' --arm wave$C SYMMETRY_ATTN_WAVE_UNITS=1024 '--clients $C --prompt-len 600 --max-model-len 2048 --steps 32 --warmup 4'"
done
eval timeout -k 10 900 python tools/ab_bench.py $O/wave_ab_long.jsonl --reps 2 $ARMS > $O/wave_ab_long.log 2>&1
