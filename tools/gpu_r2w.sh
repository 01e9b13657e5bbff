set -e
export TMPDIR=/tmp
O=gpurun_out/r2w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attn_decode or wide" > $O/pytest.log 2>&1
ARMS=""
for C in 32 64 128 256; do
  ARMS="$ARMS --arm grid$C SYMMETRY_ATTN_WAVE_UNITS=0 '--clients $C --max-model-len 1024 --steps 48 --warmup 8' --arm wave$C SYMMETRY_ATTN_WAVE_UNITS=1 '--clients $C --max-model-len 1024 --steps 48 --warmup 8'"
done
eval timeout -k 10 900 python tools/ab_bench.py $O/wave_ab.jsonl --reps 2 $ARMS > $O/wave_ab.log 2>&1
