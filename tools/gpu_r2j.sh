set -e
export TMPDIR=/tmp
O=gpurun_out/r2j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mgemm or medium_m" > $O/pytest_new.log 2>&1
ARMS=""
for C in 10 16 24 32 48 64; do
  ARMS="$ARMS --arm fused$C SYMMETRY_GENERAL_ROWS=0 '--clients $C --steps 48 --warmup 8' --arm general$C SYMMETRY_GENERAL_ROWS=1 '--clients $C --steps 48 --warmup 8'"
done
eval timeout -k 10 1000 python tools/ab_bench.py $O/general_ab.jsonl --reps 2 $ARMS > $O/general_ab.log 2>&1
