set -e
mkdir -p gpurun_out
SYMMETRY_SPLITK_RESID_ROWS=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_sk.txt 2>&1
for c in 24 32 64; do
  SYMMETRY_SPLITK_RESID_ROWS=0 timeout -k 10 200 python bench.py --clients $c --steps 64 --warmup 8 > gpurun_out/ab_off_$c.json 2> gpurun_out/ab_off_$c.err
  timeout -k 10 200 python bench.py --clients $c --steps 64 --warmup 8 > gpurun_out/ab_on_$c.json 2> gpurun_out/ab_on_$c.err
done
