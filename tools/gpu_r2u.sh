set -e
export TMPDIR=/tmp
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "logits_argmax or lm_head or sampl" tests/test_engine_gpu.py -k "wide or general_rows or logits_argmax or lm_head or sampl" > $O/pytest.log 2>&1
for C in 10 64 96 128 192 256; do
  timeout -k 10 400 python bench.py --clients $C --max-model-len 1024 --steps 48 --warmup 8 > $O/bench_$C.json 2> $O/bench_$C.err
  tail -1 $O/bench_$C.json
done
