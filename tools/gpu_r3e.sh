set -e
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for C in 64 128 256; do
  timeout -k 10 300 python bench/e2e.py --clients $C --max-model-len 1024 > $O/e2e2_$C.json 2> $O/e2e2_$C.err
done
timeout -k 10 200 python bench.py --clients 256 --max-model-len 1024 --steps 32 --warmup 4 > $O/bench256.json 2> $O/bench256.err
timeout -k 10 200 python bench.py > $O/bench10.json 2> $O/bench10.err
