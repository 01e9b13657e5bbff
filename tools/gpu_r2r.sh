set -e
export TMPDIR=/tmp
O=gpurun_out/r2r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for L in 300 512 768 1024 1280; do
  timeout -k 10 200 python bench/prefill.py --clients 1 --prompt-len $L --reps 5 >> $O/prefill.jsonl 2>>$O/prefill.err
done
timeout -k 10 200 python bench.py --steps 64 --warmup 8 > $O/bench.log 2>&1
