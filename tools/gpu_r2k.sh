set -e
export TMPDIR=/tmp
O=gpurun_out/r2k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for C in 10 24 32 64; do
  timeout -k 10 200 python bench.py --clients $C --steps 64 --warmup 8 >> $O/bench_clients.jsonl 2>>$O/bench.err
done
for L in 24 32 48 64; do
  timeout -k 10 200 python bench/prefill.py --clients 1 --prompt-len $L --reps 5 >> $O/prefill_small.jsonl 2>>$O/prefill.err
done
