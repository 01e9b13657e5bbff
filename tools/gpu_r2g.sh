set -e
export TMPDIR=/tmp
O=gpurun_out/r2g
mkdir -p $O
for L in 64 128 192 256 384 512 640 768 896 1024 1280; do
  timeout -k 10 200 python bench/prefill.py --clients 1 --prompt-len $L --reps 5 >> $O/prefill_sweep.jsonl 2>>$O/prefill_sweep.err
done
