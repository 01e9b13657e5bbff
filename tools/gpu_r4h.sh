set -e
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 900 python tools/ab_bench.py $O/ab_ttft_split.jsonl --reps 2 \
  --arm one_step '' '--steps 32 --warmup 8' \
  --arm b768_m512 '' '--steps 32 --warmup 8 --max-batched-tokens 768 --mixed-prefill-tokens 512' \
  --arm b768_m768 '' '--steps 32 --warmup 8 --max-batched-tokens 768 --mixed-prefill-tokens 768' \
  --arm b640_m640 '' '--steps 32 --warmup 8 --max-batched-tokens 640 --mixed-prefill-tokens 640' > $O/ab.log 2>&1
