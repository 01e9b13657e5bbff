set -e
export TMPDIR=/tmp
O=gpurun_out/r2p
mkdir -p $O
ARMS=""
for L in 2048 7168; do
  ARMS="$ARMS --arm grid$L SYMMETRY_ATTN_STREAM_MIN=0 '--prompt-len $L --steps 32 --warmup 4'"
  for c in 0 1 2 3 4 5; do
    ARMS="$ARMS --arm cfg${c}_$L 'SYMMETRY_ATTN_STREAM_CFG=$c' '--prompt-len $L --steps 32 --warmup 4'"
  done
done
eval timeout -k 10 1100 python tools/ab_bench.py $O/stream_cfg.jsonl --reps 1 $ARMS > $O/stream_cfg.log 2>&1
