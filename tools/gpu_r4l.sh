set -e
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 1400 python tools/ab_bench.py $O/ab_general_rows.jsonl --reps 3 \
  --arm fused16 'SYMMETRY_GENERAL_ROWS=24' '--clients 16 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm general16 'SYMMETRY_GENERAL_ROWS=12' '--clients 16 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm fused20 'SYMMETRY_GENERAL_ROWS=24' '--clients 20 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm general20 'SYMMETRY_GENERAL_ROWS=12' '--clients 20 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm fused12 'SYMMETRY_GENERAL_ROWS=24' '--clients 12 --max-model-len 1024 --steps 48 --warmup 8' \
  --arm general12 'SYMMETRY_GENERAL_ROWS=12' '--clients 12 --max-model-len 1024 --steps 48 --warmup 8' > $O/ab.log 2>&1
