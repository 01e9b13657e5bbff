set -e
export TMPDIR=/tmp
O=gpurun_out/r2x
mkdir -p $O
for S in 64 128 256; do
  timeout -k 10 200 python bench/kernels/bench_attn_decode.py --seqs $S --ctx 700 1500 3000 --layers 8 --wave 0 1 >> $O/attn_wave2.jsonl 2>> $O/attn_wave2.err
done
