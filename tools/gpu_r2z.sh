set -e
export TMPDIR=/tmp
O=gpurun_out/r2z
mkdir -p $O
for M in 1 10 16; do
  timeout -k 10 120 python bench/kernels/bench_decode_block.py --M $M --ctx 200 --cfgs 0 4 >> $O/block_ao.jsonl 2>> $O/block_ao.err
done
timeout -k 10 120 python bench/kernels/bench_decode_block.py --M 10 --ctx 600 --cfgs 0 4 >> $O/block_ao.jsonl 2>> $O/block_ao.err
