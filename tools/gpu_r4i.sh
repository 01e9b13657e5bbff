set -e
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_split.json 2> $O/bench_split.err
SYMMETRY_BURST_SPLIT=0 timeout -k 10 300 python bench.py > $O/bench_nosplit.json 2> $O/bench_nosplit.err
timeout -k 10 300 python bench.py --clients 64 --max-model-len 1024 > $O/bench_64_split.json 2> $O/bench_64.err
SYMMETRY_BURST_SPLIT=0 timeout -k 10 300 python bench.py --clients 64 --max-model-len 1024 > $O/bench_64_nosplit.json 2> $O/bench_64n.err
