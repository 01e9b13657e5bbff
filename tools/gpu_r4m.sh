set -e
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
SYMMETRY_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 16 --warmup 4 > $O/bench_dp2.json 2> $O/bench_dp2.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof64 -o run -- python3 bench.py --clients 64 --max-model-len 1024 --steps 16 --warmup 4 --profile-steps 24 > $O/prof64.log 2>&1
python tools/prof_summary.py /tmp/prof64/run_results.db $O/decode_64clients_kernels.csv --top 18 --last-ms 80 > $O/summary_64.txt 2>&1
