set -e
export TMPDIR=/tmp
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 300 python bench.py --prompt-len 2048 --steps 32 --warmup 4 > $O/bench_2k.log 2>&1
timeout -k 10 300 python bench.py --prompt-len 7168 --steps 32 --warmup 4 > $O/bench_7k.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof2k -o run -- python3 bench.py --prompt-len 2048 --steps 16 --warmup 4 --profile-steps 32 > $O/prof2k.log 2>&1
