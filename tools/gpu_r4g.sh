set -e
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python bench/e2e.py --model llama3:8b --clients 10 --max-tokens 256 > $O/e2e_10.json 2> $O/e2e_10.err
timeout -k 10 300 python bench/e2e.py --model llama3:8b --clients 1 --max-tokens 256 > $O/e2e_1.json 2> $O/e2e_1.err
