set -e
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 400 python bench/e2e.py --model mixtral:8x7b --clients 4 --data-collection > $O/e2e_mixtral.json 2> $O/e2e_mixtral.err
timeout -k 10 500 python bench/e2e.py --model llama3:70b --clients 4 > $O/e2e_70b.json 2> $O/e2e_70b.err
timeout -k 10 300 python bench/e2e.py --clients 1 > $O/e2e_1.json 2> $O/e2e_1.err
