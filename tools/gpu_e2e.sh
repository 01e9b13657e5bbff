set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench/e2e.py --model llama3:8b --clients 10 --max-tokens 256 > gpurun_out/e2e_c3.json 2> gpurun_out/e2e_c3.err && \
timeout -k 10 300 python bench/e2e.py --model llama3:8b --clients 1 --max-tokens 256 > gpurun_out/e2e_c2.json 2> gpurun_out/e2e_c2.err && \
timeout -k 10 400 python bench/e2e.py --model mixtral:8x7b --clients 4 --max-tokens 128 --data-collection > gpurun_out/e2e_c5.json 2> gpurun_out/e2e_c5.err && \
SYMMETRY_OPS=torch timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_b1.json 2> gpurun_out/bench_b1.err
