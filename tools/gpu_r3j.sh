set -e
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rope or oracle or prefill or medium or general" > $O/pytest.log 2>&1
for r in 1 2; do timeout -k 10 200 python bench.py > $O/bench_$r.json 2> $O/bench_$r.err; done
timeout -k 10 200 python bench/prefill.py --clients 1 --prompt-len 4096 > $O/prefill4k.json 2> $O/prefill4k.err || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/profp -o run -- python3 bench.py --steps 2 --warmup 0 > $O/prof.log 2>&1
python tools/prof_summary.py /tmp/profp/run_results.db $O/prefill_10x128_kernels.csv --top 24 --last-ms 28 > $O/summary.txt 2>&1
