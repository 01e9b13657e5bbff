set -e
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_gemm_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "argmax or lm_head or oracle or wide" > $O/pytest.log 2>&1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/bench_$r.json 2> $O/bench_$r.err
  tail -1 $O/bench_$r.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof10 -o run -- python3 bench.py --steps 16 --warmup 4 --profile-steps 32 > $O/prof10.log 2>&1
python tools/prof_summary.py /tmp/prof10/run_results.db $O/decode_10clients_kernels.csv --top 14 --last-ms 100 > $O/summary10.txt 2>&1
