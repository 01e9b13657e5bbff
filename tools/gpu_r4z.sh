set -e
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof10 -o run -- python3 bench.py --steps 16 --warmup 4 --profile-steps 24 > $O/prof10.log 2>&1
python tools/prof_summary.py /tmp/prof10/run_results.db $O/decode_10clients_kernels.csv --top 18 --last-ms 80 > $O/summary_10.txt 2>&1
