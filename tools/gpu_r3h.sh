set -e
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/profp -o run -- python3 bench.py --steps 2 --warmup 0 > $O/prof.log 2>&1
python tools/prof_summary.py /tmp/profp/run_results.db $O/prefill_10x128_kernels.csv --top 24 --last-ms 28 > $O/summary.txt 2>&1
