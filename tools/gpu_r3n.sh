set -e
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
for C in 32 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d /tmp/prof$C -o run -- python3 bench.py --clients $C --max-model-len 1024 --steps 16 --warmup 4 --profile-steps 24 > $O/prof$C.log 2>&1
  python tools/prof_summary.py /tmp/prof$C/run_results.db $O/decode_${C}clients_kernels.csv --top 18 --last-ms 80 > $O/summary_$C.txt 2>&1
done
