# A/B: prefill steps up to 1024 tokens / 8 sequences replayed from hipGraphs vs eager (<= 256 tokens graphs only)
set -o pipefail
G="SYMMETRY_PREFILL_GRAPH_TOKENS=1024 SYMMETRY_PREFILL_GRAPH_BUCKETS=16,32,64,128,192,256,384,512,768,1024 SYMMETRY_PREFILL_GRAPH_SEQS=1,2,4,8 SYMMETRY_PREFILL_CAPTURE_SEQS=1,8"
: > gpurun_out/prefill_graph_ab.jsonl
python tools/ab_bench.py gpurun_out/prefill_graph_ab.jsonl --script bench/prefill.py --reps 2 --timeout 300 \
  --arm eager '' '--clients 6 --reps 5' --arm graph "$G" '--clients 6 --reps 5' \
  --arm eager8 '' '--clients 8 --reps 5' --arm graph8 "$G" '--clients 8 --reps 5' > gpurun_out/prefill_graph_ab.log 2>&1 || { tail -30 gpurun_out/prefill_graph_ab.log; exit 1; }
tail -4 gpurun_out/prefill_graph_ab.log
env $G timeout -k 10 300 python -u bench.py > gpurun_out/bench_pg_graph.json 2> gpurun_out/bench_pg_graph.err || { tail -20 gpurun_out/bench_pg_graph.err; exit 1; }
grep '^{' gpurun_out/bench_pg_graph.json | python -c "import json,sys; r=json.loads(sys.stdin.read().splitlines()[-1]); print({k: r[k] for k in ('value','ms_per_step','p50_ttft_ms','engine_p50_ttft_ms','verified')}, r['client_end']['first_steps'][:3])"
