set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1
timeout -k 10 900 python tools/ab_bench.py gpurun_out/r2a/splitk.jsonl --reps 3 \
  --arm fused24 'SYMMETRY_SPLITK_RESID_ROWS=32' '--clients 24 --steps 64 --warmup 8' \
  --arm split24 'SYMMETRY_SPLITK_RESID_ROWS=24' '--clients 24 --steps 64 --warmup 8' \
  --arm fused28 'SYMMETRY_SPLITK_RESID_ROWS=32' '--clients 28 --steps 64 --warmup 8' \
  --arm split28 'SYMMETRY_SPLITK_RESID_ROWS=24' '--clients 28 --steps 64 --warmup 8' > gpurun_out/r2a/splitk.log 2>&1
timeout -k 10 600 python tools/ab_bench.py gpurun_out/r2a/nt.jsonl --reps 3 \
  --arm nt0 '' '--clients 10 --steps 64 --warmup 8 --nt-weights 0' \
  --arm nt1 '' '--clients 10 --steps 64 --warmup 8 --nt-weights 1' > gpurun_out/r2a/nt.log 2>&1
