set -e
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mgemm" > $O/pytest.log 2>&1
timeout -k 10 600 python tools/ab_bench.py $O/wide_ab.jsonl --reps 2 --arm base256 SYMMETRY_MGEMM_WIDE=0 '--clients 256 --max-model-len 1024 --steps 32 --warmup 4' --arm wide256 SYMMETRY_MGEMM_WIDE=1 '--clients 256 --max-model-len 1024 --steps 32 --warmup 4' --arm base192 SYMMETRY_MGEMM_WIDE=0 '--clients 192 --max-model-len 1024 --steps 32 --warmup 4' --arm wide192 SYMMETRY_MGEMM_WIDE=1 '--clients 192 --max-model-len 1024 --steps 32 --warmup 4' > $O/wide_ab.log 2>&1
