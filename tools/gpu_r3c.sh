set -e
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mgemm" > $O/pytest.log 2>&1
MG_TS=128,192,256 timeout -k 10 400 python bench/kernels/bench_mgemm.py > $O/mgemm_wide.jsonl 2> $O/mgemm_wide.err
timeout -k 10 900 python tools/ab_bench.py $O/wide_ab.jsonl --reps 2 --arm base256 SYMMETRY_MGEMM_WIDE=0 '--clients 256 --max-model-len 1024 --steps 32 --warmup 4' --arm wide256 SYMMETRY_MGEMM_WIDE=1 '--clients 256 --max-model-len 1024 --steps 32 --warmup 4' --arm base128 SYMMETRY_MGEMM_WIDE=0 '--clients 128 --max-model-len 1024 --steps 32 --warmup 4' --arm wide128 SYMMETRY_MGEMM_WIDE=1 '--clients 128 --max-model-len 1024 --steps 32 --warmup 4' > $O/wide_ab.log 2>&1
