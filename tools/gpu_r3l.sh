set -e
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 900 python tools/ab_bench.py $O/gu_ab.jsonl --reps 2 --arm lib96 SYMMETRY_MGEMM_WIDE_N=0 '--clients 96 --max-model-len 1024 --steps 32 --warmup 4' --arm mg96 SYMMETRY_MGEMM_WIDE_N=1 '--clients 96 --max-model-len 1024 --steps 32 --warmup 4' --arm lib128 SYMMETRY_MGEMM_WIDE_N=0 '--clients 128 --max-model-len 1024 --steps 32 --warmup 4' --arm mg128 SYMMETRY_MGEMM_WIDE_N=1 '--clients 128 --max-model-len 1024 --steps 32 --warmup 4' > $O/gu_ab.log 2>&1
