set -e
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 400 python bench/kernels/bench_blas_lib.py --tokens 300 512 1280 2048 4096 > $O/blas_lib.jsonl 2> $O/blas_lib.err
