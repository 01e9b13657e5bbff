set -e
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
for C in 10 64 128 256; do
  timeout -k 10 300 python bench/e2e.py --clients $C --max-model-len 1024 > $O/e2e_$C.json 2> $O/e2e_$C.err
done
