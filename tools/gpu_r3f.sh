set -e
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
for C in 128 256; do
  SYMMETRY_GIL_SWITCH_US=500 timeout -k 10 300 python bench/e2e.py --clients $C --max-model-len 1024 > $O/e2e_gil500_$C.json 2> $O/e2e_gil500_$C.err
  SYMMETRY_GIL_SWITCH_US=200 timeout -k 10 300 python bench/e2e.py --clients $C --max-model-len 1024 > $O/e2e_gil200_$C.json 2> $O/e2e_gil200_$C.err
done
