set -e
export TMPDIR=/tmp
O=gpurun_out/r2t
mkdir -p $O
for rep in 1 2; do
  SYMMETRY_BATCH_DELIVERY=0 SYMMETRY_GIL_SWITCH_US=0 timeout -k 10 240 python bench/e2e.py --clients 10 > $O/e2e_old_$rep.json 2>$O/e2e_old_$rep.err
  timeout -k 10 240 python bench/e2e.py --clients 10 > $O/e2e_new_$rep.json 2>$O/e2e_new_$rep.err
done
SYMMETRY_BATCH_DELIVERY=1 SYMMETRY_GIL_SWITCH_US=0 timeout -k 10 240 python bench/e2e.py --clients 10 > $O/e2e_batchonly.json 2>$O/e2e_batchonly.err
SYMMETRY_BATCH_DELIVERY=0 SYMMETRY_GIL_SWITCH_US=500 timeout -k 10 240 python bench/e2e.py --clients 10 > $O/e2e_gilonly.json 2>$O/e2e_gilonly.err
