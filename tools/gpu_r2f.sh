set -e
export TMPDIR=/tmp
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mgemm or medium_m" > $O/pytest_new.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for L in 100 128 200; do
  for on in 0 1; do
    SYMMETRY_MGEMM=$on timeout -k 10 200 python bench/prefill.py --clients 1 --prompt-len $L --reps 5 > $O/prefill_c1_L${L}_mg${on}.json 2>$O/prefill_c1_L${L}_mg${on}.err
  done
done
