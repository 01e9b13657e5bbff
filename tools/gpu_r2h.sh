set -e
export TMPDIR=/tmp
O=gpurun_out/r2h
mkdir -p $O
for on in 0 1; do
  SYMMETRY_MGEMM=$on timeout -k 10 300 python bench/multiturn.py > $O/multiturn_mg${on}.jsonl 2>$O/multiturn_mg${on}.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o run -- python3 bench/prefill.py --clients 1 --prompt-len 128 --reps 3 > $O/prof_c1.log 2>&1
