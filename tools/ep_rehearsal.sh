# One-GPU EP rehearsal sweep (bench/ep_rehearsal.py): both combine modes at world 2 and 4
set -o pipefail
out=gpurun_out/ep_crossover.jsonl
: > $out
for w in 2 4; do
  for m in a2a allreduce; do
    timeout -k 10 280 python -u bench/ep_rehearsal.py --world $w --mode $m --tokens ${TOKENS:-64,128,256,512,1024} \
      --reps 3 >> $out 2> gpurun_out/ep_${w}_${m}.err || { tail -30 gpurun_out/ep_${w}_${m}.err; exit 1; }
  done
done
cat $out
