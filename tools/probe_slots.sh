set -o pipefail
P="timeout -k 10 250 python -u bench/kernels/pgemm_probe.py --rounds 3 --variants full slots5 slots6"
$P --tokens 768 --shape 6144 4096 --cfgs 3 5 > gpurun_out/probe_slots.jsonl &&
$P --tokens 768 --shape 28672 4096 --cfgs 0 10 >> gpurun_out/probe_slots.jsonl &&
$P --tokens 768 --shape 4096 14336 --cfgs 5 3 >> gpurun_out/probe_slots.jsonl &&
$P --grouped 64 128 256 --shape 28672 4096 --cfgs 1 9 10 4 5 >> gpurun_out/probe_slots.jsonl &&
$P --grouped 64 128 256 --shape 4096 14336 --cfgs 1 9 10 4 5 >> gpurun_out/probe_slots.jsonl &&
cat gpurun_out/probe_slots.jsonl
