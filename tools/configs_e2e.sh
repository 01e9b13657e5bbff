#!/bin/bash
# BASELINE configs 2 / 5 / 4 (single-GPU variant) end to end over the encrypted swarm -> gpurun_out/e2e_*.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u bench/e2e.py --model llama3:8b --clients 1 > gpurun_out/e2e_c2.json 2> gpurun_out/e2e_c2.err || exit $?
timeout -k 10 400 python -u bench/e2e.py --model mixtral:8x7b --clients 4 --data-collection > gpurun_out/e2e_c5.json 2> gpurun_out/e2e_c5.err || exit $?
timeout -k 10 500 python -u bench/e2e.py --model llama3:70b --clients 4 > gpurun_out/e2e_c4.json 2> gpurun_out/e2e_c4.err || exit $?
