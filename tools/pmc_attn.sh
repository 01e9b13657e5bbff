#!/bin/bash
# PMC counters of the decode attention kernel alone (bench_attn_decode.py, 10 seqs, 256-token contexts), two
# passes (counter-block limits), each its own run; summary -> gpurun_out/pmc_attn.txt
set -o pipefail
root=$(pwd)
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format rocpd -d /tmp/pmc_attn$i -o run -- \
    python3 "$root/bench/kernels/bench_attn_decode.py" --seqs 10 --ctx ${CTX:-256} --layers 32 \
    > "$root/gpurun_out/pmc_attn$i.log" 2>&1 || exit $?
done
cd "$root" && python3 tools/pmc_summary.py $(ls /tmp/pmc_attn*/*/*.db /tmp/pmc_attn*/*.db 2>/dev/null) --filter attn \
  > gpurun_out/pmc_attn.txt
