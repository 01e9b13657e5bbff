#!/bin/bash
# PMC counters of one kernel under a benchmark command, two passes (counter-block limits), each its own run:
#   TAG=name FILTER=kernel_substr bash tools/pmc_kernel.sh python3 bench/kernels/bench_grouped.py --rows 128
# summary -> gpurun_out/pmc_$TAG.txt
set -o pipefail
root=$(pwd)
tag=${TAG:-kernel}
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU" \
           "FETCH_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format rocpd -d /tmp/pmc_$tag$i -o run -- "$@" \
    > "$root/gpurun_out/pmc_$tag$i.log" 2>&1 || exit $?
done
cd "$root" && python3 tools/pmc_summary.py $(ls /tmp/pmc_$tag*/*/*.db /tmp/pmc_$tag*/*.db 2>/dev/null) --filter "$FILTER" \
  > gpurun_out/pmc_$tag.txt
