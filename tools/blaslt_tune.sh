#!/bin/bash
# Offline hipBLASLt solution sweep for the library prefill GEMMs, in torch's hipBLASLt (the one the runtime
# calls) -> gpurun_out/blaslt_tune.jsonl; then: python tools/blaslt_table.py gpurun_out/blaslt_tune.jsonl
set -o pipefail
mkdir -p gpurun_out
SH=${SHAPES:-6144x4096,4096x4096,28672x4096,4096x14336}
for s in ${SH//,/ }; do
  timeout -k 10 600 python -u bench/kernels/blaslt_tune.py --shapes $s ${MS:+--ms $MS} >> gpurun_out/blaslt_tune.jsonl \
    2>> gpurun_out/blaslt_tune.err || exit $?
done
