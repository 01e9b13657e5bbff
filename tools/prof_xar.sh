#!/bin/bash
# rocprofv3 kernel traces of the TP=8 shard (8B and 70B) with the fused GEMM + all-reduce (XAR) on and off.
set -o pipefail
for f in 1 0; do
  SYMMETRY_XGMI_FUSED=$f TP=8 TAG=tp8_xar$f bash tools/prof_tp_shard.sh || exit $?
  head -9 gpurun_out/prof_tp8_xar$f.csv
done
