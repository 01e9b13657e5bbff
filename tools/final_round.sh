#!/bin/bash
# tuned-hipBLASLt A/B, then the round check (GPU tests, smoke, bench) in one box session
set -o pipefail
bash tools/blaslt_ab.sh || exit $?
bash tools/gpu_round.sh
