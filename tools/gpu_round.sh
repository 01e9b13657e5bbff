#!/bin/bash
# Round check on the gpurun box: GPU tests, driver smoke(), the 1-GPU bench.  Each step under its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; grep '^{' gpurun_out/bench1.json | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print({k: d.get(k) for k in ('value','unit','ms_per_step','p50_ttft_ms','aggregate_tokens_per_s')})"
exit $rc
