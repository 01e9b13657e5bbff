set -o pipefail
bash tools/gpu_suite.sh tp > gpurun_out/tp2_rehearsal.txt 2>&1
rc=$?; grep '^{' gpurun_out/bench_tp2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], d['per_rank_ms_per_step'], d['host_ms_per_step'], d['client_end']['engine']['step_phase_ms'], d['tp'])"; [ $rc -eq 0 ] || exit $rc
SYMMETRY_XGMI_FUSED=1 TP=8 TAG=tp8_xar bash tools/prof_tp_shard.sh && head -9 gpurun_out/prof_tp8_xar.csv
SYMMETRY_XGMI_FUSED=1 timeout -k 10 300 python -u bench/tp_shard.py --tp 8 --clients 4 --model llama3:70b > gpurun_out/tp_shard_70b_f1.json 2>gpurun_out/tp_shard_70b_f1.err
rc=$?; echo "70b fused $(tail -1 gpurun_out/tp_shard_70b_f1.json)"; exit $rc
