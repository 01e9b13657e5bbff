# PMC passes over the prefill GEMM (pgemm) and hipBLASLt at one shape: bash tools/gpu_pgemm_pmc.sh T N K
set -e
export TMPDIR=/tmp
T=${1:-4096}; N=${2:-4096}; K=${3:-4096}
O=gpurun_out/pmc_${T}_${N}_${K}
mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench/kernels/pgemm_dev/bench_pgemm.py --one $T $N $K > $O/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/p1 -o run -- python3 bench/kernels/pgemm_dev/bench_pgemm.py --one $T $N $K 5 > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_WAVES -d $O/p2 -o run -- python3 bench/kernels/pgemm_dev/bench_pgemm.py --one $T $N $K 5 > $O/p2.log 2>&1
