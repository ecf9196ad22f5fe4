#!/bin/bash
# PMC passes of the C4 / SWEEP config kernels (tools/bench_configs.py) -> gpurun_out/$1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_c4}
mkdir -p $OUT
B="python3 tools/bench_configs.py --only ${ONLY:-C4,SWEEP} --spp ${SPP:-256}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/mem -o run --output-format csv -- $B > $OUT/mem.log 2>&1
echo "exit=$?" > $OUT/done.txt
