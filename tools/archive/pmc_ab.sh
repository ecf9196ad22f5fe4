#!/bin/bash
# PMC passes (lane utilisation, wait, busy, VALU counts) of C4 for each
# RT_QC setting: bash tools/pmc_ab.sh OUT  (ONLY=C4 SPP=64 by default)
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_ab}
mkdir -p $OUT
B="python3 tools/bench_configs.py --only ${ONLY:-C4} --spp ${SPP:-64}"
for v in ${VARIANTS:-0 1}; do
  export RT_QC=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt$v -o run --output-format csv -- $B > $OUT/kt$v.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM -d $OUT/sq$v -o run --output-format csv -- $B > $OUT/sq$v.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU -d $OUT/sq2$v -o run --output-format csv -- $B > $OUT/sq2$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
done
echo done > $OUT/done.txt
