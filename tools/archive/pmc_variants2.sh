#!/bin/bash
# SQ counters + kernel trace of C2 per library variant (tools/variants/*.so).
export TMPDIR=/tmp
OUT=gpurun_out/pmcv
rm -rf $OUT; mkdir -p $OUT
for v in tools/variants/*.so; do
  n=$(basename $v .so)
  RT_HIP_LIB=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/$n -o run --output-format csv -- python3 tools/bench_configs.py --only C2 --spp-scale 0.25 > $OUT/$n.log 2>&1 || exit 1
  RT_HIP_LIB=$v timeout -s KILL 120 rocprofv3 --kernel-trace -d $OUT/kt_$n -o run --output-format csv -- python3 tools/bench_configs.py --only C2 --spp-scale 0.25 > $OUT/kt_$n.log 2>&1 || exit 1
done
