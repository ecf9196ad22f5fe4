set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/c4prof}
mkdir -p $OUT
B="python3 tools/bench_configs.py --only C4 --spp-scale 0.5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE -d $OUT/fl -o run --output-format csv -- $B > $OUT/fl.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d $OUT/w -o run --output-format csv -- $B > $OUT/w.log 2>&1
echo "exit=$?" > $OUT/done.txt
