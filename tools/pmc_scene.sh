#!/bin/bash
# SQ counters for one roofline-sweep scene: bash tools/pmc_scene.sh Ns:Nt TAG
export TMPDIR=/tmp
OUT=gpurun_out/pmcs/$2
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- python3 tools/roofline_sweep.py --only $1 --spp 32 --reps 1 > $OUT/sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/roofline_sweep.py --only $1 --spp 32 --reps 1 > $OUT/kt.log 2>&1
