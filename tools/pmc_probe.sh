#!/bin/bash
# PMC passes (as tools/pmc_c4.sh) of tools/probes/nonopq_scenes.py under a library variant.
# Usage: LIB=tools/variants/x.so bash tools/pmc_probe.sh OUT [spp]
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_probe}
mkdir -p $OUT
B="python3 tools/probes/nonopq_scenes.py ${2:-64}"
export RT_HIP_LIB=${LIB:-tipe-raytracer_amd/librt_hip.so}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/mem -o run --output-format csv -- $B > $OUT/mem.log 2>&1
echo "exit=$?" > $OUT/done.txt
