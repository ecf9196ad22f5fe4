#!/bin/bash
# Instruction counters of render_kernel for each tools/variants/*.so on one
# config.  Usage: ONLY=C2 bash tools/pmc_variants.sh
set -o pipefail
export TMPDIR=/tmp
for v in tools/variants/*.so; do
  n=$(basename $v .so)
  RT_HIP_LIB=$v timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_BRANCH -d gpurun_out/pmcv/$n -o run --output-format csv -- python3 tools/bench_configs.py --only ${ONLY:-C2} --spp-scale 0.25 > gpurun_out/pmcv/$n.log 2>&1 || exit 1
done
