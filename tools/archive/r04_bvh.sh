#!/bin/bash
# Round-4 BVH builder A/B: the triangle-path GPU suites through the variant
# library ($V, default b_sweep), then the C4 / SWEEP A/B of every
# tools/variants/*.so at 256 spp.  Usage: bash tools/r04_bvh.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_bvh}
mkdir -p $O
V=${V:-b_sweep}
RT_HIP_LIB=tools/variants/$V.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_fallback.py \
   tests/test_gpu_instantiations.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_$V.log 2>&1 || { tail -30 $O/pytest_$V.log; exit 1; }
echo "parity $V: $(tail -1 $O/pytest_$V.log)"
ONLY=${ONLY:-C4,SWEEP} ARGS="--spp 256" bash tools/ab_configs.sh ${ROUNDS:-3} > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
