#!/bin/bash
# Round-4 call: the full -m gpu suite on the default build, then the variant
# A/B (tools/variants/*.so) on $ONLY at 256 spp.  Usage: bash tools/r04_c.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
ONLY=${ONLY:-C2,C3,C4} ARGS="--spp 256" bash tools/ab_configs.sh ${ROUNDS:-2} > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
