#!/bin/bash
# Round-5 A/B step on the GPU box: parity subset ($K) for every variant in
# tools/variants/ except a_base, then interleaved config rates (ONLY, ARGS).
# Usage: K="bvh or tree" ONLY=C4,SWEEP ARGS="--spp 256" bash tools/r05_ab.sh TAG [rounds]
set -o pipefail
TAG=${1:-r05_ab}; R=${2:-3}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in tools/variants/*.so; do
  n=$(basename $v .so)
  [ "$n" = a_base ] && continue
  echo "[$(date +%T)] tests $n"
  RT_HIP_LIB=$v timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -k "${K:-bvh or tree}" \
    ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_fuzz.py tests/test_gpu_reference.py} > $OUT/tests_$n.log 2>&1 \
    || { echo "tests $n failed"; tail -30 $OUT/tests_$n.log; exit 1; }
  tail -1 $OUT/tests_$n.log
done
echo "[$(date +%T)] configs"
ONLY=${ONLY:-C4,SWEEP} ARGS="${ARGS:---spp 256}" bash tools/ab_configs.sh $R 2>&1 | tee $OUT/ab.txt
echo "[$(date +%T)] done"
