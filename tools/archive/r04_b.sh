#!/bin/bash
# Round-4 measurement call B: slice-count A/B + split probe (tools/r04_chunks.sh),
# library variant A/B (tools/variants/*.so) on C2/C3, and a PC-sampling pass of
# the C2 queue kernel.  Usage: bash tools/r04_b.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04_b}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$NOCHUNKS" ]; then
NOTESTS=1 bash tools/r04_chunks.sh $TAG || exit 1
fi
if [ -n "$PARITY_LIB" ]; then
  RT_HIP_LIB=$PARITY_LIB timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu \
     --timeout 300 --timeout-method thread > $O/pytest_variant.log 2>&1 || { tail -30 $O/pytest_variant.log; exit 1; }
  echo "variant parity ($PARITY_LIB): $(tail -1 $O/pytest_variant.log)"
fi
if ls tools/variants/*.so >/dev/null 2>&1; then
  ONLY=${ONLY:-C2,C3,C4} bash tools/ab_configs.sh ${ROUNDS:-2} > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
  cat $O/ab.txt
fi
