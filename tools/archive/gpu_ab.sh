#!/bin/bash
# GPU step: focused tests (optional, $TESTS) then interleaved A/B of tools/variants/*.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread ${K:+-k "$K"} $TESTS > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -3 gpurun_out/ab_tests.log
fi
bash tools/ab_variants.sh ${ROUNDS:-2} 2>&1 | tee gpurun_out/ab.log
