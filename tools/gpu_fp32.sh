#!/bin/bash
# GPU step: FP32-mode tolerance tests, then the whole GPU suite and the bench.
# A crash (exit > 1) of the first step ends the call.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-f1}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fp32_mode.py -v -s -m gpu --timeout 120 --timeout-method thread > $OUT/fp32.log 2>&1
rc=$?
echo "fp32_exit=$rc" >> $OUT/fp32.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/fp32_bias.py > $OUT/fp32_bias.jsonl 2> $OUT/fp32_bias.err || exit 1
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
