#!/bin/bash
# One GPU call: the working tree's GPU parity suite (or the tests in $TESTS /
# -k $K), then an interleaved A/B of tools/variants/*.so on tools/bench_configs.py
# ($ONLY configs at $SPP spp, $ROUNDS rounds).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests/} ${K:+-k "$K"} \
    > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
ONLY=${ONLY:-C2,C4,SWEEP} ARGS="${SPP:+--spp $SPP}" bash tools/ab_configs.sh ${ROUNDS:-2}
