#!/bin/bash
# Round-4 GPU call: parity suite, a short bench line, op-rate probe, A/B of
# tools/variants/*.so, then a PC-sampling probe of the C2 queue kernel
# (rocprofv3 beta; host_trap, time unit).
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04_a}
mkdir -p $O
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json; echo
timeout -k 10 120 tools/probes/op_rates2 > $O/op_rates2.txt 2>&1 || exit 1
grep "waves/SIMD 8" $O/op_rates2.txt | head -30
if ls tools/variants/*.so >/dev/null 2>&1; then
  ONLY=${ONLY:-C2,C3,C4,SWEEP} bash tools/ab_configs.sh ${ROUNDS:-2} > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
  cat $O/ab.txt
fi
