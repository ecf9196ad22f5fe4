#!/bin/bash
# A/B timing of library variants in tools/variants/*.so (one process each,
# interleaved rounds).  Usage: bash tools/ab_variants.sh [rounds]
R=${1:-2}
for r in $(seq $R); do
  for v in tools/variants/*.so; do
   for ch in ${CHUNKS:-32}; do
    RT_BENCH_CHUNKS=$ch RT_HIP_LIB=$v timeout -k 10 240 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/ab_tmp.json 2>/dev/null || { echo "$v FAILED"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); print('$v', 'chunks', $ch, 'round', $r, d['value'], 'Ms/s kernel_ms', d['roofline']['kernel_ms'])"
   done
  done
done
