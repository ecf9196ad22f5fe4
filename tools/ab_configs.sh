#!/bin/bash
# A/B of library variants (tools/variants/*.so) on tools/bench_configs.py.
# Usage: ONLY=C4 bash tools/ab_configs.sh [rounds]
R=${1:-1}
for r in $(seq $R); do
  for v in tools/variants/*.so; do
    RT_HIP_LIB=$v timeout -k 10 300 python3 tools/bench_configs.py --only ${ONLY:-C2,C3,C4} ${ARGS} > gpurun_out/ab_cfg.jsonl 2>/dev/null || { echo "$v FAILED"; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ab_cfg.jsonl'):
    d=json.loads(l); print('$v', 'round', $r, d['config'], d['kernel_msamples_per_s'], 'Ms/s', d['kernel_ms'], 'ms')"
  done
done
