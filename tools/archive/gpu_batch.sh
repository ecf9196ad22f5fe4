#!/bin/bash
# One GPU call: focused parity tests, C2 A/B of tools/variants, and the
# small-mesh BVH threshold (RT_BVH_MIN_TRIS) on C3/C5 with its parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "device_math or phi or normalize or task_queue or cornell or sphere or bvh or tree or duplicate or grazing or synthetic" > gpurun_out/b_tests.log 2>&1 || { tail -20 gpurun_out/b_tests.log; exit 1; }
tail -1 gpurun_out/b_tests.log
RT_BVH_MIN_TRIS=1 timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "pyramid or refract or alpha or mineways or texture or sky" > gpurun_out/b_tests2.log 2>&1 || { tail -20 gpurun_out/b_tests2.log; exit 1; }
tail -1 gpurun_out/b_tests2.log
ONLY=C2,C4,SWEEP bash tools/ab_configs.sh 2 || exit 1
for T in 1 32; do
  RT_BVH_MIN_TRIS=$T timeout -k 10 300 python3 tools/bench_configs.py --only C3,C5 > gpurun_out/b_cfg_$T.jsonl 2>/dev/null || exit 1
  python3 -c "
import json
for l in open('gpurun_out/b_cfg_$T.jsonl'):
    d=json.loads(l); print('min_tris $T', d['config'], d['kernel_msamples_per_s'])"
done
