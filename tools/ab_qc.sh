#!/bin/bash
# GPU step: BVH-scene parity (render_kernel_qc is the default) then A/B of
# render_kernel_q (RT_QC=0) against render_kernel_qc (RT_QC=1) on C4 and the
# sweep scene at 256 spp (8 samples per slice).  Usage: bash tools/ab_qc.sh OUT [rounds]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab_qc}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_scale.py -k "bvh or tree or sweep or mineways or sky or tiny" > $OUT/pytest_bvh.log 2>&1 \
  || { echo "tests failed"; tail -30 $OUT/pytest_bvh.log; exit 1; }
tail -2 $OUT/pytest_bvh.log
fi
for r in $(seq ${2:-2}); do
  for v in 0 1; do
    RT_QC=$v timeout -k 10 200 python3 tools/bench_configs.py --only ${ONLY:-C4,SWEEP} --spp ${SPP:-256} > $OUT/qc${v}_r$r.jsonl 2> $OUT/qc${v}_r$r.err || { echo "RT_QC=$v failed"; tail -5 $OUT/qc${v}_r$r.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/qc${v}_r$r.jsonl'):
    d = json.loads(l); print('RT_QC=$v round $r', d['config'], d['kernel_msamples_per_s'], 'Ms/s', d['kernel_ms'], 'ms')"
  done
done
