#!/bin/bash
# A/B of config rates over library variants (tools/variants/*.so) and
# environment settings.  Usage: bash tools/ab_lib.sh OUT ROUNDS "name:lib:ENV=V ..." ...
# e.g. bash tools/ab_lib.sh ab 2 "q:tools/variants/a_qc.so:RT_QC=0" "qc:tools/variants/a_qc.so:RT_QC=1"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab_lib}; R=${2:-2}; shift 2
mkdir -p $OUT
for r in $(seq $R); do
  for spec in "$@"; do
    IFS=: read -r name lib envs <<< "$spec"
    env RT_HIP_LIB=$lib $envs timeout -k 10 200 python3 tools/bench_configs.py --only ${ONLY:-C4,SWEEP} --spp ${SPP:-256} > $OUT/${name}_r$r.jsonl 2> $OUT/${name}_r$r.err || { echo "$name failed"; tail -5 $OUT/${name}_r$r.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/${name}_r$r.jsonl'):
    d = json.loads(l); print('$name round $r', d['config'], d['kernel_msamples_per_s'], 'Ms/s', d['kernel_ms'], 'ms')"
  done
done
