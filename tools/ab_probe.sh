#!/bin/bash
# A/B of library variants on a probe script: bash tools/ab_probe.sh OUT ROUNDS "python3 tools/probes/x.py args" name:lib ...
OUT=gpurun_out/${1:-ab_probe}; R=${2:-2}; CMD=$3; shift 3
mkdir -p $OUT
for r in $(seq $R); do
  for spec in "$@"; do
    IFS=: read -r name lib <<< "$spec"
    RT_HIP_LIB=$lib timeout -k 10 300 $CMD > $OUT/${name}_r$r.jsonl 2> $OUT/${name}_r$r.err || { echo "$name failed"; tail -5 $OUT/${name}_r$r.err; exit 1; }
    sed "s/^/$name r$r /" $OUT/${name}_r$r.jsonl
  done
done
