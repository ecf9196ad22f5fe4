#!/bin/bash
# A/B of BVH-walk variants: non-opaque scenes (nature, mineways, water tree) at
# 128 spp and the C4 / sweep configs at a quarter of their spp, R rounds, plus
# the BVH parity tests on the last variant.
#   bash tools/ab_bvh.sh OUT R name:lib ...
OUT=gpurun_out/${1:-ab_bvh}; R=${2:-2}; shift 2
mkdir -p $OUT
for r in $(seq $R); do
  for spec in "$@"; do
    IFS=: read -r name lib <<< "$spec"
    RT_HIP_LIB=$lib timeout -k 10 300 python3 tools/probes/nonopq_scenes.py 128 > $OUT/${name}_nq_r$r.jsonl 2> $OUT/${name}_nq_r$r.err || { echo "$name failed"; tail -5 $OUT/${name}_nq_r$r.err; exit 1; }
    RT_HIP_LIB=$lib timeout -k 10 300 python3 tools/bench_configs.py --only C4,SWEEP,NATURE --spp 128 > $OUT/${name}_cfg_r$r.jsonl 2> $OUT/${name}_cfg_r$r.err || { echo "$name cfg failed"; tail -5 $OUT/${name}_cfg_r$r.err; exit 1; }
    sed "s/^/$name r$r /" $OUT/${name}_nq_r$r.jsonl | cut -c1-400
    sed "s/^/$name r$r /" $OUT/${name}_cfg_r$r.jsonl | cut -c1-400
  done
done
