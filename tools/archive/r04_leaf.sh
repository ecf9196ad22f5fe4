#!/bin/bash
# Leaf size (RT_BVH_LEAF, read by rt_bvh.cpp at upload) on the sweep-SAH tree:
# C4 / SWEEP at 256 spp, alternating rounds.  Usage: bash tools/r04_leaf.sh TAG
set -o pipefail
O=gpurun_out/${1:-r04_leaf}
mkdir -p $O
for r in 1 2; do
  for l in ${LEAVES:-1 2}; do
    RT_BVH_LEAF=$l timeout -k 10 300 python3 tools/bench_configs.py --only C4,SWEEP --spp 256 > $O/leaf$l.jsonl 2>/dev/null || { echo "leaf $l FAILED"; exit 1; }
    python3 -c "
import json
for l in open('$O/leaf$l.jsonl'):
    d=json.loads(l); print('leaf $l round $r', d['config'], d['kernel_msamples_per_s'], 'Ms/s')" | tee -a $O/ab.txt
  done
done
