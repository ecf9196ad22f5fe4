#!/bin/bash
# Config rates + per-sample events (incl. exact_rescans) of each library
# variant in tools/variants/*.so.  Usage: bash tools/ab_configs_variants.sh OUTDIR
OUT=${1:-gpurun_out/abv}
mkdir -p $OUT
for v in tools/variants/*.so; do
  n=$(basename $v .so)
  RT_HIP_LIB=$v timeout -k 10 200 python3 tools/bench_configs.py > $OUT/$n.jsonl 2> $OUT/$n.err || { echo "$v FAILED"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/$n.jsonl'):
    d = json.loads(l); e = d['events_per_sample']
    print('$n', d['config'], round(d['kernel_msamples_per_s'], 1), 'Ms/s  rescans/cast', round(e['exact_rescans'] / e['casts'], 6))"
done
