#!/bin/bash
# Taper-threshold A/B: rank shares (N = 1..8) at 32 slices and the C2 / C3
# frames at their full 1000 spp, per variant library.  Usage: bash tools/r04_taper.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_taper}
mkdir -p $O
for r in 1 2; do
for v in ${VARIANTS:-a_base v_t16}; do
  RT_HIP_LIB=tools/variants/$v.so timeout -k 10 300 python tools/rank_share_rate.py --chunks 32 --pipeline --tile-rows 1 > $O/share_${v}_r$r.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  python3 -c "
import json
r = [json.loads(l) for l in open('$O/share_${v}_r$r.jsonl')]
print('share $v round $r', ' '.join('n%d %.1f (%.4f)' % (d['n'], d['msamples_per_s_share'], d['efficiency_vs_n1']) for d in r))"
  RT_HIP_LIB=tools/variants/$v.so timeout -k 10 300 python tools/bench_configs.py --only C2,C3 --full-spp > $O/cfg_${v}_r$r.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  python3 -c "
import json
for l in open('$O/cfg_${v}_r$r.jsonl'):
    d = json.loads(l); print('cfg $v round $r', d['config'], d['spp_measured'], d['kernel_msamples_per_s'])"
done
done
