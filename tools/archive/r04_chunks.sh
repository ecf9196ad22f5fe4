#!/bin/bash
# Slice-count A/B (rt_chunk_bound with 5 taper levels): bench.py at 32/16/12/8
# slices (two rounds), the C3/C4/C5 frames at their full spp for each, and the
# split-traffic probe.  Usage: NOTESTS=1 bash tools/r04_chunks.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_chunks}
mkdir -p $O
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 120 tools/probes/split_traffic > $O/split_traffic.json 2>&1 && cat $O/split_traffic.json || exit 1
for r in 1 2; do
  for c in ${CHUNKS:-32 16 12 8}; do
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-extras --no-cpu-baseline --chunks $c > $O/bench_c${c}_r$r.json 2>> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_c${c}_r$r.json')); print('bench chunks $c round $r', d['value'], d['roofline']['kernel_ms'])"
  done
done
for c in ${CHUNKS:-32 16 12 8}; do
  timeout -k 10 300 python tools/bench_configs.py --only ${ONLY:-C3,C4,C5} --full-spp --chunks $c > $O/cfg_c$c.jsonl 2>> $O/cfg.err || { tail -5 $O/cfg.err; exit 1; }
  python3 -c "
import json
for l in open('$O/cfg_c$c.jsonl'):
    d = json.loads(l); print('cfg chunks', $c, d['config'], d['spp_measured'], d['kernel_msamples_per_s'])"
done
for c in ${CHUNKS:-32 16 12 8}; do
  timeout -k 10 300 python tools/rank_share_rate.py --chunks $c --pipeline --tile-rows 1 > $O/share_c$c.jsonl 2>> $O/share.err || { tail -5 $O/share.err; exit 1; }
  echo "share chunks $c"; cat $O/share_c$c.jsonl
done
