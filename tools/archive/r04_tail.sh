#!/bin/bash
# Round-4 call C: parity of the candidate-pass (c_min2) and tail-grab
# (e_qtail1) variants through the GPU parity/scale suites, rank shares
# (tools/rank_share_rate.py) per variant and slice count, and the C2/C3/C4
# variant A/B at 256 spp.  Usage: bash tools/r04_tail.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_tail}
mkdir -p $O
for v in ${PARITY_VARIANTS:-c_min2 e_qtail1}; do
  RT_HIP_LIB=tools/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu \
     --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/pytest_$v.log)"
done
for v in ${SHARE_VARIANTS-a_base e_qtail1 f_qtail2}; do
  for c in ${CHUNKS:-32 12 8}; do
    RT_HIP_LIB=tools/variants/$v.so timeout -k 10 300 python tools/rank_share_rate.py --chunks $c --pipeline --tile-rows 1 > $O/share_${v}_c$c.jsonl 2>> $O/share.err || { tail -5 $O/share.err; exit 1; }
    python3 -c "
import json
r = [json.loads(l) for l in open('$O/share_${v}_c$c.jsonl')]
print('share $v chunks $c', ' '.join('n%d %.1f (%.4f)' % (d['n'], d['msamples_per_s_share'], d['efficiency_vs_n1']) for d in r))"
  done
done
ONLY=${ONLY:-C2,C3,C4} ARGS="--spp 256" bash tools/ab_configs.sh ${ROUNDS:-2} > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
