for L in 1 2 3 4; do
  RT_BVH_LEAF=$L timeout -k 10 300 python3 tools/bench_configs.py --only C4,SWEEP > gpurun_out/leaf_$L.jsonl 2>/dev/null || { echo fail; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/leaf_$L.jsonl'):
    d=json.loads(l); print('leaf $L', d['config'], d['kernel_msamples_per_s'])"
done
