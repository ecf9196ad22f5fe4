#!/bin/bash
# C2 Msamples/s of render_kernel_q against its grid size (RT_QUEUE_BLOCKS).
for b in ${BLOCKS:-512 768 1024 2048 4096}; do
  RT_QUEUE_VERBOSE=1 RT_QUEUE_BLOCKS=$b timeout -k 10 120 python3 tools/bench_configs.py --only C2 > gpurun_out/qg.jsonl 2> gpurun_out/qg.err || exit 1
  python3 -c "
import json
for l in open('gpurun_out/qg.jsonl'):
    d=json.loads(l); print('blocks', $b, d['config'], d['kernel_msamples_per_s'], d['events_per_sample']['cast_lane_slots'])"
done
head -2 gpurun_out/qg.err
