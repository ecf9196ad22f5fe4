#!/bin/bash
# A/B of library variants (tools/variants/*.so) on the mesh scenes: C4 and the
# 10-sphere / 100-triangle sweep scene (bench.py's configs extra, kernel rates).
R=${1:-1}
for r in $(seq $R); do
  for v in tools/variants/*.so; do
    RT_HIP_LIB=$v timeout -k 10 300 python3 -c "
import sys, json; sys.path.insert(0, 'tipe-raytracer_amd'); sys.argv = ['bench']
import torch, bench, tipe_rt
from tipe_rt import scenes
bench.CONFIGS = {k: v for k, v in bench.CONFIGS.items() if k in '${ONLY:-C4,sweep_10s_100t}'.split(',')}
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ('origin', 'target', 'up', 'vfov', 'ratio')})
dev = torch.device('cuda', 0)
for k, d in bench.configs_extra(dev, torch.cuda.current_stream(dev), cam).items():
    print('$v', 'round', $r, k, d['kernel_msamples_per_s'], 'Ms/s frac', d['frac'])
" 2>/dev/null || { echo "$v FAILED"; exit 1; }
  done
done
