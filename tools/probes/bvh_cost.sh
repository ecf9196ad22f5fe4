#!/bin/bash
# Host SAH cost (tools/probes/bvh_cost.cpp) of the C4 tree and the sweep mesh
# (r04: the binned builder gave node visits 6.586 / 4.145, the full sweep
# 6.354 / 4.121; a spatial-split build added 41 references to the tree and
# left both proxies unchanged, 6.359 / 2.385, so it was dropped).
set -e
cd "$(dirname "$0")/../.."
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude -Itipe-raytracer_amd/csrc -o /tmp/bvh_cost tools/probes/bvh_cost.cpp tipe-raytracer_amd/csrc/rt_bvh.cpp
python3 - <<'PY' > /tmp/tree_tris.txt
import sys
sys.path.insert(0, "tipe-raytracer_amd")
from tipe_rt import scenes
for t in scenes.tree_mesh()[0]:
    print(*[t.A.e[i] for i in range(3)], *[t.B.e[i] for i in range(3)], *[t.C.e[i] for i in range(3)])
PY
python3 - <<'PY' > /tmp/sweep_tris.txt
import sys
sys.path.insert(0, "tipe-raytracer_amd")
from tipe_rt import scenes
for t in scenes.synthetic_cornell(10, 100)[1][0]:
    print(*[t.A.e[i] for i in range(3)], *[t.B.e[i] for i in range(3)], *[t.C.e[i] for i in range(3)])
PY
for m in tree sweep; do
  echo "$m $(/tmp/bvh_cost < /tmp/${m}_tris.txt)"
done
