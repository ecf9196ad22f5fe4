#!/bin/bash
# Host check of the 64-byte BVH nodes on the C4 tree and the sweep mesh.
set -e
cd "$(dirname "$0")/../.."
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude -Itipe-raytracer_amd/csrc -o /tmp/bvh_h_check tools/probes/bvh_h_check.cpp tipe-raytracer_amd/csrc/rt_bvh.cpp
python3 - <<'PY' > /tmp/tree_tris.txt
import sys
sys.path.insert(0, "tipe-raytracer_amd")
from tipe_rt import scenes
for t in scenes.tree_mesh()[0]:
    print(*[t.A.e[i] for i in range(3)], *[t.B.e[i] for i in range(3)], *[t.C.e[i] for i in range(3)])
PY
/tmp/bvh_h_check < /tmp/tree_tris.txt
python3 - <<'PY' > /tmp/sweep_tris.txt
import sys
sys.path.insert(0, "tipe-raytracer_amd")
from tipe_rt import scenes
for t in scenes.synthetic_cornell(10, 100)[1][0]:
    print(*[t.A.e[i] for i in range(3)], *[t.B.e[i] for i in range(3)], *[t.C.e[i] for i in range(3)])
PY
/tmp/bvh_h_check < /tmp/sweep_tris.txt
