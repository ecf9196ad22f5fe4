#!/bin/bash
# Build tools/variants/a_head.so from git HEAD (a scratch worktree) and
# tools/variants/b_work.so from the working tree, for tools/ab_*.sh.
#   bash tools/build_ab_head.sh [ref]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
REF=${1:-HEAD}
WT=/tmp/rt_ab_head
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f --detach "$WT" "$REF" >/dev/null
mkdir -p "$ROOT/tools/variants"; rm -f "$ROOT"/tools/variants/*.so
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -shared csrc/rt_kernels.hip csrc/rt_api.cpp csrc/rt_bvh.cpp"
src() { [ -f "$1/tipe-raytracer_amd/csrc/rt_rccl.cpp" ] && echo "csrc/rt_rccl.cpp -ldl"; }   # r06 on
(cd "$WT/tipe-raytracer_amd" && /opt/rocm/bin/hipcc $F $(src "$WT") -o "$ROOT/tools/variants/a_head.so") &
(cd "$ROOT/tipe-raytracer_amd" && /opt/rocm/bin/hipcc $F $(src "$ROOT") -o "$ROOT/tools/variants/b_work.so") &
wait
git -C "$ROOT" worktree remove --force "$WT"
ls "$ROOT/tools/variants"
