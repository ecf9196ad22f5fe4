"""Host check of the BVH traversal-stack bound (rt_bvh.cpp BvhBuild::stack4), CPU only.

r04 admits a tree to the queue kernel's 24-entry LDS stack by an exact bound
(the largest sum over root-to-node paths of internal children - 1) instead of
3 * depth4 + 1.  The kernel does not check the stack pointer,
so an undercount would corrupt a neighbouring lane's stack.
tools/probes/bvh_stack_check.cpp runs bvh_step's push rule as depth-first walks
that hit every child box (entering the first or the last internal child) and
for random rays against the float boxes, and reports each walk's largest stack
size; this test builds it with g++ and checks the bound on the C4 tree, the
sweep mesh and synthetic soups (clustered, wide, thin and duplicate triangles).
"""
import json
import os
import subprocess

import numpy as np
import pytest

from tipe_rt import scenes

from test_bvh_pack import mesh_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K_STACK_Q = 24          # rt_kernels.hip kStackQ
K_STACK4 = 48           # rt_bvh.h kStack4 (the fixed-grid kernel's stacks)


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bvhs") / "bvh_stack_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "tipe-raytracer_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "tools", "probes", "bvh_stack_check.cpp"),
                    os.path.join(ROOT, "tipe-raytracer_amd", "csrc", "rt_bvh.cpp")], check=True)
    return exe


def run(checker, tris, rays=2000):
    text = "\n".join(" ".join(repr(float(x)) for x in row) for row in tris) + "\n"
    p = subprocess.run([checker, str(rays)], input=text, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


def check(rec):
    assert rec["bvh"], rec
    assert rec["all_hit_peak"] <= rec["stack4"] <= 3 * rec["depth4"], rec
    assert rec["ray_peak"] <= rec["stack4"] <= K_STACK4, rec


def test_c4_tree_fits_the_queue_stack(checker):
    rec = run(checker, mesh_rows(scenes.tree_mesh()[0]))
    check(rec)
    # the sweep-SAH tree is 8 levels deep (3 * 8 + 1 > 24) yet needs 20 entries:
    # the exact bound keeps C4 on the queue kernel (test_gpu_instantiations.py)
    assert rec["depth4"] == 8 and rec["stack4"] <= K_STACK_Q, rec


def test_sweep_mesh_bound(checker):
    check(run(checker, mesh_rows(scenes.synthetic_cornell(10, 100)[1][0])))


@pytest.mark.parametrize("seed,n,scale,size,thin", [
    (1, 40, 1.0, 0.1, False),        # just above the 32-triangle BVH threshold
    (2, 600, 50.0, 2.0, False),      # a wide scene
    (3, 2000, 1.0, 0.02, False),     # many small triangles
    (4, 800, 1.0, 0.5, True),        # long thin triangles (heavy box overlap)
    (5, 1500, 0.05, 0.01, False),    # one tight cluster
])
def test_synthetic_soups_bound(checker, seed, n, scale, size, thin):
    rng = np.random.default_rng(seed)
    c = scale * rng.uniform(-1, 1, (n, 3))
    b = c + size * rng.normal(size=(n, 3))
    e = c + (0.01 * size if thin else size) * rng.normal(size=(n, 3))
    rows = np.concatenate([c, b, e], axis=1)
    rows = np.concatenate([rows, rows[:15]])          # duplicate triangles too
    check(run(checker, rows))
