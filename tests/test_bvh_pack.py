"""Host check of the 64-byte BVH nodes (rt_bvh.cpp pack_bvh_h), CPU only.

The deep-tree queue kernel walks BvhNodeH: binary16 planes relative to a
binary16 node origin, rounded outward.  The kernel's culling is
exact only if every decoded plane pair contains the 128-byte node's float box
and stays within rbox, and if the child and count fields survive the packing.
tools/probes/bvh_h_check.cpp checks exactly that for one mesh; this test builds
it with g++ (rt_bvh.cpp is plain C++) and runs it on the C4 tree, the sweep
mesh, and synthetic meshes.  A packing that does not fit binary16 is reported
as packed = false and is allowed: the kernel then keeps its 128-byte nodes.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from tipe_rt import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bvhh") / "bvh_h_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "tipe-raytracer_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "tools", "probes", "bvh_h_check.cpp"),
                    os.path.join(ROOT, "tipe-raytracer_amd", "csrc", "rt_bvh.cpp")], check=True)
    return exe


def run(checker, tris):
    """tris: (n, 9) array of A, B, C.  Returns the checker's JSON record."""
    text = "\n".join(" ".join(repr(float(x)) for x in row) for row in tris) + "\n"
    p = subprocess.run([checker], input=text, capture_output=True, text=True, timeout=120)
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, rec
    return rec


def mesh_rows(tris):
    return np.array([[t.A.e[0], t.A.e[1], t.A.e[2], t.B.e[0], t.B.e[1], t.B.e[2], t.C.e[0], t.C.e[1], t.C.e[2]]
                     for t in tris])


def test_c4_tree_nodes_contain_their_boxes(checker):
    rec = run(checker, mesh_rows(scenes.tree_mesh()[0]))
    assert rec["packed"] and rec["violations"] == 0
    assert rec["nodes"] > 100 and rec["volume_growth"] < 1.01


def test_sweep_mesh_nodes_contain_their_boxes(checker):
    rec = run(checker, mesh_rows(scenes.synthetic_cornell(10, 100)[1][0]))
    assert rec["packed"] and rec["violations"] == 0


@pytest.mark.parametrize("seed,center,scale,size", [
    (1, 0.0, 1.0, 0.1),          # a soup around the origin
    (2, 0.0, 50.0, 2.0),         # a wide scene
    (3, 3.7, 0.01, 1e-4),        # tiny triangles off the origin
    (4, -250.0, 5.0, 0.3),       # far from the origin: coarse binary16 origins
    (5, 0.0, 1.0, 0.0),          # degenerate (point) triangles
    (6, 1e6, 1.0, 0.1),          # beyond binary16's range: must refuse to pack
])
def test_synthetic_meshes_pack_conservatively(checker, seed, center, scale, size):
    rng = np.random.default_rng(seed)
    n = 600
    c = center + scale * rng.uniform(-1, 1, (n, 3))
    rows = np.concatenate([c, c + size * rng.normal(size=(n, 3)), c + size * rng.normal(size=(n, 3))], axis=1)
    rows = np.concatenate([rows, rows[:20]])          # duplicate triangles (ties) too
    rec = run(checker, rows)
    assert rec["packed"] == (abs(center) < 1e4), rec
    if rec["packed"]:
        assert rec["violations"] == 0, rec
