"""BVH trees whose 64-byte binary16 form does not exist.

rt_scene_upload packs the tree a second time into 64-byte nodes (binary16
planes, rt_bvh.cpp pack_bvh_h) for the deep-tree queue kernel.  It refuses
when a coordinate lies beyond binary16's range (65504), a leaf index above
65535 or a leaf holds too many triangles.  Then:
  * a deep tree (the queue kernel's QB 3 instantiation, which walks the
    64-byte nodes) renders with the fixed-grid BVH kernel;
  * a shallow tree (QB 4, which walks the 128-byte nodes anyway) keeps the
    task-queue kernel.
Both must stay bit-exact against the oracle (mesh.h:70-94 through
closest_hit main.c:52-92), and rt_last_render_kernel names the path taken.
"""
import ctypes as C

import numpy as np
import pytest

import helpers
import tipe_rt
from tipe_rt import scenes
from tipe_rt.types import Triangle

from test_gpu_parity import assert_same, gpu_render

pytestmark = pytest.mark.gpu

FAR = 2.0e5      # beyond binary16's 65504, inside the AO / zero-exit gates' 2^20


def with_far_triangle(mesh):
    """The mesh plus one small triangle at z = +FAR (behind the camera,
    outside the README box): it never changes a pixel, but its coordinates
    stop pack_bvh_h."""
    tris, qm, mats, tw, th, nm = mesh
    n = len(tris)
    t2 = (Triangle * (n + 1))()
    q2 = (C.c_int * (n + 1))()
    C.memmove(t2, tris, C.sizeof(Triangle) * n)
    C.memmove(q2, qm, C.sizeof(C.c_int) * n)
    far = t2[n]
    for P, xy in ((far.A, (0.0, 0.0)), (far.B, (1.0, 0.0)), (far.C, (0.0, 1.0))):
        P.e[0], P.e[1], P.e[2] = xy[0], xy[1], FAR
    q2[n] = 0
    return t2, q2, mats, tw, th, nm


def render_and_compare(bundle, p):
    ref = helpers.oracle_render(bundle, p)
    canva, alb, nrm, rad = gpu_render(bundle, p)
    kernel = tipe_rt.last_render_kernel()
    assert_same(canva, ref["canva"], "canva")
    assert_same(rad, ref["radiance"], "radiance")
    assert_same(alb, ref["albedo"], "albedo")
    assert_same(nrm, ref["normal"], "normal")
    return kernel


def test_deep_tree_without_binary16_nodes_takes_fixed_grid():
    bundle = helpers.SceneBundle(scenes.cornell_spheres(),
                                 with_far_triangle(scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE)))
    p = helpers.params(40, 30, 6, 8, use_ao=True, chunks=4)
    assert render_and_compare(bundle, p) == "render_kernel<BVH>"


def test_deep_tree_with_binary16_nodes_takes_queue_qb3():
    """Control: the same tree without the far triangle packs, and runs the
    deep-tree queue kernel (its opaque-material instantiation: the tree's
    texels and the README spheres are opaque, test_gpu_instantiations.py)."""
    p = helpers.params(40, 30, 6, 8, use_ao=True, chunks=4)
    assert render_and_compare(helpers.tree_scene(), p) == "render_kernel_q<QB=3,OP>"


def test_shallow_tree_without_binary16_nodes_keeps_queue_qb4():
    sph, mesh = scenes.synthetic_cornell(10, 100)
    bundle = helpers.SceneBundle(sph, with_far_triangle(mesh))
    p = helpers.params(48, 36, 8, 6, chunks=4)
    assert render_and_compare(bundle, p) == "render_kernel_q<QB=4>"


def test_far_triangle_is_invisible():
    """The appended triangle changes no pixel (so the fallback tests compare
    the same picture as the packed tree)."""
    p = helpers.params(24, 18, 2, 6, chunks=2)
    a = helpers.oracle_render(helpers.tree_scene(), p)["canva"]
    b = helpers.oracle_render(helpers.SceneBundle(scenes.cornell_spheres(), with_far_triangle(
        scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE))), p)["canva"]
    assert np.array_equal(a, b)
