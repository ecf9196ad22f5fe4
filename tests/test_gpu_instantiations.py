"""Which task-queue instantiation a scene takes, and that each is bit-exact.

r04 splits render_kernel_q by what the scene can reach (DESIGN §4a
"Instantiations"):
  * QB = -2: spheres only, every material opaque -- no triangle scan, no
    alpha-hole or refraction branch compiled in (the C2 bench scene);
  * QB = -1: spheres only, some material transparent or a hole;
  * QB = 0: spheres and brute-force triangles (<= 32, no BVH);
  * QB = 3 with OPQ: the deep-tree kernel when every sphere material, every
    texel and every material index (no 3 or 4, tri_material's overrides)
    is opaque (C4).
The host picks them (rt_kernels.hip launch_render) from the scene upload's
material flags.  main.c:196-234 decides per hit: alpha < 0.0001 is a hole,
alpha <= 0.99 refracts, anything else (NaN included) shades; the opaque
gate is exactly "no material takes either of the first two branches", so a
material at alpha = 0.99 must keep the refraction code and one just above
it must not.  Every render is compared with the oracle bit for bit.
"""
import pytest

import helpers
import tipe_rt
from tipe_rt import scenes

from test_gpu_bvh_fallback import render_and_compare

pytestmark = pytest.mark.gpu


def one_transparent(alpha):
    """README box plus one extra small sphere of the given alpha in view."""
    extra = [((0.1, -0.9, -1.8), 0.3, scenes.material((0.8, 0.8, 0.8), alpha=alpha, ior=1.5))]
    return helpers.SceneBundle(scenes.cornell_spheres(extra=extra))


P = dict(W=40, H=30, spp=8, bounces=6)


def prm(**kw):
    q = dict(P)
    q.update(kw)
    return helpers.params(q["W"], q["H"], q["spp"], q["bounces"], chunks=4)


def test_opaque_sphere_scene_takes_qb_minus2():
    assert render_and_compare(helpers.cornell(), prm()) == "render_kernel_q<QB=-2>"


@pytest.mark.parametrize("alpha", [0.5, 0.99, 0.00005, 0.0])
def test_transparent_or_hole_sphere_takes_qb_minus1(alpha):
    assert render_and_compare(one_transparent(alpha), prm()) == "render_kernel_q<QB=-1>"


def test_alpha_just_above_refraction_threshold_is_opaque():
    assert render_and_compare(one_transparent(0.9900001), prm()) == "render_kernel_q<QB=-2>"


def test_whole_box_transparent_takes_qb_minus1():
    bundle = helpers.SceneBundle(scenes.cornell_spheres(alpha=0.5))
    assert render_and_compare(bundle, prm()) == "render_kernel_q<QB=-1>"


def test_triangle_scene_takes_qb0():
    assert render_and_compare(helpers.pyramid_scene(), prm()) == "render_kernel_q<QB=0>"


def test_tree_scene_takes_deep_tree_opaque_instantiation():
    """C4: README spheres + the 1320-triangle tree, all opaque."""
    p = helpers.params(40, 30, 6, 8, use_ao=True, chunks=4)
    assert render_and_compare(helpers.tree_scene(), p) == "render_kernel_q<QB=3,OP>"


def test_tree_scene_with_transparent_sphere_keeps_qb3():
    extra = [((0.1, -0.9, -1.8), 0.3, scenes.material((0.8, 0.8, 0.8), alpha=0.5, ior=1.5))]
    bundle = helpers.SceneBundle(scenes.cornell_spheres(extra=extra),
                                 scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE))
    p = helpers.params(40, 30, 6, 8, use_ao=True, chunks=4)
    assert render_and_compare(bundle, p) == "render_kernel_q<QB=3>"


@pytest.mark.parametrize("mat_index", [3, 4])
def test_tree_with_override_material_keeps_qb3(mat_index):
    """tri_material's material indices 3 and 4 force alpha 0.1 / 0.6 whatever
    the texel holds: a tree whose first triangles use one of them is not
    opaque.  The texel table gets entries up to that index (copies of
    material 0), so the scene stays valid."""
    tris, qm, mats, tw, th, nm = scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE)
    from tipe_rt.types import Material
    n_new = max(nm, mat_index + 1)
    mats2 = (Material * (n_new * tw * th))()
    for k in range(n_new * tw * th):
        mats2[k] = mats[k] if k < nm * tw * th else mats[0]
    for k in range(0, len(tris), 7):
        qm[k] = mat_index
    bundle = helpers.SceneBundle(scenes.cornell_spheres(), (tris, qm, mats2, tw, th, n_new))
    p = helpers.params(40, 30, 6, 8, use_ao=True, chunks=4)
    assert render_and_compare(bundle, p) == "render_kernel_q<QB=3>"


@pytest.mark.parametrize("scene", ["tree", "sweep", "mineways", "nature", "main_regime"])
def test_bvh_stack_bound_holds_on_the_gpu(scene):
    """rt_count_async checks every BVH push against the LDS stack of the
    kernel launch_render picks for the tree (rt.h RT_CNT_BVH_STACK_OVER):
    the C4 tree (deep-tree queue kernel, 24 entries), the 100-triangle sweep
    mesh and mineways (606 triangles), over a whole frame with AO."""
    from test_gpu_parity import assert_stack_bound_holds
    if scene == "tree":
        bundle = helpers.tree_scene()
    elif scene == "mineways":
        bundle = helpers.mineways_scene()
    elif scene in ("nature", "main_regime"):       # 5812 triangles, stack4 22 / main()'s scale
        bundle = helpers.nature_scene() if scene == "nature" else helpers.main_regime_scene()
        p = helpers.params(120, 90, 4, 10, use_ao=True, ao=2.5, chunks=4,
                           cam=helpers.camera_of(scenes.NATURE_CAMERA if scene == "nature" else scenes.MAIN_CAMERA))
        c = assert_stack_bound_holds(bundle, p)
        assert c[tipe_rt.types.RT_CNT_BVH_NODES] > 0
        return
    else:
        sph, mesh = scenes.synthetic_cornell(10, 100)
        bundle = helpers.SceneBundle(sph, mesh)
    p = helpers.params(120, 90, 4, 8, use_ao=True, ao=2.5, chunks=4)
    c = assert_stack_bound_holds(bundle, p)
    assert c[tipe_rt.types.RT_CNT_BVH_NODES] > 0          # the tree was walked


def _nature(opaque, far_z=4e4):
    """RTX_MAP/nature plus one 0.1-unit triangle at z = far_z, behind the
    camera: the triangles' coordinate bound R_b becomes 4e4, which widens
    every box's padding, and the tree's exact stack bound becomes 26."""
    from tipe_rt.types import Triangle
    import ctypes as C
    tris, qm, mats, tw, th, nm = scenes.nature_mesh()
    n = len(tris)
    t2, q2 = (Triangle * (n + 1))(), (C.c_int * (n + 1))()
    C.memmove(t2, tris, C.sizeof(Triangle) * n)
    C.memmove(q2, qm, C.sizeof(C.c_int) * n)
    for P, xy in ((t2[n].A, (0.0, 0.0)), (t2[n].B, (0.1, 0.0)), (t2[n].C, (0.0, 0.1))):
        P.e[0], P.e[1], P.e[2] = xy[0], xy[1], far_z
    q2[n] = 0
    if opaque:                          # every texel at alpha 1, no material index 3 / 4 override
        for k in range(len(mats)):
            mats[k].alpha = 1.0
        for k in range(n + 1):
            if q2[k] in (3, 4):
                q2[k] = 0
    return helpers.SceneBundle(scenes.main_spheres(), (t2, q2, mats, tw, th, nm))


@pytest.mark.parametrize("opaque", [False, True])
def test_tree_with_stack_bound_above_24_keeps_the_queue_kernel(opaque):
    """A tree whose exact stack bound is 26 (> 24, _nature above).  The
    non-opaque deep-tree kernel has 32 LDS stack entries (kStackQN; 38 KiB
    per block, still 4 blocks per CU), so it takes such trees -- an opaque
    one too, instead of the 24-entry OPQ kernel -- rather than the fixed
    grid; every push stays inside (RT_CNT_BVH_STACK_OVER == 0), bit for bit
    vs the oracle."""
    from test_gpu_parity import assert_stack_bound_holds
    bundle = _nature(opaque)
    p = helpers.params(32, 24, 4, 10, chunks=4, cam=helpers.camera_of(scenes.NATURE_CAMERA))
    assert render_and_compare(bundle, p) == "render_kernel_q<QB=3>"
    assert_stack_bound_holds(bundle, p)
