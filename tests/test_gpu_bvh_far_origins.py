"""BVH walks from ray origins beyond the tree's padding radius (r06).

rt_scene_upload pads every triangle's box for ray origins within R_b, the
triangles' own coordinate bound (rt_bvh.cpp; the padding is a first-order
rounding bound of mesh.h:70-94 that grows with |o|).  A ray from farther out
-- the camera, a hit point on one of the README box's radius-500 walls, on
main.c:346's radius-1e5 sky sphere -- widens its own slab margins by
k_delta (|o|_inf - R_b) and its distance slack to s_rel |o|_inf
(rt_kernels.hip ray32).  Before r06 R_b also covered every sphere, so a sky
sphere fattened every box, and a camera outside R_b sent the whole launch to
the every-triangle scan.  Each case is bit for bit against the oracle (whose
scan has no BVH), with the zero-throughput exit off where rays must leave
the sky sphere, and with the stack bound checked on the GPU."""
import pytest

import helpers
import tipe_rt
from tipe_rt import scenes
from tipe_rt.types import Sphere, Vec3

from test_gpu_bvh_fallback import render_and_compare
from test_gpu_parity import assert_stack_bound_holds

pytestmark = pytest.mark.gpu


def with_sky(spheres, radius=1e5, diffuse=(0.0, 0.0, 0.0)):
    """The spheres plus main.c:346's sky sphere (emission SKY, strength 1),
    last; a non-black diffuse keeps paths alive after a sky hit."""
    n = len(spheres)
    arr = (Sphere * (n + 1))()
    for k in range(n):
        arr[k] = spheres[k]
    arr[n].center = Vec3(0.0, 0.0, 0.0)
    arr[n].radius = radius
    arr[n].mat = scenes.material(diffuse, scenes.SKY, 1.0, 0.0, 1.0, 1.0)
    return arr


def test_camera_outside_the_tree_bound_walks_the_bvh():
    """The C4 tree lit by main.c:345's sun alone, camera at z = 6 (beyond the
    tree's R_b ~ 3): the deep-tree queue kernel with per-ray margins (its
    non-opaque instantiation: the OPQ one has no far-origin margins), not the
    brute-force scan the launch took before r06."""
    cam = tipe_rt.init_camera((0.3, 0.2, 6.0), (0.2, -0.5, -2.1), (0, 1, 0), 40.0, 4.0 / 3.0)
    p = helpers.params(40, 30, 6, 8, use_ao=True, chunks=4, cam=cam)
    sun = (Sphere * 1)(scenes.main_spheres()[0])
    bundle = helpers.SceneBundle(sun, scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE))
    assert render_and_compare(bundle, p) == "render_kernel_q<QB=3>"
    assert_stack_bound_holds(bundle, p)


def test_opaque_tree_without_far_origins_keeps_the_opq_kernel():
    """Control: the C4 scene itself (camera and walls inside R_b = 1001)."""
    p = helpers.params(40, 30, 6, 8, use_ao=True, chunks=4)
    assert render_and_compare(helpers.tree_scene(), p) == "render_kernel_q<QB=3,OP>"


@pytest.mark.parametrize("ao", [False, True])
def test_rays_from_the_sky_sphere_walk_the_bvh(ao):
    """The C4 tree in the README box under a radius-1e5 sky whose diffuse
    colour is not black, zero-throughput exit off: rays escaping the open
    box hit the sky and bounce on from |o| ~ 1e5 (and AO rays start there)."""
    bundle = helpers.SceneBundle(with_sky(scenes.cornell_spheres(), diffuse=(0.5, 0.6, 0.7)),
                                 scenes.moved(scenes.load_tree_fixture(), scenes.TREE_MOVE))
    p = helpers.params(40, 30, 6, 6, use_ao=ao, ao=2.5, chunks=4)
    with tipe_rt.reference_counts():            # zero-throughput exit off for the render too
        render_and_compare(bundle, p)
    assert_stack_bound_holds(bundle, p)


def test_nature_under_the_sky_zero_exit_off():
    """RTX_MAP/nature under main.c:346's black sky, zero-throughput exit off:
    every sky hit continues from |o| ~ 1e5 through the 5812-triangle tree."""
    p = helpers.params(24, 18, 4, 10, chunks=4, cam=helpers.camera_of(scenes.NATURE_CAMERA))
    with tipe_rt.reference_counts():
        assert render_and_compare(helpers.nature_scene(), p) == "render_kernel_q<QB=3>"


def test_far_camera_on_a_scaled_mesh():
    """main()'s regime the other way round: the tree scaled by 200 and viewed
    from |o| ~ 3000 (far outside R_b), sky sphere behind."""
    tris, qm, mats, tw, th, nm = scenes.load_tree_fixture()
    for t in tris:
        for P in (t.A, t.B, t.C):
            P.e[0], P.e[1], P.e[2] = 200 * P.e[0], 200 * P.e[1] - 100, 200 * P.e[2]
    bundle = helpers.SceneBundle(with_sky(scenes.main_spheres()[:1]), (tris, qm, mats, tw, th, nm))
    cam = tipe_rt.init_camera((800.0, 600.0, -2900.0), (0.0, 60.0, 0.0), (0, 1, 0), 12.0, 4.0 / 3.0)
    p = helpers.params(32, 24, 4, 8, chunks=4, cam=cam)
    k = render_and_compare(bundle, p)
    assert k.startswith("render_kernel_q<QB=3")
    assert_stack_bound_holds(bundle, p)
