"""Scenes beyond the candidate pass's 16-bit sphere slot.

The sphere candidate pass tags each running minimum with its sphere slot in
16 mantissa bits (rt_kernels.hip spheres_closest, RT_CAND_TAG).  Above 65534
spheres the upload switches that pass off (cand_lmax = +inf, ns_cand = 0)
and every cast takes the exact reference scan (main.c:59-78) -- the
reference itself has no sphere limit.  Both sides of the threshold must
render bit for bit like the oracle, through every kernel family a sphere
scene can take.
"""
import numpy as np
import pytest

import helpers
from tipe_rt import scenes
from tipe_rt.types import Sphere, Vec3
from test_gpu_parity import check_parity

pytestmark = pytest.mark.gpu


def _many(n, seed=5):
    """README box + (n - 10) small spheres: a visible grid of mirrors /
    lights / diffuse balls in front of the camera, the rest far behind it."""
    base = scenes.cornell_spheres()
    rng = np.random.default_rng(seed)
    sph = (Sphere * n)()
    for k in range(len(base)):
        sph[k] = base[k]
    for k in range(len(base), n):
        if k < len(base) + 400:
            c = rng.uniform([-1.5, -1.2, -4.0], [1.5, 1.2, -1.5])
            r = float(rng.uniform(0.02, 0.08))
        else:                                   # behind the camera, each still tested by every cast
            c = rng.uniform([-50, -50, 5], [50, 50, 60])
            r = float(rng.uniform(0.01, 0.3))
        kind = k % 3
        m = scenes.material(tuple(rng.uniform(0, 1, 3)),
                            tuple(rng.uniform(0.2, 1, 3)) if kind == 1 else (0, 0, 0),
                            2.0 if kind == 1 else 0.0, 0.9 if kind == 2 else 0.0, 1.0, 1.0)
        sph[k].center = Vec3(*c)
        sph[k].radius = r
        sph[k].mat = m
    return helpers.SceneBundle(sph)


@pytest.mark.parametrize("n", [65534, 65535, 70001])
@pytest.mark.parametrize("chunks", [1, 2])
def test_many_spheres_bitexact(n, chunks):
    """chunks 1: the fixed-grid kernel; 2: the persistent queue kernel."""
    bundle = _many(n)
    p = helpers.params(12, 9, 2, 4, chunks=chunks)
    check_parity(bundle, p)


def test_many_spheres_with_ao_bitexact():
    bundle = _many(65537, seed=9)
    p = helpers.params(10, 8, 2, 3, use_ao=True, ao=2.5, chunks=2)
    check_parity(bundle, p)
