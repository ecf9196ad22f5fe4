"""Where a render_kernel_q round spends its time, phase by phase, at HEAD
(the dynamic counterpart of tools/isa_hist.py's static histogram).

    bash tools/build_variants.sh phase "-DRT_PHASE_CLOCK=1"
    RT_HIP_LIB=tools/variants/phase.so python tools/phase_clock.py [c2,c3,c4,sweep] [spp]

The diagnostic build adds s_memtime reads at the round's wave-uniform points
(rt_kernels.hip RT_PHASE_CLOCK) and writes each wave's cycle sums per phase
into its RT_QUEUE_TRACE record.  With four VALU-bound waves per SIMD a
wave's wall cycles in a phase are in proportion to the issue it takes there,
so the shares are the round's time shares.  One JSON line per scene."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch  # noqa: E402
import tipe_rt  # noqa: E402
from tipe_rt import scenes  # noqa: E402

WORDS = 9
PHASES = ("sphere_cast", "bvh_walk", "resolve_hit", "task_handout", "next_ray_and_finish")


def scene_of(kind):
    if kind == "nature":
        return tipe_rt.make_scene(scenes.main_spheres(), *scenes.nature_mesh()), 10, False
    sph = scenes.cornell_spheres()
    if kind == "c2":
        return tipe_rt.make_scene(sph), 6, False
    if kind == "c4":
        return tipe_rt.make_scene(sph, *scenes.tree_mesh()), 8, True
    if kind == "sweep":
        sph, mesh = scenes.synthetic_cornell(10, 100)
        return tipe_rt.make_scene(sph, *mesh), 6, False
    return tipe_rt.make_scene(sph, *scenes.pyramid_mesh()), 6, False


def run(kind, spp):
    path = os.path.join(ROOT, "gpurun_out", "phase_clock_%s.bin" % kind)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.exists(path):
        os.remove(path)
    sc, bounces, ao = scene_of(kind)
    spec = scenes.NATURE_CAMERA if kind == "nature" else scenes.README_CAMERA
    cam = tipe_rt.init_camera(**{k: spec[k] for k in ("origin", "target", "up", "vfov", "ratio")})
    p = tipe_rt.make_params(1200, 900, spp, bounces, cam, focus=3.0, seed=1010, chunks=32, use_ao=ao, ao=2.5)
    ds = tipe_rt.DeviceScene(sc, 0)
    out = torch.empty((3, 900, 1200, 3), dtype=torch.float64, device="cuda:0")
    os.environ["RT_QUEUE_TRACE"] = path
    tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, 899), out[0].data_ptr(), out[1].data_ptr(),
                         out[2].data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del os.environ["RT_QUEUE_TRACE"]
    d = np.fromfile(path, dtype=np.uint64).reshape(-1, WORDS)
    w = d[::64]                                  # the sums are wave-uniform: lane 0 of each wave
    w = w[w[:, 2] > 0]                           # waves that ran
    ph = w[:, 4:9].astype(np.float64).sum(0)
    rounds = float(w[:, 2].astype(np.float64).sum())
    res = {"scene": kind, "spp": spp, "kernel": tipe_rt.last_render_kernel() if hasattr(tipe_rt, "last_render_kernel")
           else None, "waves": int(len(w)), "rounds_per_wave": rounds / len(w),
           "cycles_per_round": ph.sum() / rounds,
           "share": {k: round(float(v / ph.sum()), 4) for k, v in zip(PHASES, ph)},
           "cycles_per_round_by_phase": {k: round(float(v / rounds), 1) for k, v in zip(PHASES, ph)}}
    os.remove(path)
    return res


if __name__ == "__main__":
    kinds = (sys.argv[1] if len(sys.argv) > 1 else "c2,c3,c4,sweep").split(",")
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    for k in kinds:
        print(json.dumps(run(k, spp or (32 if k in ("c4", "nature") else 128))), flush=True)
