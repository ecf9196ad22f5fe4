"""Kernel rates of the render path on every BASELINE single-frame scene
(SURVEY.md §8 "Config resolution"), one JSON line per config.

    python tools/bench_configs.py [--spp-scale F] [--only C3,C4]

bench.py's headline is C2 only; this reports the mesh scenes beside it (the
rows §8(f-2) acceleration targets) and C5's 4K frame (3840x2880, C3 scene;
`full_frame_s_on_config_gpus_linear` divides by the config's GPU count,
which the row tiling achieves up to the gather).  Full frames at a reduced spp
(Msamples/s is spp-independent: pixels are independent and the per-sample
work does not depend on S); spp_chunks RT_SPP_CHUNKS_AUTO as bench.py (so
--spp sets the task size: S/32 samples per slice from 32 spp on); kernel
time from HIP events on the launch stream, events/sample from rt_count_async
at 4 spp.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))

import torch  # noqa: E402  (before librt_hip.so)

import tipe_rt  # noqa: E402
from tipe_rt import scenes  # noqa: E402

CONFIGS = {
    # name: (mesh builder or None, spp measured, bounces, useAO, AO_intensity, full spp, W, H, GPUs of the config)
    "C2": (None, 200, 6, False, 2.5, 1000, 1200, 900, 1),
    "C3": (scenes.pyramid_mesh, 200, 6, False, 2.5, 1000, 1200, 900, 1),
    "C4": (scenes.tree_mesh, 16, 8, True, 2.5, 2000, 1200, 900, 4),
    # C5: 4K frame of the C3 scene (SURVEY.md §8 config resolution), 5000 spp over 8 GPUs
    "C5": (scenes.pyramid_mesh, 20, 6, False, 2.5, 5000, 3840, 2880, 8),
    # roofline-sweep scene: README box + 10 random spheres... (synthetic_cornell(10, 100))
    "SWEEP": ("sweep", 32, 6, False, 2.5, 32, 1200, 900, 1),
    # the reference's RTX_MAP/nature scene at its own settings (1000 rays, nbRebondMax 10)
    "NATURE": (scenes.nature_mesh, 64, 10, False, 2.5, 1000, 1200, 900, 1),
}


def run(name, spp_scale, dev, stream, spp_override=0, chunks=None):
    mesh_fn, spp, bounces, ao, ao_int, full_spp, W, H, gpus = CONFIGS[name]
    spp = spp_override or max(1, int(spp * spp_scale))
    spheres = scenes.main_spheres() if name == "NATURE" else scenes.cornell_spheres()
    if mesh_fn == "sweep":
        spheres, (tris, qm, mats, tw, th, nm) = scenes.synthetic_cornell(10, 100)
        scene = tipe_rt.make_scene(spheres, tris, qm, mats, tw, th, nm)
        nt = len(tris)
    elif mesh_fn is None:
        scene = tipe_rt.make_scene(spheres)
        nt = 0
    else:
        tris, qm, mats, tw, th, nm = mesh_fn()
        scene = tipe_rt.make_scene(spheres, tris, qm, mats, tw, th, nm)
        nt = len(tris)
    spec = scenes.NATURE_CAMERA if name == "NATURE" else scenes.README_CAMERA
    cam = tipe_rt.init_camera(**{k: spec[k] for k in ("origin", "target", "up", "vfov", "ratio")})
    p = tipe_rt.make_params(W, H, spp, bounces, cam, focus=3.0, use_ao=ao, ao=ao_int,
                            chunks=tipe_rt.RT_SPP_CHUNKS_AUTO if chunks is None else chunks)
    ds = tipe_rt.DeviceScene(scene, dev.index)
    tiling = tipe_rt.band_tiling(0, H - 1)
    out = torch.empty((3, H, W, 3), dtype=torch.float64, device=dev)
    sptr = stream.cuda_stream

    def launch():
        tipe_rt.render_async(ds, p, tiling, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), None, sptr)

    launch()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    n = 2
    t0 = time.perf_counter()
    ev[0].record(stream)
    for _ in range(n):
        launch()
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / n
    ms = ev[0].elapsed_time(ev[1]) / n
    kname = tipe_rt.last_render_kernel()
    pc = tipe_rt.make_params(W, H, 4, bounces, cam, focus=3.0, use_ao=ao, ao=ao_int)
    d_cnt = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device=dev)
    tipe_rt.count_async(ds, pc, tiling, d_cnt.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    cnt = [int(x) for x in d_cnt.cpu()]
    ds.close()
    samples = W * H * spp
    rate = samples / (ms * 1e-3) / 1e6
    return {"config": name, "kernel": kname, "width": W, "height": H, "triangles": nt, "spheres": len(spheres), "bounces": bounces,
            "ao": ao, "spp_measured": spp, "kernel_ms": round(ms, 3), "wall_ms": round(wall * 1e3, 3),
            "kernel_msamples_per_s": round(rate, 3),
            "full_frame_s_at_config_spp": round(W * H * full_spp / (rate * 1e6), 2),
            "config_gpus": gpus, "spp_chunks": tipe_rt.types.rt_resolve_spp_chunks(p.spp_chunks, spp),
            "full_frame_s_on_config_gpus_linear": round(W * H * full_spp / (rate * 1e6) / gpus, 2),
            "events_per_sample": {k: round(cnt[i] / max(cnt[0], 1), 7) for i, k in enumerate(tipe_rt.COUNTER_NAMES)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp-scale", type=float, default=1.0)
    ap.add_argument("--only", default=",".join(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="spp of every config (default: the table's, x --spp-scale)")
    ap.add_argument("--chunks", type=int, default=None, help="rt_params.spp_chunks (default RT_SPP_CHUNKS_AUTO)")
    ap.add_argument("--full-spp", action="store_true", help="each config at its full spp")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    for name in args.only.split(","):
        spp = CONFIGS[name][5] if args.full_spp else args.spp
        print(json.dumps(run(name, args.spp_scale, dev, stream, spp, args.chunks)), flush=True)


if __name__ == "__main__":
    main()
