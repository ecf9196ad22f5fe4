"""SURVEY.md §8(d) roofline sweep: synthetic Cornell scenes with N spheres in
{10, 32, 128} and N triangles in {0, 100, 1000} (tipe_rt.scenes.
synthetic_cornell), 1200x900, 6 bounces, --spp samples (chunks 8).  Reports
Msamples/s, the kernel's own event counts per sample and executed
algorithmic FP64 FLOPs against the FP64 vector peak.  FLOPs per sample:
40 + C(25 Ns + 18) + 40 tri_tests + 48 bvh_nodes + 5 D + 100 shade + 80 tex +
40 refract, with tri_tests the triangle tests done (brute force: C Nt; BVH:
leaf tests) and 4 slab tests of 12 FLOPs per BVH node.  Parity of these
scenes: tests/test_gpu_parity.py::test_synthetic_sweep_scenes_bitexact."""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch
import tipe_rt
from tipe_rt import scenes

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--only", default="", help="Ns:Nt[,Ns:Nt...] subset")
args = ap.parse_args()
W, H, B = 1200, 900, 6
PEAK = 78.6
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
st = torch.cuda.current_stream().cuda_stream
T = tipe_rt.types
grid = [(ns, nt) for ns in (10, 32, 128) for nt in (0, 100, 1000)]
if args.only:
    grid = [tuple(int(v) for v in x.split(":")) for x in args.only.split(",")]
for ns, nt in grid:
    if True:
        sph, mesh = scenes.synthetic_cornell(ns, nt)
        scene = tipe_rt.make_scene(sph, *mesh) if mesh else tipe_rt.make_scene(sph)
        ds = tipe_rt.DeviceScene(scene, 0)
        p = tipe_rt.make_params(W, H, args.spp, B, cam, focus=3.0, seed=1010, chunks=8)
        out = torch.empty((3, H, W, 3), dtype=torch.float64, device="cuda:0")
        tiling = tipe_rt.band_tiling(0, H - 1)
        tipe_rt.render_async(ds, p, tiling, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), None, st)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(args.reps):
            tipe_rt.render_async(ds, p, tiling, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), None, st)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / args.reps
        pc = tipe_rt.make_params(W, H, 4, B, cam, focus=3.0, seed=1010)
        d = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device="cuda:0")
        tipe_rt.count_async(ds, pc, tiling, d.data_ptr(), st)
        torch.cuda.synchronize()
        c = [int(x) for x in d.cpu()]
        s = max(c[T.RT_CNT_SAMPLES], 1)
        bvh = c[T.RT_CNT_BVH_NODES] > 0
        tri_done = c[T.RT_CNT_BVH_TRI_TESTS] if bvh else c[T.RT_CNT_TRI_TESTS]
        f = (40 * s + c[T.RT_CNT_CASTS] * (25 * ns + 18) + 40 * tri_done + 48 * c[T.RT_CNT_BVH_NODES]
             + 5 * c[T.RT_CNT_SPHERE_DISC] + 100 * c[T.RT_CNT_SHADE] + 80 * c[T.RT_CNT_TEX_HITS]
             + 40 * c[T.RT_CNT_REFRACT]) / s
        rate = W * H * args.spp / (ms * 1e-3) / 1e6
        tf = rate * 1e6 * f / 1e12
        print(json.dumps({"spheres": ns, "triangles": nt, "bvh": bvh, "spp": args.spp, "ms": round(ms, 3),
                          "msamples_per_s": round(rate, 1), "casts_per_sample": round(c[T.RT_CNT_CASTS] / s, 3),
                          "tri_tests_per_sample": round(tri_done / s, 2),
                          "bvh_nodes_per_sample": round(c[T.RT_CNT_BVH_NODES] / s, 2),
                          "flops_per_sample": round(f, 1), "tflops": round(tf, 3), "frac": round(tf / PEAK, 4)}),
              flush=True)
        ds.close()
