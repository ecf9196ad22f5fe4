"""Per-rank compute rate of the bench frame (C2) for N = 1, 2, 4, 8: renders
rank 0's cyclic 2-row tiles of an N-way split on this one GPU and reports
Msamples/s of that share.  Predicts the compute part of strong scaling (the
gather is not included); usage: python tools/rank_share_rate.py [--spp S]."""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import torch
import tipe_rt
from tipe_rt import scenes

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--chunks", type=int, default=32)
ap.add_argument("--pipeline", action="store_true", help="alternate two streams (bench.py default)")
ap.add_argument("--tile-rows", type=int, default=2)
args = ap.parse_args()
W, H = 1200, 900
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
p = tipe_rt.make_params(W, H, args.spp, 6, cam, focus=3.0, seed=1010, chunks=args.chunks)
ds = tipe_rt.DeviceScene(tipe_rt.make_scene(scenes.cornell_spheres()), 0)
st = torch.cuda.current_stream().cuda_stream
base = None
for n in (1, 2, 4, 8):
    t = tipe_rt.band_tiling(0, H - 1) if n == 1 else tipe_rt.cyclic_tiling(H, args.tile_rows, 0, n)
    rows = t.n_tiles * t.tile_rows
    nb = 2 if args.pipeline else 1
    outs = [torch.empty((3, rows, W, 3), dtype=torch.float64, device="cuda:0") for _ in range(nb)]
    sts = [torch.cuda.Stream() for _ in range(nb)] if args.pipeline else [torch.cuda.current_stream()]
    def frame(k):
        o, s_ = outs[k % nb], sts[k % nb]
        tipe_rt.render_async(ds, p, t, o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), None, s_.cuda_stream)
    frame(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.reps):
        frame(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    valid = sum(1 for lt in range(t.n_tiles) for y in range(t.tile_rows)
                if t.row_base + (t.tile_first + lt * t.tile_step) * t.tile_rows + y < H)
    rate = valid * W * args.spp / dt / 1e6
    base = base or rate
    print(json.dumps({"chunks": args.chunks, "pipeline": args.pipeline, "n": n, "rows": valid, "ms": round(dt * 1e3, 3), "msamples_per_s_share": round(rate, 1),
                      "efficiency_vs_n1": round(rate / base, 4)}), flush=True)
ds.close()
