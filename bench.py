#!/usr/bin/env python3
"""bench.py — Msamples/s of the MI355X render path on BASELINE config C2.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

One step = one full frame of config C2 (README 10-sphere Cornell box,
1200x900, 1000 spp, 6 bounces; Philox stream, seed 1010) rendered into HBM.
With N > 1 (launched one rank per GPU by torch.distributed.run) the frame is
split into cyclic 2-row tiles (tile t -> rank t mod N), each rank renders its
tiles, the tiles are gathered to rank 0 over RCCL (torch.distributed.gather,
backend "nccl") and rank 0 un-permutes them (rt_assemble_async): total work
per step is fixed, so scaling is "strong".

Rank 0 prints ONE JSON line.  `roofline` prices the render kernel against
the FP64 vector peak: algorithmic FLOPs per launch = the per-sample formula
of SURVEY.md §8(d) evaluated on event counts from rt_count_async (a counting
pass outside the timed region), divided by the kernel's mean duration from
HIP events on the launch stream.  `cpu_baseline` times the CPU restatement
(oracle/, Philox stream, pthreads, rank 0 at N = 1 only) on a bounded sample
of the same frame.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (before librt_hip.so: share torch's HIP runtime)
import torch.distributed as dist  # noqa: E402

import tipe_rt  # noqa: E402
from tipe_rt import scenes  # noqa: E402

METRIC = "Msamples/s (pixels×spp/s) at 1200×900, 1000spp, 6 bounces; 1/2/4/8 GPU"
W, H, SPP, BOUNCES, SEED = 1200, 900, 1000, 6, 1010
TILE_ROWS = 2        # cyclic 2-row tiles: 450 tiles, the busiest of 8 ranks renders 57 (98.7 % balance;
                     # 8-row tiles left one rank 15 of 113, 94 %)
FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X FP64 vector, AMD spec (= 1/2 of the 157.3 FP32 vector peak)
HBM_PEAK_GBS = 8000.0


def flops_per_launch(cnt, ns, nt):
    """F = 40 + C(25 Ns + 40 Nt + 18) + 5 D + 100 Bn + 80 T + 40 R per sample."""
    s, casts, disc, shade, tex, refr = (cnt[i] for i in (0, 1, 3, 5, 6, 7))   # rt.h RT_CNT_*
    return 40 * s + casts * (25 * ns + 40 * nt + 18) + 5 * disc + 100 * shade + 80 * tex + 40 * refr


def valid_rows(t):
    """Global rows (< H) a tiling renders (rt.h rt_tiling)."""
    return sum(1 for lt in range(t.n_tiles) for y in range(t.tile_rows)
               if t.row_base + (t.tile_first + lt * t.tile_step) * t.tile_rows + y < H)


def load_pmc_traffic():
    """HBM bytes per render launch from the committed rocprofv3 --pmc pass, or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("render_kernel_hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(p, scene_bundle, threads=12):
    """Oracle (CPU restatement, Philox stream = per-pixel, i.e. the 'fair'
    per-thread RNG) with `threads` pthreads on 5 bands of `threads` rows of
    the C2 frame at the full 1000 spp."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi
    o = oracle_ffi.oracle()
    canva = np.zeros((H, W, 3))
    starts = [100, 250, 400, 550, 700, 850]
    t0 = time.perf_counter()
    for lo in starts:
        rc = o.oracle_render_rows(C.byref(scene_bundle), C.byref(p), lo + threads - 1, lo, threads, 0,
                                  canva.ctypes.data, None, None, None, None)
        assert rc == 0
    dt = time.perf_counter() - t0
    samples = len(starts) * threads * W * SPP
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "%d bands x %d rows of the 1200x900 C2 frame at 1000 spp (%d samples, %.1f s), "
                      "oracle/rt_oracle.c, Philox per-pixel stream, %d pthreads over contiguous row bands "
                      "(main.c:407-449)" % (len(starts), threads, samples, dt, threads),
            "host_nproc": os.cpu_count()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=12)
    ap.add_argument("--chunks", type=int, default=int(os.environ.get("RT_BENCH_CHUNKS", "32")),
                    help="rt_params.spp_chunks (fixed slice grouping of each pixel's samples; the same "
                         "for every N, so the image does not depend on the GPU count)")
    ap.add_argument("--verify", action="store_true",
                    help="N>1: rank 0 re-renders the frame alone and checks the assembled planes bit for bit")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one stream: frame k+1 starts after frame k (default: two streams, see step())")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: gather through host copies (rehearsing N>1 with all ranks on one GPU); "
                         "nccl (= RCCL) is the measured configuration")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = local_rank if args.dist_backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(gpu)
        dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    spheres = scenes.cornell_spheres()
    scene = tipe_rt.make_scene(spheres)
    cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
    p = tipe_rt.make_params(W, H, SPP, BOUNCES, cam, focus=3.0, seed=SEED, chunks=args.chunks)
    ds = tipe_rt.DeviceScene(scene, gpu)

    if world == 1:
        tiling = tipe_rt.band_tiling(0, H - 1)
    else:
        tiling = tipe_rt.cyclic_tiling(H, TILE_ROWS, rank, world)
    rows = tiling.n_tiles * tiling.tile_rows
    # Frames alternate between two streams with their own buffers, so frame
    # k+1's persistent render blocks start on the CUs that frame k's last
    # tasks leave idle (the queue kernel's tail); stream order
    # keeps frame k+2 behind frame k's gather and assembly.
    nbuf = 1 if args.no_pipeline else 2
    streams = [stream] if nbuf == 1 else [torch.cuda.Stream(dev) for _ in range(nbuf)]
    # frame planes: canva | albedo | normal (the reference's three outputs)
    locals_ = [torch.empty((3, rows, W, 3), dtype=torch.float64, device=dev) for _ in range(nbuf)]
    gathered_ = gather_lists = fulls = [None] * nbuf
    if world > 1 and rank == 0:
        gathered_ = [torch.empty((world, 3, rows, W, 3), dtype=torch.float64, device=dev) for _ in range(nbuf)]
        gather_lists = [[g[r] for r in range(world)] for g in gathered_]
        fulls = [torch.empty((3, H, W, 3), dtype=torch.float64, device=dev) for _ in range(nbuf)]
    last = [0]

    def step(k):
        b = k % nbuf
        last[0] = b
        st = streams[b]
        local, gathered, gather_list, full = locals_[b], gathered_[b], gather_lists[b], fulls[b]
        with torch.cuda.stream(st):
            tipe_rt.render_async(ds, p, tiling, local[0].data_ptr(), local[1].data_ptr(), local[2].data_ptr(),
                                 None, st.cuda_stream)
            if world > 1:
                if args.dist_backend == "nccl":
                    dist.gather(local, gather_list, dst=0)     # RCCL over xGMI
                else:
                    host = [torch.empty_like(local, device="cpu") for _ in range(world)] if rank == 0 else None
                    dist.gather(local.cpu(), host, dst=0)
                    if rank == 0:
                        for r in range(world):
                            gathered[r].copy_(host[r])
                if rank == 0:
                    for pl in range(3):                     # (world, plane, rows, W, 3) -> (plane, H, W, 3)
                        tipe_rt.assemble_async(gathered[0, pl].data_ptr(), world, TILE_ROWS, rows, W, H,
                                               full[pl].data_ptr(), st.cuda_stream, rank_stride=3 * rows * W)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    verified = None
    if args.verify and world > 1 and rank == 0:
        ref = torch.empty((3, H, W, 3), dtype=torch.float64, device=dev)
        tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, H - 1), ref[0].data_ptr(), ref[1].data_ptr(),
                             ref[2].data_ptr(), None, sptr)
        torch.cuda.synchronize(dev)
        used = fulls[:min(nbuf, args.warmup + args.steps)]            # every buffer that held a frame
        verified = all(bool(torch.equal(ref, f)) for f in used)
        if not verified:
            print("verify: assembled frame differs from the single-device frame", file=sys.stderr)

    # --- kernel-only timing with HIP events on the launch stream ------------
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    n_k = max(1, min(args.steps, 3))
    local = locals_[0]
    ev[0].record(stream)
    for _ in range(n_k):
        tipe_rt.render_async(ds, p, tiling, local[0].data_ptr(), local[1].data_ptr(), local[2].data_ptr(),
                             None, sptr)
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = ev[0].elapsed_time(ev[1]) / n_k

    # --- algorithmic FLOPs from a counting pass (8 spp, same frame) ---------
    p_cnt = tipe_rt.make_params(W, H, 8, BOUNCES, cam, focus=3.0, seed=SEED)
    d_cnt = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device=dev)
    tipe_rt.count_async(ds, p_cnt, tiling, d_cnt.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    cnt = [int(x) for x in d_cnt.cpu()]
    px_local = valid_rows(tiling) * W
    launch_samples = px_local * SPP
    flops = flops_per_launch(cnt, len(spheres), 0) * (launch_samples / max(cnt[0], 1))
    achieved_tflops = flops / (kernel_ms * 1e-3) / 1e12
    # the reference's own work (no zero-throughput exit: every path runs its
    # bounces) at the same rate: what the frame costs main.c's algorithm
    d_ref = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device=dev)
    with tipe_rt.reference_counts():
        tipe_rt.count_async(ds, p_cnt, tiling, d_ref.data_ptr(), sptr)
        torch.cuda.synchronize(dev)
    cnt_ref = [int(x) for x in d_ref.cpu()]
    flops_ref = flops_per_launch(cnt_ref, len(spheres), 0) * (launch_samples / max(cnt_ref[0], 1))
    out_bytes = px_local * 3 * 24
    traffic = load_pmc_traffic()

    total_samples = W * H * SPP * args.steps
    value = total_samples / elapsed / 1e6
    if rank == 0:
        per = {k: cnt[i] / max(cnt[0], 1) for i, k in enumerate(tipe_rt.COUNTER_NAMES)}
        rec = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic scene: README 10-sphere Cornell box (alpha=1, materialIndex=1), Philox seed 1010",
            "config": {"workload": "C2: 10-sphere Cornell box, 1200x900, 1000 spp, 6 bounces",
                       "width": W, "height": H, "spp": SPP, "bounces": BOUNCES,
                       "tile_rows": TILE_ROWS if world > 1 else H, "parallelism": "row-tiles x%d" % world, "frames_in_flight": nbuf,
                       "collective": ("rccl gather" if args.dist_backend == "nccl" else "gloo gather (host)")
                       if world > 1 else None,
                       "rng": "philox4x32-10", "spp_chunks": args.chunks,
                       "arith": "fp64, reference op order (bit-exact vs oracle)"},
            "roofline": {"bound": "valu", "achieved": round(achieved_tflops, 3), "peak": FP64_VECTOR_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tflops / FP64_VECTOR_PEAK_TFLOPS, 4),
                         "traffic": traffic, "kernel": "render_kernel_q<false, false> (persistent task queue) + combine_kernel",
                         "kernel_ms": round(kernel_ms, 3), "flops_per_launch": flops,
                         "flops_per_sample": round(flops / launch_samples, 1),
                         "note": "achieved = algorithmic FLOPs of the work done (SURVEY 8d formula on the "
                                 "kernel's own event counts; paths end at zero throughput) / kernel time",
                         "reference_work": {"flops_per_sample": round(flops_ref / launch_samples, 1),
                                            "tflops_equivalent": round(flops_ref / (kernel_ms * 1e-3) / 1e12, 3),
                                            "frac": round(flops_ref / (kernel_ms * 1e-3) / 1e12
                                                          / FP64_VECTOR_PEAK_TFLOPS, 4)},
                         "hbm": {"achieved_GBps": round(out_bytes / (kernel_ms * 1e-3) / 1e9, 4),
                                 "peak_GBps": HBM_PEAK_GBS,
                                 "frac": out_bytes / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                 "algorithmic_bytes_per_launch": out_bytes}},
            "events_per_sample": {k: round(v, 3) for k, v in per.items()},
            "kernel_msamples_per_s": round(launch_samples / (kernel_ms * 1e-3) / 1e6, 3),
        }
        if verified is not None:
            rec["verified_vs_single_device"] = verified
        if world == 1 and not args.no_cpu_baseline:
            pc = tipe_rt.make_params(W, H, SPP, BOUNCES, cam, focus=3.0, seed=SEED, chunks=args.chunks)
            rec["cpu_baseline"] = cpu_baseline(pc, scene, threads=args.cpu_threads)
            rec["speedup_vs_cpu_baseline"] = round(value / rec["cpu_baseline"]["value"], 1)
        print(json.dumps(rec))
    ds.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
