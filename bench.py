#!/usr/bin/env python3
"""bench.py — Msamples/s of the MI355X render path on BASELINE config C2.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

One step = one full frame of config C2 (README 10-sphere Cornell box,
1200x900, 1000 spp, 6 bounces; Philox stream, seed 1010) rendered into HBM.
With N > 1 the bench runs one rank per GPU: either launched by
torch.distributed.run (RANK/WORLD_SIZE set), or, when `--gpus N` is given
without that environment, this script starts the N rank processes itself
(spawn_ranks: the parent never initialises the GPU, and fails with exit 2
if fewer than N GPUs are visible).  The frame is
split into cyclic 1-row tiles (row t -> rank t mod N), each rank renders its
tiles, the tiles' colour (the canva plane: write_color_canva integers, exact
in float32, so 12 B/px -- SURVEY §8(e)'s float3 colour payload; `--gather
all` sends canva + albedo + normal as doubles, 72 B/px, for a denoiser) is
gathered to rank 0 over RCCL (torch.distributed.gather, backend "nccl") and
rank 0 un-permutes it (rt_assemble_async): total work per step is fixed, so
scaling is "strong".  At N > 1 the line's `configs` then holds BASELINE
configs 3-5 (pyramid; tree + AO; the 4K pyramid frame) at their full spp,
row-tiled over the same N ranks with the same RCCL gather (configs_sharded:
Msamples/s, ms per frame, gather ms, per-rank render spread).  At N > 1 rank
0 also times `single_process`: the
library's own one-process multi-device frame (rt_render_gather_async over
the N devices, its own RCCL ncclGather over xGMI), the path a C caller of
rt.h uses.

Rank 0 prints ONE JSON line.  Besides the C2 headline it carries (N = 1,
rank 0): `configs` (C3, C4, C5 and the 10-sphere/100-triangle sweep scene at
reduced spp, kernel rates and roofline fractions), `end_to_end` (host-buffer
rates of the drop-ins rt_render_rows and rt_fill_canva x 12 pthreads, i.e.
upload -> render -> assembled host framebuffer) and `cpu_baseline` with six
legs (1, 12 and the box's CPU share of threads x faithful / fair RNG).
`roofline` prices the render kernel against
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
TILE_ROWS = 1        # cyclic 1-row tiles: the busiest of 8 ranks renders 113 of 900 rows (99.6 % balance;
                     # 2-row tiles: 114, 98.7 %; 8-row tiles: 120, 94 %)
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
    """HBM bytes per render launch from the committed rocprofv3 --pmc pass
    (profiles/pmc_traffic.json: value, profile directory, commit), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("render_kernel_hbm_bytes_per_launch"), {k: v for k, v in d.items()
                                                             if k != "render_kernel_hbm_bytes_per_launch"}
    except Exception:
        return None, None


def cpu_share():
    """CPUs this process may use: the cgroup quota (cpu.max) if any, else the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except Exception:
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_smt():
    try:
        return int(open("/sys/devices/system/cpu/smt/active").read().strip()) == 1
    except Exception:
        return None


def cpu_baseline(scene, cam, threads=12):
    """The CPU restatement (oracle/rt_oracle.c) on the full C2 frame at
    reduced spp, main.c's partition (NUM_THREADS contiguous row bands,
    main.c:407-449), in six legs: NUM_THREADS in {1, `threads`, the box's
    CPU share} x RNG mode
      faithful: one global glibc rand() stream shared by every thread, as
                main.c's threads share it (lock-serialised; libm math);
      fair:     a lock-free stream per pixel (Philox; portable math).
    Msamples/s does not depend on spp (pixels are independent), so each leg
    renders the 1200x900 frame at 1-32 spp (about 1-14 s each on the GPU
    box's 16-CPU share).  The headline is fair x 12 at 32 spp."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi
    o = oracle_ffi.oracle()
    canva = np.zeros((H, W, 3))
    share = cpu_share()
    legs = {}
    for mode, rng in (("fair", tipe_rt.RT_RNG_PHILOX), ("faithful", tipe_rt.RT_RNG_GLIBC)):
        for nt in sorted({1, threads, share}):
            # the headline leg (fair, `threads`) renders 32 spp (~5 s on 12 threads); the
            # others 1-8 spp, so the six legs take about 45 s together
            spp = (32 if nt == threads else 8 if nt > 1 else 2) if mode == "fair" else (2 if nt == 1 else 1)
            p = tipe_rt.make_params(W, H, spp, BOUNCES, cam, focus=3.0, seed=SEED, rng=rng, chunks=1)
            t0 = time.perf_counter()
            rc = o.oracle_render_rows(C.byref(scene), C.byref(p), H - 1, 0, nt, 1, canva.ctypes.data,
                                      None, None, None, None)
            dt = time.perf_counter() - t0
            assert rc == 0
            legs["%s_%dt" % (mode, nt)] = {"value": round(W * H * spp / dt / 1e6, 4), "threads": nt,
                                            "spp": spp, "seconds": round(dt, 2)}
    head = legs["fair_%dt" % threads]
    return {"value": head["value"], "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "full 1200x900 C2 frame at %d spp (other legs: see legs), oracle/rt_oracle.c (CPU restatement of main.c), "
                      "%d pthreads over main.c's contiguous row bands (main.c:407-449), Philox per-pixel "
                      "stream (the 'fair' leg; see legs)" % (head["spp"], threads),
            "legs": legs, "cpu_model": cpu_model(), "smt": cpu_smt(), "host_logical_cpus": os.cpu_count(),
            "cpu_share": share,
            "note": "faithful = one lock-serialised glibc rand() stream shared by all threads (main.c's "
                    "behaviour, rtutility.h:229-231); fair = lock-free per-pixel stream"}


# ---- other BASELINE configs (kernel rates in their own task regime, N = 1) ----
CONFIGS = {
    # name: (scene builder, spp measured, bounces, useAO, W, H, full spp, GPUs of the config)
    # C3/C4/C5 are timed at their FULL spp on the full frame with spp_chunks AUTO
    # (tapered slices: rt.h rt_chunk_bound), i.e. exactly the tasks the
    # config's own frame hands out (C4: ~67 samples per slice, C5: ~167); the
    # sweep scene is defined at 64 spp.
    "C3": ("pyramid", 1000, 6, False, 1200, 900, 1000, 1),
    "C4": ("tree", 2000, 8, True, 1200, 900, 2000, 4),
    "C5": ("pyramid", 5000, 6, False, 3840, 2880, 5000, 8),
    "sweep_10s_100t": ("sweep", 64, 6, False, 1200, 900, 64, 1),
    # the reference's own production scene (RTX_MAP/nature, 5812 textured triangles with
    # alpha holes, lit by main.c:345-346's sun and radius-1e5 sky) at its own render
    # settings: 1000 rays, nbRebondMax 10 (RTX_nature_1000RAYS_9RB, .MISSING_LARGE_BLOBS:8,
    # name rule main.c:328); 1200x900 as the other configs; camera scenes.NATURE_CAMERA
    "nature": ("nature", 1000, 10, False, 1200, 900, 1000, 1),
}
CONFIG_CAMERA = {"nature": scenes.NATURE_CAMERA}


def config_scene(kind):
    if kind == "nature":
        sph = scenes.main_spheres()
        tris, qm, mats, tw, th, nm = scenes.nature_mesh()
        return tipe_rt.make_scene(sph, tris, qm, mats, tw, th, nm), len(sph), len(tris)
    sph = scenes.cornell_spheres()
    if kind == "pyramid":
        return tipe_rt.make_scene(sph, *scenes.pyramid_mesh()), len(sph), 5
    if kind == "tree":
        tris, qm, mats, tw, th, nm = scenes.tree_mesh()
        return tipe_rt.make_scene(sph, tris, qm, mats, tw, th, nm), len(sph), len(tris)
    sph, (tris, qm, mats, tw, th, nm) = scenes.synthetic_cornell(10, 100)
    return tipe_rt.make_scene(sph, tris, qm, mats, tw, th, nm), len(sph), len(tris)


def work_flops(c, ns):
    """FLOPs of the work done per launch (roofline sweep convention):
    SURVEY 8(d)'s terms with 40 per triangle test made and 48 per BVH node."""
    T = tipe_rt.types
    bvh = c[T.RT_CNT_BVH_NODES] > 0
    tri_done = c[T.RT_CNT_BVH_TRI_TESTS] if bvh else c[T.RT_CNT_TRI_TESTS]
    return (40 * c[0] + c[T.RT_CNT_CASTS] * (25 * ns + 18) + 40 * tri_done + 48 * c[T.RT_CNT_BVH_NODES]
            + 5 * c[T.RT_CNT_SPHERE_DISC] + 100 * c[T.RT_CNT_SHADE] + 80 * c[T.RT_CNT_TEX_HITS]
            + 40 * c[T.RT_CNT_REFRACT])


def task_regime(spp, w, h):
    """The (chunk, pixel) tasks one launch hands out: rt_chunk_bound's slices."""
    P = tipe_rt.types.rt_resolve_spp_chunks(tipe_rt.RT_SPP_CHUNKS_AUTO, spp)
    L = tipe_rt.types.rt_chunk_taper_levels(spp, P)
    den = (P - L) * (1 << L) + (1 << L) - 1 if L else P
    main = spp * (1 << L) / den if L else spp / P
    return {"spp_chunks": P, "tapered": bool(L), "taper_levels": L, "samples_per_main_slice": round(main, 1),
            "tasks": w * h * P}


def config_camera(name, cam):
    spec = CONFIG_CAMERA.get(name)
    return cam if spec is None else tipe_rt.init_camera(**{k: spec[k] for k in ("origin", "target", "up", "vfov",
                                                                                 "ratio")})


def configs_extra(dev, stream, cam0):
    out = {}
    sptr = stream.cuda_stream
    for name, (kind, spp, bounces, ao, w, h, full_spp, gpus) in CONFIGS.items():
        sc, ns, nt = config_scene(kind)
        cam = config_camera(name, cam0)
        p = tipe_rt.make_params(w, h, spp, bounces, cam, focus=3.0, use_ao=ao, ao=2.5, seed=SEED,
                                chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
        ds = tipe_rt.DeviceScene(sc, dev.index)
        tiling = tipe_rt.band_tiling(0, h - 1)
        buf = torch.empty((3, h, w, 3), dtype=torch.float64, device=dev)

        def launch():
            tipe_rt.render_async(ds, p, tiling, buf[0].data_ptr(), buf[1].data_ptr(), buf[2].data_ptr(), None, sptr)
        # long full-spp frames (>= 1 s) are timed once after a short warm-up frame
        # of the same scene; short ones twice after a full warm-up frame
        long_frame = w * h * spp >= 2e9
        if long_frame:
            pw = tipe_rt.make_params(w, h, 8, bounces, cam, focus=3.0, use_ao=ao, ao=2.5, seed=SEED,
                                     chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
            tipe_rt.render_async(ds, pw, tiling, buf[0].data_ptr(), buf[1].data_ptr(), buf[2].data_ptr(), None, sptr)
        else:
            launch()
        torch.cuda.synchronize(dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 1 if long_frame else 2
        ev[0].record(stream)
        for _ in range(reps):
            launch()
        ev[1].record(stream)
        torch.cuda.synchronize(dev)
        ms = ev[0].elapsed_time(ev[1]) / reps
        kname = tipe_rt.last_render_kernel()
        pc = tipe_rt.make_params(w, h, 2, bounces, cam, focus=3.0, use_ao=ao, ao=2.5, seed=SEED)
        d = torch.zeros(tipe_rt.RT_NCOUNTERS, dtype=torch.int64, device=dev)
        tipe_rt.count_async(ds, pc, tiling, d.data_ptr(), sptr)
        torch.cuda.synchronize(dev)
        c = [int(x) for x in d.cpu()]
        ds.close()
        rate = w * h * spp / (ms * 1e-3) / 1e6
        fps = work_flops(c, ns) / max(c[0], 1)
        tf = rate * 1e6 * fps / 1e12
        T = tipe_rt.types
        rec = {"kernel_msamples_per_s": round(rate, 1), "spp_measured": spp, "kernel_ms": round(ms, 3),
               "launches_timed": reps, "task_regime": task_regime(spp, w, h),
               "width": w, "height": h, "bounces": bounces, "ao": ao, "spheres": ns, "triangles": nt,
               "flops_per_sample_work_done": round(fps, 1), "achieved_tflops": round(tf, 3),
               "frac": round(tf / FP64_VECTOR_PEAK_TFLOPS, 4),
               "casts_per_sample": round(c[T.RT_CNT_CASTS] / max(c[0], 1), 3)}
        if ao:
            # make_params' default compat_int_truncation = 1: ThreadData's int AO_intensity
            # (main.c:43) turns the requested 2.5 into 2, as the reference's fill_canva does
            rec["ao_intensity"] = 2.5
            rec["ao_intensity_effective"] = float(int(2.5)) if p.compat_int_truncation else 2.5
        rec["kernel"] = kname
        if c[T.RT_CNT_BVH_NODES]:
            rec["bvh_nodes_per_sample"] = round(c[T.RT_CNT_BVH_NODES] / c[0], 3)
            rec["bvh_tri_tests_per_sample"] = round(c[T.RT_CNT_BVH_TRI_TESTS] / c[0], 3)
            rec["bvh_simd_efficiency"] = round(c[T.RT_CNT_BVH_NODES] / max(c[T.RT_CNT_BVH_LANE_SLOTS], 1), 4)
            # with a BVH the brute-force F (every cast tests all N_t triangles,
            # main.c:81-90) is reported beside the work-done figure; its "frac" exceeds 1 by
            # what the tree saves
            fref = flops_per_launch(c, ns, nt) / max(c[0], 1)
            rec["flops_per_sample_reference"] = round(fref, 1)
            rec["frac_reference_bruteforce"] = round(rate * 1e6 * fref / 1e12 / FP64_VECTOR_PEAK_TFLOPS, 4)
        if kind != "sweep":
            rec["full_frame_s_1gpu"] = round(ms * 1e-3 * full_spp / spp, 3)
            rec["config_gpus"] = gpus
        out[name] = rec
    return out


# ---- C3 / C4 / C5 row-tiled over the N ranks (N > 1) -------------------------
def _max_over_ranks(x, dev, backend):
    t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def configs_sharded(args, rank, world, dev, cam, names):
    """BASELINE configs 3-5 at N > 1 (config 4 is quoted on 4 GPUs, config 5
    on 8 with an RCCL gather; BASELINE.md §4 asks for every config at every
    N): each rank renders its cyclic 1-row tiles of the config's full frame
    (rt_render_async with rt.h's cyclic rt_tiling; the reference's row bands,
    main.c:404-453, and main_cuda.cu:280-339's single-GPU staging are what
    this replaces), the canva plane travels to rank 0 as float32 over RCCL
    (torch.distributed.gather) and rank 0 un-permutes it (rt_assemble_async).
    One frame is timed per config after a short warm-up frame, bracketed by
    barrier + synchronize, max over ranks; `gather_ms` times the gather +
    assembly alone in a second bracket.  `--config-spp` reduces the spp (for
    tests); `--verify` re-renders the frame on rank 0 alone and compares."""
    out = {}
    gpu = dev.index
    st = torch.cuda.current_stream(dev)
    cam0 = cam
    for name in names:
        kind, _, bounces, ao, w, h, full_spp, gpus = CONFIGS[name]
        spp = args.config_spp or full_spp
        sc, ns, nt = config_scene(kind)
        cam = config_camera(name, cam0)
        ds = tipe_rt.DeviceScene(sc, gpu)
        tiling = tipe_rt.cyclic_tiling(h, TILE_ROWS, rank, world)
        rows = tiling.n_tiles * TILE_ROWS
        p = tipe_rt.make_params(w, h, spp, bounces, cam, focus=3.0, use_ao=ao, ao=2.5, seed=SEED,
                                chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
        local = torch.empty((rows, w, 3), dtype=torch.float64, device=dev)
        send = torch.empty((1, rows, w, 3), dtype=torch.float32, device=dev)
        gathered = g64 = full = gather_list = None
        if rank == 0:
            gathered = torch.empty((world, 1, rows, w, 3), dtype=torch.float32, device=dev)
            gather_list = [gathered[r] for r in range(world)]
            g64 = torch.empty_like(gathered, dtype=torch.float64)
            full = torch.empty((h, w, 3), dtype=torch.float64, device=dev)

        def gather():
            if args.dist_backend == "nccl":
                dist.gather(send, gather_list, dst=0)
            else:
                host = [torch.empty_like(send, device="cpu") for _ in range(world)] if rank == 0 else None
                dist.gather(send.cpu(), host, dst=0)
                if rank == 0:
                    for r in range(world):
                        gathered[r].copy_(host[r])
            if rank == 0:
                g64.copy_(gathered)
                tipe_rt.assemble_async(g64[0, 0].data_ptr(), world, TILE_ROWS, rows, w, h, full.data_ptr(),
                                       st.cuda_stream, rank_stride=rows * w)

        def frame(pp):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(st)
            tipe_rt.render_async(ds, pp, tiling, local.data_ptr(), stream=st.cuda_stream)
            ev1.record(st)
            send[0].copy_(local)                      # canva integers, exact in float32
            gather()
            return ev0, ev1

        long_frame = w * h * spp >= 2e9
        warm = p if not long_frame else tipe_rt.make_params(w, h, 8, bounces, cam, focus=3.0, use_ao=ao, ao=2.5,
                                                             seed=SEED, chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
        frame(warm)
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0, ev1 = frame(p)
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = _max_over_ranks(time.perf_counter() - t0, dev, args.dist_backend)
        render_ms = ev0.elapsed_time(ev1)
        render_ms_max = _max_over_ranks(render_ms, dev, args.dist_backend)
        render_ms_min = -_max_over_ranks(-render_ms, dev, args.dist_backend)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        gather()
        torch.cuda.synchronize(dev)
        dist.barrier()
        gather_s = _max_over_ranks(time.perf_counter() - t1, dev, args.dist_backend)
        rec = {"n_gpus": world, "msamples_per_s": round(w * h * spp / elapsed / 1e6, 1),
               "ms_per_frame": round(elapsed * 1e3, 3), "gather_ms": round(gather_s * 1e3, 3),
               "rank_render_ms_max": round(render_ms_max, 3), "rank_render_ms_min": round(render_ms_min, 3),
               "spp": spp, "full_spp": full_spp, "width": w, "height": h, "bounces": bounces, "ao": ao,
               "spheres": ns, "triangles": nt, "config_gpus": gpus, "tile_rows": TILE_ROWS,
               "rows_per_rank": rows, "frames_timed": 1, "warmup_spp": warm.nbRayonParPixel,
               "collective": "rccl gather" if args.dist_backend == "nccl" else "gloo gather (host)",
               "gather_payload": "canva as float32, 12 B/px", "scaling": "strong"}
        if ao:
            rec["ao_intensity_effective"] = float(int(2.5)) if p.compat_int_truncation else 2.5
        if args.verify and rank == 0:
            ref = torch.empty((h, w, 3), dtype=torch.float64, device=dev)
            tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, h - 1), ref.data_ptr(), stream=st.cuda_stream)
            torch.cuda.synchronize(dev)
            rec["verified_vs_single_device"] = bool(torch.equal(ref, full))
            if not rec["verified_vs_single_device"]:
                print("verify: %s assembled frame differs from the single-device frame" % name, file=sys.stderr)
            del ref
        dist.barrier()
        ds.close()
        del local, send, gathered, g64, full
        torch.cuda.empty_cache()
        out[name] = rec
    return out


# ---- end-to-end host-buffer rates of the drop-ins (N = 1) --------------------
def end_to_end(scene, spheres, cam, reps=2):
    """Upload -> render -> assembled host framebuffer through the C-ABI:
    rt_render_rows (one call, whole frame, canva + albedo + normal) and
    rt_fill_canva on 12 threads over main.c's row bands (main.c:404-453).
    Both use RT_SPP_CHUNKS_AUTO; the scene cache holds the upload after the
    first (untimed) call, as it does for every frame after a program's first."""
    import threading
    from tipe_rt.types import ThreadData, Sphere
    L = tipe_rt.lib()
    p = tipe_rt.make_params(W, H, SPP, BOUNCES, cam, focus=3.0, seed=SEED, chunks=tipe_rt.RT_SPP_CHUNKS_AUTO)
    canva, alb, nrm = (np.zeros((H, W, 3)) for _ in range(3))

    def rows_call():
        tipe_rt.check(L.rt_render_rows(C.byref(scene), C.byref(p), H - 1, 0, canva.ctypes.data, alb.ctypes.data,
                                       nrm.ctypes.data))
    NT = 12
    rows = H // NT
    tds = []
    for t in range(NT):
        hi = H - 1 - t * rows
        td = ThreadData()
        td.start_row, td.end_row = hi, (hi - rows + 1 if t < NT - 1 else 0)
        td.canva = C.cast(canva.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.albedo_tab = C.cast(alb.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.normal_tab = C.cast(nrm.ctypes.data, C.POINTER(tipe_rt.Vec3))
        td.cam = cam
        td.largeur_image, td.hauteur_image = W, H
        td.nbRayonParPixel, td.nbRebondMax = SPP, BOUNCES
        td.total_pixels = W * H
        td.sphere_list = C.cast(spheres, C.POINTER(Sphere))
        td.nbSpheres = len(spheres)
        td.focus_distance = 3
        tds.append(td)

    def fill_call():
        res = []
        ths = [threading.Thread(target=lambda t=t: res.append(L.rt_fill_canva(C.byref(t)))) for t in tds]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert all(r is None for r in res), L.rt_last_error()
    out = {}
    for name, fn in (("rt_render_rows", rows_call), ("rt_fill_canva_x12_pthreads", fill_call)):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) / reps
        out[name] = {"msamples_per_s": round(W * H * SPP / dt / 1e6, 1), "ms_per_frame": round(dt * 1e3, 2)}
    out["note"] = ("C2 frame, host buffers (canva, albedo, normal: 78 MB over PCIe), spp_chunks AUTO; "
                   "the scene upload is cached after the first call; %d timed frames each" % reps)
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv):
    """`python bench.py --gpus N` with no torch.distributed environment: start
    N rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as
    torch.distributed.run sets them, rendezvous on 127.0.0.1) and return the
    exit code.  This parent never touches the GPU (torch.cuda.device_count()
    does not initialise it on ROCm), so no GPU process is ever replaced by
    exec; the ranks are children.  With the nccl (RCCL) backend every rank
    needs its own device: fewer than N visible devices is an error (exit 2),
    never a silent N = 1 run.  Rank 0 prints the JSON line."""
    import signal
    import subprocess
    n = args.gpus
    visible = torch.cuda.device_count()
    if args.dist_backend == "nccl" and visible < n:
        print("bench.py: --gpus %d needs %d visible GPUs, found %d" % (n, n, visible), file=sys.stderr)
        return 2
    if visible < 1:
        print("bench.py: no GPU visible", file=sys.stderr)
        return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print("bench.py: rank %d exited with %d; stopping the others" % (procs.index(p), c),
                          file=sys.stderr)
                    stop()
            time.sleep(0.2)
    finally:
        stop()
        for p in procs:
            try:
                p.wait(timeout=30)
            except Exception:
                p.kill()
        signal.signal(signal.SIGTERM, old)
    return rc


def single_process_leg(scene, p, world, devs, steps, verify_ref=None):
    """§8(e)'s in-library path for a C caller: one process, rt_init over the N
    devices, rt_render_gather_async per frame (every device renders its cyclic
    1-row tiles on a pooled stream, the canva planes travel to the first
    device by the library's RCCL ncclGather over xGMI -- peer copies when a
    rehearsal repeats a device -- and are assembled there; `transport` names
    the one used).  Timed over `steps` frames after one warm-up frame; canva
    only, as the bench's gather."""
    L = tipe_rt.lib()
    tipe_rt.check(L.rt_init(len(devs), (C.c_int * len(devs))(*devs)))
    # the library's RCCL gather (ncclGather over one communicator per device) on
    # distinct devices; peer copies, explicitly, when a rehearsal repeats a device
    import copy
    p = copy.copy(p)
    p.gather = tipe_rt.types.RT_GATHER_RCCL if len(set(devs)) == len(devs) else tipe_rt.types.RT_GATHER_PEER
    dev = torch.device("cuda", devs[0])
    st = torch.cuda.current_stream(dev)
    try:
        full = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        tipe_rt.render_gather_async(scene, p, TILE_ROWS, full.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize(dev)
        ok = None if verify_ref is None else bool(torch.equal(full, verify_ref))
        t0 = time.perf_counter()
        for _ in range(steps):
            tipe_rt.render_gather_async(scene, p, TILE_ROWS, full.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        transport = tipe_rt.last_gather_transport()
    finally:
        L.rt_shutdown()
        tipe_rt.check(L.rt_init(0, None))
    rec = {"value": round(W * H * SPP * steps / dt / 1e6, 3), "unit": "Msamples/s", "devices": list(devs),
           "distinct_devices": len(set(devs)), "steps": steps, "ms_per_step": round(dt / steps * 1e3, 3),
           "entry_point": "rt_render_gather_async (include/rt/rt.h)", "payload": "canva plane, float64",
           "transport": transport}
    if ok is not None:
        rec["verified_vs_single_device"] = ok
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the configs / end_to_end keys")
    ap.add_argument("--cpu-threads", type=int, default=12)
    ap.add_argument("--chunks", type=int, default=int(os.environ.get("RT_BENCH_CHUNKS", "32")),
                    help="rt_params.spp_chunks (fixed slice grouping of each pixel's samples; the same "
                         "for every N, so the image does not depend on the GPU count)")
    ap.add_argument("--verify", action="store_true",
                    help="N>1: rank 0 re-renders the frame alone and checks the assembled planes bit for bit")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one stream: frame k+1 starts after frame k (default: two streams, see step())")
    ap.add_argument("--gather", default="colour", choices=["colour", "all"],
                    help="N>1 payload: colour = the canva plane as float32 (12 B/px); all = canva, albedo and "
                         "normal as float64 (72 B/px, what a denoiser needs)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: gather through host copies (rehearsing N>1 with all ranks on one GPU); "
                         "nccl (= RCCL) is the measured configuration")
    ap.add_argument("--no-single-process", action="store_true",
                    help="N>1: skip the single_process leg (rt_render_gather_async over the N devices)")
    ap.add_argument("--configs", default="C3,C4,C5",
                    help="N>1: BASELINE configs rendered row-tiled over the N ranks after the C2 headline "
                         "(comma list of C3, C4, C5, nature; empty: none)")
    ap.add_argument("--config-spp", type=int, default=0,
                    help="N>1 config legs: render at this spp instead of each config's full spp (tests)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args, sys.argv[1:]))
    if torch.cuda.device_count() < 1:
        print("bench.py: no GPU visible", file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE %d; rendering on the %d ranks launched" % (args.gpus, world, world),
              file=sys.stderr)
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
    colour = args.gather == "colour"
    npl = 1 if colour else 3                  # planes gathered and assembled
    gdt = torch.float32 if colour else torch.float64
    sends = [torch.empty((npl, rows, W, 3), dtype=gdt, device=dev) for _ in range(nbuf)] if colour else locals_
    gathered_ = gather_lists = fulls = gathered64_ = [None] * nbuf
    if world > 1 and rank == 0:
        gathered_ = [torch.empty((world, npl, rows, W, 3), dtype=gdt, device=dev) for _ in range(nbuf)]
        gather_lists = [[g[r] for r in range(world)] for g in gathered_]
        gathered64_ = ([torch.empty((world, npl, rows, W, 3), dtype=torch.float64, device=dev) for _ in range(nbuf)]
                       if colour else gathered_)
        fulls = [torch.empty((npl, H, W, 3), dtype=torch.float64, device=dev) for _ in range(nbuf)]
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
                send = sends[b]
                if colour:
                    send[0].copy_(local[0])                  # canva integers, exact in float32
                if args.dist_backend == "nccl":
                    dist.gather(send, gather_list, dst=0)      # RCCL over xGMI
                else:
                    host = [torch.empty_like(send, device="cpu") for _ in range(world)] if rank == 0 else None
                    dist.gather(send.cpu(), host, dst=0)
                    if rank == 0:
                        for r in range(world):
                            gathered[r].copy_(host[r])
                if rank == 0:
                    g64 = gathered64_[b]
                    if colour:
                        g64.copy_(gathered)
                    for pl in range(npl):                   # (world, plane, rows, W, 3) -> (plane, H, W, 3)
                        tipe_rt.assemble_async(g64[0, pl].data_ptr(), world, TILE_ROWS, rows, W, H,
                                               full[pl].data_ptr(), st.cuda_stream, rank_stride=npl * rows * W)

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
    ref = None
    if args.verify and world > 1 and rank == 0:
        ref = torch.empty((3, H, W, 3), dtype=torch.float64, device=dev)
        tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, H - 1), ref[0].data_ptr(), ref[1].data_ptr(),
                             ref[2].data_ptr(), None, sptr)
        torch.cuda.synchronize(dev)
        used = fulls[:min(nbuf, args.warmup + args.steps)]            # every buffer that held a frame
        verified = all(bool(torch.equal(ref[:npl], f)) for f in used)
        if not verified:
            print("verify: assembled frame differs from the single-device frame", file=sys.stderr)

    # --- the library's own single-process multi-device frame (N > 1) --------
    single = None
    if world > 1 and not args.no_single_process:
        # host-side barriers (gloo), so the other ranks wait without a
        # collective kernel spinning on the devices rank 0 now renders on
        cpu_group = dist.new_group(backend="gloo")
        dist.barrier(group=cpu_group)
        if rank == 0:
            ndev = torch.cuda.device_count()
            devs = [r if args.dist_backend == "nccl" else r % max(1, ndev) for r in range(world)]
            try:
                single = single_process_leg(scene, p, world, devs, max(1, min(args.steps, 5)),
                                            None if ref is None else ref[0])
            except Exception as e:       # reported, never fatal to the RCCL measurement above
                single = {"error": repr(e), "devices": devs}
                print("single_process leg failed: %r" % e, file=sys.stderr)
            if single.get("verified_vs_single_device") is False:
                print("verify: rt_render_gather_async frame differs from the single-device frame", file=sys.stderr)
        dist.barrier(group=cpu_group)
        torch.cuda.set_device(dev)

    # --- C3 / C4 / C5 row-tiled over the N ranks ------------------------------
    sharded = None
    if world > 1 and args.configs:
        names = [n.strip() for n in args.configs.split(",") if n.strip()]
        bad = [n for n in names if n not in ("C3", "C4", "C5", "nature")]
        if bad:
            raise SystemExit("bench.py: unknown --configs %s" % bad)
        sharded = configs_sharded(args, rank, world, dev, cam, names)
        torch.cuda.set_device(dev)

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
    traffic, traffic_src = load_pmc_traffic()
    # HBM bytes by construction (in-run model, beside the committed PMC value):
    # the render kernel writes one 72-B partial per (chunk, pixel) task,
    # combine_kernel reads them back once and writes the three output planes
    # (72 B/px); with one chunk the render kernel writes the frame itself
    chunks = tipe_rt.types.rt_resolve_spp_chunks(args.chunks, SPP)
    traffic_model = px_local * 72 * chunks if chunks > 1 else out_bytes
    traffic_model_frame = 2 * px_local * 72 * chunks + out_bytes if chunks > 1 else out_bytes

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
                       "gather_payload": ("canva as float32, 12 B/px" if colour else "canva+albedo+normal as float64, 72 B/px")
                       if world > 1 else None,
                       "rng": "philox4x32-10", "spp_chunks": args.chunks,
                       "arith": "fp64, reference op order (bit-exact vs oracle)"},
            "roofline": {"bound": "valu", "achieved": round(achieved_tflops, 3), "peak": FP64_VECTOR_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tflops / FP64_VECTOR_PEAK_TFLOPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_model_bytes_per_launch": traffic_model,
                         "traffic_model_frame_bytes": traffic_model_frame,
                         "traffic_model_note": "model: render kernel = chunks x px x 72 B partial writes; frame = "
                                               "that x 2 (combine_kernel reads them) + 72 B/px output; `traffic` "
                                               "is the last committed rocprofv3 PMC value (traffic_source)",
                         "kernel": "render_kernel_q<false, 0, -2, false> (persistent task queue, sphere-only opaque-material instantiation; no sky, no AO, no BVH) + combine_kernel",
                         "kernel_ms": round(kernel_ms, 3), "flops_per_launch": flops,
                         "scope": "whole frame (1 GPU)" if world == 1 else
                                  "per rank: rank 0's cyclic row tiles (%d of %d rows), its own kernel time"
                                  % (valid_rows(tiling), H),
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
        if world > 1:
            rec["config"]["devices"] = len({r if args.dist_backend == "nccl" else r % max(1, torch.cuda.device_count())
                                            for r in range(world)})
        if single is not None:
            rec["single_process"] = single
        if sharded is not None:
            rec["configs"] = sharded
        if world == 1 and not args.no_extras:
            rec["configs"] = configs_extra(dev, stream, cam)
            rec["end_to_end"] = end_to_end(scene, spheres, cam)
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(scene, cam, threads=args.cpu_threads)
            rec["speedup_vs_cpu_baseline"] = round(value / rec["cpu_baseline"]["value"], 1)
        print(json.dumps(rec), flush=True)
    ds.close()
    torch.cuda.synchronize(dev)
    tipe_rt.lib().rt_shutdown()      # cached scenes, pooled streams and pinned buffers of the drop-in legs
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
