"""Multi-rank row-tile sharding on CPU (gloo, world_size 2; virtual ranks
1..8).  Each rank renders the cyclic k-row tiles rt_tiling assigns it
(tile t -> rank t mod G, tipe_rt.cyclic_tiling) into a rank-local frame laid
out as rt_render_async writes it, the frames are gathered to rank 0
(dist.gather, the same call bench.py makes over RCCL), and rank 0
un-permutes them with rt_assemble_async's index map.  The image must be
bit-identical to a single-rank render for every rank count: pixels are
independent and the Philox stream is keyed by the global pixel index.

Rendering uses the CPU oracle (test infrastructure); on the GPU box the same
flow runs through librt_hip.so (test_gpu_parity / bench.py)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import helpers
import tipe_rt

W, H, SPP, B, K = 24, 19, 3, 5, 4


def render_local_frame(rank, world):
    """What rank `rank` holds after rt_render_async with cyclic_tiling."""
    bundle = helpers.cornell()
    p = helpers.params(W, H, SPP, B)
    t = tipe_rt.cyclic_tiling(H, K, rank, world)
    local = np.zeros((t.n_tiles * t.tile_rows, W, 3))
    for lt in range(t.n_tiles):
        g0 = t.row_base + (t.tile_first + lt * t.tile_step) * t.tile_rows
        if g0 >= H:
            continue
        g1 = min(g0 + t.tile_rows, H) - 1
        out = helpers.oracle_render(bundle, p, row_hi=g1, row_lo=g0)
        local[lt * K: lt * K + (g1 - g0 + 1)] = out["canva"][g0:g1 + 1]
    return local


def assemble(gathered, world, rows_per_rank):
    """rt_assemble_async's map (rt_kernels.hip assemble_kernel)."""
    full = np.zeros((H, W, 3))
    for g in range(H):
        t, y = divmod(g, K)
        r, lt = t % world, t // world
        full[g] = gathered[r][lt * K + y]
    return full


def reference_frame():
    return helpers.oracle_render(helpers.cornell(), helpers.params(W, H, SPP, B))["canva"]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_virtual_ranks_assemble_bit_identical(world):
    frames = [render_local_frame(r, world) for r in range(world)]
    rows = frames[0].shape[0]
    assert all(f.shape[0] == rows for f in frames)
    assert (assemble(frames, world, rows) == reference_frame()).all()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        local = torch.from_numpy(render_local_frame(rank, world))
        # bench.py's payload: the canva plane as float32 (write_color_canva
        # integers 0..255, exact), 12 B/px instead of 72
        send = local.float()
        exact = bool((send.double() == local).all())
        gl = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
        dist.gather(send, gl, dst=0)
        if rank == 0:
            full = assemble([g.double().numpy() for g in gl], world, local.shape[0])
            q.put(exact and bool((full == reference_frame()).all()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_gather_assemble():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 2000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_bench_accounting_helpers():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(helpers.oracle_ffi.ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    # every row of the C2 frame is rendered exactly once across ranks
    for world in (1, 2, 4, 8):
        rows = sum(bench.valid_rows(tipe_rt.cyclic_tiling(bench.H, bench.TILE_ROWS, r, world))
                   for r in range(world))
        assert rows == bench.H
    cnt = [100, 574, 5740, 2865, 0, 568, 0, 0, 1537]
    f = bench.flops_per_launch(cnt, 10, 0)
    assert f == 40 * 100 + 574 * (250 + 18) + 5 * 2865 + 100 * 568
