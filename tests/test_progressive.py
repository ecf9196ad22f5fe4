"""Progressive rendering / checkpoint-resume (rt_accumulate_async +
rt_resolve_async).  With spp_chunks = 1 any split of the
samples into ordered batches reproduces the one-shot frame bit for bit,
including a checkpoint (sums copied to the host and back) between batches;
the oracle confirms the one-shot frame."""
import ctypes as C

import numpy as np
import pytest

import helpers
import tipe_rt
from test_gpu_parity import gpu_render, assert_same

pytestmark = pytest.mark.gpu


def progressive(bundle, p_full, batches, chunks=1, checkpoint_after=None):
    import torch
    W, H, S = p_full.largeur_image, p_full.hauteur_image, p_full.nbRayonParPixel
    dev = torch.device("cuda:0")
    tiling = tipe_rt.band_tiling(0, H - 1)
    sums = torch.zeros((H, W, 9), dtype=torch.float64, device=dev)
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    stream = torch.cuda.current_stream().cuda_stream
    off = 0
    for k, n in enumerate(batches):
        p = helpers.params(W, H, n, p_full.nbRebondMax, use_ao=bool(p_full.useAO), ao=p_full.AO_intensity,
                           seed=p_full.seed, chunks=chunks)
        tipe_rt.accumulate_async(ds, p, off, tiling, sums.data_ptr(), stream)
        off += n
        if checkpoint_after == k:                 # save, wipe, restore
            torch.cuda.synchronize()
            saved = sums.cpu().numpy().copy()
            sums.fill_(float("nan"))
            sums.copy_(torch.from_numpy(saved))
    assert off == S
    planes = [torch.full((H, W, 3), -1.0, dtype=torch.float64, device=dev) for _ in range(4)]
    tipe_rt.resolve_async(sums.data_ptr(), p_full, S, tiling, *(t.data_ptr() for t in planes), stream=stream)
    torch.cuda.synchronize()
    ds.close()
    return [t.cpu().numpy() for t in planes]


@pytest.mark.parametrize("batches", [[12], [5, 7], [1, 1, 10], [3, 3, 3, 3]])
def test_batches_equal_one_shot(batches):
    bundle = helpers.pyramid_scene()
    p = helpers.params(40, 30, 12, 6)
    one = gpu_render(bundle, p)
    got = progressive(bundle, p, batches, checkpoint_after=0)
    for g, o, name in zip(got, one, ["canva", "albedo", "normal", "radiance"]):
        assert_same(g, o, name)
    ref = helpers.oracle_render(bundle, p)
    assert_same(got[0], ref["canva"], "canva vs oracle")


def test_chunked_batches_are_deterministic():
    bundle = helpers.cornell()
    p = helpers.params(33, 21, 10, 5)
    a = progressive(bundle, p, [4, 6], chunks=3)
    b = progressive(bundle, p, [4, 6], chunks=3)
    for x, y in zip(a, b):
        assert (x.view(np.uint64) == y.view(np.uint64)).all()
    one = gpu_render(bundle, p)
    assert (helpers.rmse_per_channel(a[3], one[3]) <= 1e-12).all()


def test_offset_beyond_32_bits_rejected():
    import torch
    bundle = helpers.cornell()
    ds = tipe_rt.DeviceScene(bundle.scene, 0)
    sums = torch.zeros((6, 8, 9), dtype=torch.float64, device="cuda:0")
    p = helpers.params(8, 6, 4, 3)
    rc = tipe_rt.lib().rt_accumulate_async(ds.handle, C.byref(p), (1 << 32) - 2, C.byref(tipe_rt.band_tiling(0, 5)),
                                           sums.data_ptr(), None)
    ds.close()
    assert rc == tipe_rt.types.RT_EINVAL
