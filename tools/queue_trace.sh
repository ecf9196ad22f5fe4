#!/bin/bash
# Per-lane start/end clocks, rounds and tasks of render_kernel_q (C2, 1 launch).
rm -f gpurun_out/qtrace.bin
RT_QUEUE_TRACE=gpurun_out/qtrace.bin timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'tipe-raytracer_amd'); sys.path.insert(0, '.')
import torch, tipe_rt, bench
from tipe_rt import scenes
cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ('origin', 'target', 'up', 'vfov', 'ratio')})
p = tipe_rt.make_params(1200, 900, int(sys.argv[1]), 6, cam, focus=3.0, seed=1010, chunks=32)
ds = tipe_rt.DeviceScene(tipe_rt.make_scene(scenes.cornell_spheres()), 0)
out = torch.empty((3, 900, 1200, 3), dtype=torch.float64, device='cuda:0')
tipe_rt.render_async(ds, p, tipe_rt.band_tiling(0, 899), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), None, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
" ${SPP:-250}
