"""FP32 mode vs FP64: image-mean differences at high spp against the
seed-to-seed Monte-Carlo spread (is the fp32 difference bias or noise?).
GPU only.  Prints one JSON line per scene."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
import helpers  # noqa: E402
from test_gpu_parity import gpu_render  # noqa: E402
from tipe_rt import types as T  # noqa: E402


def means(bundle, p):
    r = np.nan_to_num(gpu_render(bundle, p)[3])
    return r.reshape(-1, 3).mean(0)


for name, mk in (("cornell", lambda: (helpers.cornell(), helpers.params(160, 120, 1024, 6, chunks=32))),
                 ("pyramid", lambda: (helpers.pyramid_scene(), helpers.params(160, 120, 512, 6, chunks=32)))):
    bundle, p = mk()
    m64 = means(bundle, p)
    seeds = []
    for sd in (1011, 1012, 1013):
        p.seed = sd
        seeds.append(means(bundle, p))
    p.seed = 1010
    p.precision = T.RT_PREC_FP32
    m32 = means(bundle, p)
    spread = np.std(np.array(seeds + [m64]), axis=0, ddof=1)
    print(json.dumps({"scene": name, "spp": p.nbRayonParPixel, "rel_fp32_minus_fp64": list(np.round((m32 - m64) / m64, 5)),
                      "rel_seed_spread": list(np.round(spread / m64, 5))}), flush=True)
