"""Stress counts of the sphere candidate pass (rt_verify_sphere_pass) on the
README box and the adversarial sphere scene: python tools/verify_sphere_pass.py [n]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))

import torch  # noqa: E402,F401  (before librt_hip.so)

import helpers  # noqa: E402
import test_gpu_parity as t  # noqa: E402
import tipe_rt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
for which, seed in (("cornell", 7), ("adversarial", 8)):
    b = helpers.cornell() if which == "cornell" else t.adversarial_sphere_scene()
    fb, bad = tipe_rt.verify_sphere_pass(b.scene, t._stress_rays(b.spheres, n, seed))
    print(json.dumps({"scene": which, "rays": n, "exact_fallbacks": fb, "mismatches": bad}), flush=True)
