"""bench.py's multi-GPU launch contract.

The driver's scaling run invokes `python3 bench.py --gpus N` with no
torch.distributed environment.  bench.py must then start N rank processes
itself (never exec from a GPU process), report n_gpus = N, and refuse to run
when fewer than N GPUs are visible for the RCCL backend instead of silently
rendering on one GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-3000:]
    return json.loads(lines[0])


def test_gpus_n_without_devices_fails_loudly():
    """No GPU here (or fewer than N on a box): exit 2 and no JSON line, rather
    than a one-GPU number labelled N."""
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1",
                        "--warmup", "0", "--no-extras", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs %d visible GPUs" % n in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_zero_rejected():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"],
                       capture_output=True, text=True, timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode != 0


@pytest.mark.gpu
def test_gpus_2_spawns_two_ranks_and_verifies():
    """Two ranks on the one-GPU box (gloo gather through host copies), as the
    8-GPU run does with RCCL: n_gpus must be 2, the assembled frame must equal
    a single-device render bit for bit, and the single-process leg
    (rt_render_gather_async over both slots) must too.  The C3 / C4 / C5
    legs (row-tiled over the ranks at a reduced 2 spp) must each assemble
    the single-device frame bit for bit -- C4 through the BVH queue kernel
    on cyclic tiles, C5 at 3840x2880."""
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend",
                        "gloo", "--steps", "1", "--warmup", "0", "--no-extras", "--no-cpu-baseline", "--verify",
                        "--config-spp", "2"],
                       capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2
    assert rec["verified_vs_single_device"] is True
    assert rec["config"]["parallelism"] == "row-tiles x2"
    sp = rec["single_process"]
    assert sp["verified_vs_single_device"] is True
    assert len(sp["devices"]) == 2
    assert rec["value"] > 0
    assert sorted(rec["configs"]) == ["C3", "C4", "C5"]
    for name, c in rec["configs"].items():
        assert c["n_gpus"] == 2 and c["spp"] == 2, name
        assert c["verified_vs_single_device"] is True, name
        assert c["msamples_per_s"] > 0 and c["gather_ms"] >= 0, name
    assert rec["configs"]["C5"]["rows_per_rank"] == 1440
