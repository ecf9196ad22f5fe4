import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librt_hip.so on cuda:0)")
    config.addinivalue_line("markers", "slow: CPU test taking more than ~10 s")

# Import torch (when present) before anything loads librt_hip.so, so both
# share torch's bundled HIP runtime (same SONAME libamdhip64.so.7) instead of
# pulling a second runtime into the process.
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover - CPU-only environments
    torch = None
