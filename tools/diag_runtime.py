"""Diagnostic: HIP runtime sharing between torch and librt_hip.so."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch
print("torch.cuda", torch.cuda.is_available(), torch.cuda.device_count(), torch.version.hip, flush=True)
h = ctypes.CDLL("libamdhip64.so.7")
n = ctypes.c_int()
print("hipGetDeviceCount via soname", h.hipGetDeviceCount(ctypes.byref(n)), n.value, flush=True)
path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tipe-raytracer_amd", "librt_hip.so")
L = ctypes.CDLL(path)
print("loaded", path, flush=True)
print("hipGetDeviceCount after load", h.hipGetDeviceCount(ctypes.byref(n)), n.value, flush=True)
L.rt_device_count.restype = ctypes.c_int
print("rt_device_count", L.rt_device_count(), flush=True)
for l in open('/proc/self/maps'):
    if 'amdhip' in l or 'hsa-runtime' in l:
        print(l.split()[-1])
