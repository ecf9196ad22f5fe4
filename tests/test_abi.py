"""C-ABI boundary (no GPU needed): the libraries load, export every entry
point their headers declare, the reference-shaped structs have the
reference's x86-64 layout, and argument validation fails loudly before any
device work."""
import ctypes as C
import os
import re
import subprocess

import pytest

import tipe_rt
from tipe_rt import types as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include", "rt")


def declared(header):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"static inline[^{;]*\{.*?\n\}", "", src, flags=re.S)   # header-only helpers
    return sorted(set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", src)) - {"rt_version_t"})


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_rt_h_symbols_exported():
    syms = exported(tipe_rt.LIB_PATH)
    missing = [s for s in declared("rt.h") if s not in syms]
    assert not missing, missing
    assert set(tipe_rt.EXPORTED_SYMBOLS) <= syms


def test_host_h_symbols_exported():
    syms = exported(tipe_rt.HOST_LIB_PATH)
    missing = [s for s in declared("host.h") if s not in syms]
    assert not missing, missing


def test_library_loads_and_reports_version():
    L = tipe_rt.lib()
    assert b"gfx950" in L.rt_version()
    assert b"(abi %d," % L.rt_abi_version() in L.rt_version()       # the string names the ABI it exports
    p = T.Params()
    L.rt_params_init(C.byref(p))
    assert p.rng == T.RT_RNG_PHILOX and p.seed == 1010 and p.compat_int_truncation == 1 and p.spp_chunks == T.RT_SPP_CHUNKS_AUTO
    assert p.gather == T.RT_GATHER_RCCL
    assert L.rt_abi_version() == T.RT_ABI_VERSION


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "rt/rt.h"
#define P(t) printf(#t " %zu\n", sizeof(t))
#define O(t, f) printf(#t "." #f " %zu\n", offsetof(t, f))
int main(void) {
  P(rt_vec3); P(rt_material); P(rt_sphere); P(rt_triangle); P(rt_camera); P(rt_thread_data);
  P(rt_scene); P(rt_params); P(rt_tiling); P(rt_frame);
  O(rt_material, alpha); O(rt_triangle, uvB); O(rt_thread_data, nbRayonParPixel);
  O(rt_thread_data, triangle_list); O(rt_thread_data, AO_intensity); O(rt_scene, quelMatPourTri);
  O(rt_params, cam); O(rt_params, focus_distance); O(rt_params, rng); O(rt_params, spp_chunks);
  O(rt_params, seed); O(rt_params, semantics); O(rt_params, precision); O(rt_params, gather);
  O(rt_frame, radiance);
  return 0;
}
"""


def test_struct_layouts_match_ctypes_mirror(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.splitlines())
    got = {k: int(v) for k, v in got.items()}
    mirror = {"rt_vec3": T.Vec3, "rt_material": T.Material, "rt_sphere": T.Sphere, "rt_triangle": T.Triangle,
              "rt_camera": T.Camera, "rt_thread_data": T.ThreadData, "rt_scene": T.Scene, "rt_params": T.Params,
              "rt_tiling": T.Tiling, "rt_frame": T.Frame}
    for name, cls in mirror.items():
        assert got[name] == C.sizeof(cls), name
    for key, val in got.items():
        if "." in key:
            t, f = key.split(".")
            assert getattr(mirror[t], f).offset == val, key
    # the reference's own sizes
    assert (got["rt_material"], got["rt_sphere"], got["rt_triangle"], got["rt_camera"],
            got["rt_thread_data"]) == (80, 112, 200, 96, 248)


def test_validation_errors_without_device():
    L = tipe_rt.lib()
    sc = T.Scene()
    p = T.Params()
    L.rt_params_init(C.byref(p))
    p.largeur_image, p.hauteur_image, p.nbRayonParPixel, p.nbRebondMax = 8, 6, 1, 5
    buf = (C.c_double * (8 * 6 * 3))()
    assert L.rt_render_rows(None, C.byref(p), 5, 0, buf, None, None) == T.RT_EINVAL
    assert L.rt_render_rows(C.byref(sc), C.byref(p), 6, 0, buf, None, None) == T.RT_EINVAL   # row out of range
    p.nbRayonParPixel = 0
    assert L.rt_render_rows(C.byref(sc), C.byref(p), 5, 0, buf, None, None) == T.RT_EINVAL
    assert b"nbRayonParPixel" in L.rt_last_error()
    p.nbRayonParPixel = 1
    p.rng = T.RT_RNG_GLIBC
    assert L.rt_render_rows(C.byref(sc), C.byref(p), 5, 0, buf, None, None) == T.RT_EUNSUPPORTED
    sc.nbTriangles = 1                    # triangles without arrays
    p.rng = T.RT_RNG_PHILOX
    assert L.rt_render_rows(C.byref(sc), C.byref(p), 5, 0, buf, None, None) == T.RT_EINVAL
    assert L.rt_assemble_async(None, 0, 1, 1, 1, 1, 1, None, None) == T.RT_EINVAL
    assert L.rt_selftest_math(10, buf, buf, 1) == T.RT_EINVAL


def test_product_has_no_cpu_fallback(monkeypatch, tmp_path):
    """The Python mirror refuses to run without librt_hip.so."""
    import importlib
    monkeypatch.setenv("RT_HIP_LIB", str(tmp_path / "nope.so"))
    mod = importlib.reload(tipe_rt)
    try:
        mod._lib = None
        with pytest.raises(RuntimeError, match="no CPU fallback"):
            mod.lib()
    finally:
        monkeypatch.delenv("RT_HIP_LIB")
        importlib.reload(tipe_rt)


def test_kernel_resource_usage_builds_for_gfx950():
    """The HIP sources cross-compile for gfx950 within the VGPR/spill
    budgets recorded in DESIGN.md (build check, no GPU)."""
    out = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tipe-raytracer_amd"), "resource-usage"],
                         capture_output=True, text=True)
    txt = out.stdout + out.stderr
    budgets = {"ILb0ELb0ELb0E": (128, 48),    # sphere scenes: 4 waves/SIMD
               "ILb0ELb1ELb0E": (168, 40),    # BVH scenes: 3 waves/SIMD (LDS stack)
               "_qILb0ELi0ELin2E": (104, 0),  # sphere-only scenes, opaque materials (C2), r04: 97 VGPRs with
                                              # incomingLight / rayColor in LDS (109 before), no spills
               "_qILb0ELi0ELin1E": (112, 0),  # sphere-only scenes, r04: no triangle code, 104 VGPRs, no spills
               "_qILb0ELi0ELi0E": (128, 4),   # sphere + brute-force triangle scenes with spp_chunks > 1 (no AO;
                                              # 1 slot since the LDS task table, r03: C2 +3.5 % net; 3 since
                                              # the candidate pass's second minimum, r04: C2 +4.3 % net)
               "_qILb0ELi1ELi0E": (128, 12),  # the task-queue kernel with AO rays
               "_qILb0ELi1ELi3ELb0E": (128, 24),  # ... on BVH scenes (resumable walks), with AO
               "_qILb0ELi1ELi3ELb1E": (128, 2)}   # ... opaque materials (C4), r04: no spills with incomingLight
                                                  # in LDS (4 without, 18 before the opaque instantiation)
    for sym, (max_vgpr, max_spill) in budgets.items():
        m = re.search(r"render_kernel" + sym + r".*?VGPRs: (\d+).*?VGPRs Spill: (\d+)", txt, re.S)
        assert m, txt[-2000:]
        vgprs, spills = int(m.group(1)), int(m.group(2))
        assert vgprs <= max_vgpr and spills <= max_spill, (sym, vgprs, spills)


CHUNK_C = r"""
#include <stdio.h>
#include "rt/rt.h"
int main(void) {
  const int S[] = {1, 2, 7, 8, 39, 40, 100, 383, 384, 1000, 2000, 5000, 1 << 30};
  const int P[] = {1, 2, 4, 5, 6, 8, 11, 12, 13, 16, 32, 64};
  for (unsigned i = 0; i < sizeof S / sizeof S[0]; ++i)
    for (unsigned j = 0; j < sizeof P / sizeof P[0]; ++j) {
      int p = rt_resolve_spp_chunks(P[j], S[i]);
      for (int c = 0; c <= p; ++c) printf("%d %d %d %lld\n", S[i], p, c, rt_chunk_bound(c, S[i], p));
    }
  return 0;
}
"""


def test_chunk_bounds_header_matches_mirror(tmp_path):
    """rt.h rt_chunk_bound (compiled here) equals the Python mirror; slices
    cover [0, S) in order, are non-empty, equal before the taper and halve
    over the last three when tapered."""
    src = tmp_path / "chunks.c"
    src.write_text(CHUNK_C)
    exe = tmp_path / "chunks"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    rows = [tuple(int(x) for x in line.split()) for line in
            subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines()]
    by = {}
    for S, P, c, b in rows:
        assert b == T.rt_chunk_bound(c, S, P), (S, P, c)
        by.setdefault((S, P), {})[c] = b
    for (S, P), d in by.items():
        bs = [d[c] for c in range(P + 1)]
        assert bs[0] == 0 and bs[-1] == S and len(bs) == P + 1
        sizes = [bs[c + 1] - bs[c] for c in range(P)]
        assert min(sizes) >= 1, (S, P, sizes)
        L = T.rt_chunk_taper_levels(S, P)
        assert L == (5 if P >= 8 and S >= 32 * P else 3 if P >= 5 and S >= 8 * P else 0)
        if L:
            full = sizes[:P - L]
            assert max(full) - min(full) <= 1
            tail = sizes[P - L:]
            assert tail[0] < min(full) and all(b <= a for a, b in zip(tail, tail[1:])), (S, P, sizes)
            assert tail[-1] * (1 << L) <= min(full) + (1 << L), (S, P, sizes)   # about 2^-L of a full slice
    assert T.rt_chunk_bound(29, 1000, 32) == 970 and T.rt_chunk_bound(31, 1000, 32) == 995   # L = 3
    # L = 5 at 12 slices: 7 x 125.5, then 62.7, 31.4, 15.7, 7.8, 3.9 samples
    assert [T.rt_chunk_bound(c, 1000, 12) for c in (7, 8, 11, 12)] == [878, 941, 996, 1000]
