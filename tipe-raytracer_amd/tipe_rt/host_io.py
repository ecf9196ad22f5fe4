"""ctypes mirror of the C host library (include/rt/host.h, librt_host.so):
OBJ/MTL mesh loading, texture tables and PPM IO, for Python callers and the
fixture scripts.  The C library is the implementation; this only marshals."""
import ctypes as C

from . import host
from .types import Vec3, Triangle, Material

RT_OBJ_COMPAT_QUADS = 0
RT_OBJ_FAN_QUADS = 1


class Mesh(C.Structure):
    """rt_mesh, host.h."""
    _fields_ = [("triangles", C.POINTER(Triangle)), ("nbTriangles", C.c_int),
                ("quelMatPourTri", C.POINTER(C.c_int)), ("nbMaterials", C.c_int),
                ("material_names", C.POINTER(C.c_char_p)), ("texture_paths", C.POINTER(C.c_char_p)),
                ("kd", C.POINTER(Vec3)), ("ns", C.POINTER(C.c_double))]


def lib():
    H = host()
    H.rt_host_load_obj.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(Mesh)]
    H.rt_host_load_textures.argtypes = [C.POINTER(Mesh), C.c_int, C.POINTER(C.POINTER(Material)),
                                        C.POINTER(C.c_int), C.POINTER(C.c_int)]
    H.rt_host_free_mesh.argtypes = [C.POINTER(Mesh)]
    H.rt_host_read_ppm.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                   C.POINTER(C.POINTER(C.c_int))]
    H.rt_host_write_ppm.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int]
    H.rt_host_free.argtypes = [C.c_void_p]
    H.rt_host_move_mesh.argtypes = [C.c_double, C.c_double, C.c_double, C.POINTER(Triangle), C.c_int]
    return H


def load(obj, mtl, mode=RT_OBJ_COMPAT_QUADS, kd_fallback=1):
    """rt_host_load_obj + rt_host_load_textures.  Returns (rc, mesh, (mats,
    tw, th)); the caller frees with free_mesh / rt_host_free."""
    H = lib()
    m = Mesh()
    rc = H.rt_host_load_obj(obj.encode(), mtl.encode() if mtl else None, mode, C.byref(m))
    if rc:
        return rc, None, None
    mats = C.POINTER(Material)()
    tw, th = C.c_int(), C.c_int()
    rc = H.rt_host_load_textures(C.byref(m), kd_fallback, C.byref(mats), C.byref(tw), C.byref(th))
    return rc, m, (mats, tw.value, th.value)


def free(mesh, mats=None):
    H = lib()
    if mats:
        H.rt_host_free(C.cast(mats, C.c_void_p))
    H.rt_host_free_mesh(C.byref(mesh))
