"""ctypes bindings to the CPU oracle (oracle/liboracle.so) and to the
reference leaf build (oracle/_ref/libref_leaf.so).  TEST INFRASTRUCTURE:
imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
only."""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tipe-raytracer_amd"))

from tipe_rt.types import (Vec3, Ray, Material, Sphere, Triangle, Camera, Scene,  # noqa: E402
                           Params, RT_NCOUNTERS)

ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libref_leaf.so")
REF_TRACER_SO = os.path.join(ORACLE_DIR, "_ref", "libref_tracer.so")
REF_TRACER_PHILOX_SO = os.path.join(ORACLE_DIR, "_ref", "libref_tracer_philox.so")


class OracleHit(C.Structure):
    _fields_ = [("didHit", C.c_int), ("dst", C.c_double), ("hitPoint", Vec3),
                ("normal", Vec3), ("mat", Material)]


_oracle = None
_ref = None
_ref_tracer = None
_ref_tracer_philox = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        lib = C.CDLL(ORACLE_SO)
        P = C.POINTER
        lib.oracle_render_rows.argtypes = [P(Scene), P(Params), C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           P(C.c_ulonglong)]
        lib.oracle_render_rows.restype = C.c_int
        lib.oracle_set_math.argtypes = [C.c_int]
        lib.oracle_set_mesh_cull.argtypes = [C.c_int]
        lib.oracle_hit_sphere.argtypes = [Vec3, C.c_double, Ray]
        lib.oracle_hit_sphere.restype = OracleHit
        lib.oracle_hit_sphere_cuda.argtypes = [Vec3, C.c_double, Ray]
        lib.oracle_hit_sphere_cuda.restype = OracleHit
        lib.oracle_hit_triangle.argtypes = [P(Triangle), Ray]
        lib.oracle_hit_triangle.restype = OracleHit
        lib.oracle_tri_uvmapping.argtypes = [P(Triangle), P(OracleHit), P(Material), C.c_int, C.c_int,
                                             C.c_int, P(C.c_int)]
        lib.oracle_tri_uvmapping.restype = Material
        lib.oracle_refracted_vec.argtypes = [Vec3, Vec3, C.c_double, C.c_double]
        lib.oracle_refracted_vec.restype = Vec3
        lib.oracle_reflected_vec.argtypes = [Vec3, Vec3]
        lib.oracle_reflected_vec.restype = Vec3
        lib.oracle_write_color_canva.argtypes = [Vec3, C.c_int]
        lib.oracle_write_color_canva.restype = Vec3
        lib.oracle_rgb_to_hsl.argtypes = [Vec3]
        lib.oracle_rgb_to_hsl.restype = Vec3
        lib.oracle_hsl_to_rgb.argtypes = [Vec3]
        lib.oracle_hsl_to_rgb.restype = Vec3
        lib.oracle_init_camera.argtypes = [Vec3, Vec3, Vec3, C.c_double, C.c_double]
        lib.oracle_init_camera.restype = Camera
        lib.oracle_get_ray.argtypes = [C.c_double, C.c_double, P(Camera), C.c_double, C.c_double, C.c_double]
        lib.oracle_get_ray.restype = Ray
        lib.oracle_trace_sample.argtypes = [P(Scene), P(Params), Ray, C.c_uint, C.c_uint, P(Vec3)]
        lib.oracle_pile_sequence.argtypes = [P(C.c_double), P(C.c_int), C.c_int, P(C.c_double), P(C.c_double)]
        lib.oracle_pm_acos.argtypes = [C.c_double]
        lib.oracle_pm_acos.restype = C.c_double
        lib.oracle_pm_sinf.argtypes = [C.c_float]
        lib.oracle_pm_sinf.restype = C.c_float
        lib.oracle_pm_cosf.argtypes = [C.c_float]
        lib.oracle_pm_cosf.restype = C.c_float
        lib.oracle_pm_pow.argtypes = [C.c_double, C.c_double]
        lib.oracle_pm_pow.restype = C.c_double
        lib.oracle_pm_pow_n.argtypes = [P(C.c_double), P(C.c_double), C.c_longlong]
        lib.oracle_pm_atan2.argtypes = [C.c_double, C.c_double]
        lib.oracle_pm_atan2.restype = C.c_double
        lib.oracle_sky_index.argtypes = [Vec3, C.c_double, Vec3, C.c_int, C.c_int, C.c_int]
        lib.oracle_sky_index.restype = C.c_longlong
        lib.oracle_philox.argtypes = [P(C.c_uint), P(C.c_uint), P(C.c_uint)]
        ull = P(C.c_ulonglong)
        lib.oracle_scan_sincosf.argtypes = [C.c_float, C.c_float, C.c_int, ull, ull, ull]
        lib.oracle_scan_sincosf_cr.argtypes = [C.c_float, C.c_float, C.c_longlong, C.c_int, ull, ull, ull]
        lib.oracle_scan_acos.argtypes = [C.c_longlong, C.c_longlong, C.c_longlong, C.c_int, ull, ull, ull]
        _oracle = lib
    return _oracle


def ref():
    """Reference leaf build, or None when /root/reference was absent."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO):
            if os.path.exists("/root/reference/sphere.h"):
                build_oracle()
            if not os.path.exists(REF_SO):
                return None
        lib = C.CDLL(REF_SO)
        P = C.POINTER
        lib.ref_hit_sphere.argtypes = [P(Vec3), C.c_double, P(Ray), P(OracleHit)]
        lib.ref_hit_triangle.argtypes = [P(Triangle), P(Ray), P(OracleHit)]
        lib.ref_tri_uvmapping.argtypes = [P(Triangle), P(OracleHit), P(Material), C.c_int, C.c_int, C.c_int,
                                          P(C.c_int), P(Material)]
        lib.ref_refracted_vec.argtypes = [P(Vec3), P(Vec3), C.c_double, C.c_double, P(Vec3)]
        lib.ref_reflected_vec.argtypes = [P(Vec3), P(Vec3), P(Vec3)]
        lib.ref_vec3_lerp.argtypes = [P(Vec3), P(Vec3), C.c_double, P(Vec3)]
        lib.ref_write_color_canva.argtypes = [P(Vec3), C.c_int, P(Vec3)]
        lib.ref_rgb_to_hsl.argtypes = [P(Vec3), P(Vec3)]
        lib.ref_hsl_to_rgb.argtypes = [P(Vec3), P(Vec3)]
        lib.ref_init_camera.argtypes = [P(Vec3), P(Vec3), P(Vec3), C.c_double, C.c_double, P(Camera)]
        lib.ref_get_ray.argtypes = [C.c_double, C.c_double, P(Camera), C.c_double, C.c_double, C.c_double, P(Ray)]
        lib.ref_srand.argtypes = [C.c_uint]
        lib.ref_rand.restype = C.c_int
        lib.ref_randomDouble.argtypes = [C.c_double, C.c_double]
        lib.ref_randomDouble.restype = C.c_double
        lib.ref_random_dir_no_norm.argtypes = [P(Vec3)]
        lib.ref_pile_sequence.argtypes = [P(C.c_double), P(C.c_int), C.c_int, P(C.c_double), P(C.c_double)]
        lib.ref_list_of_mesh.argtypes = [C.c_char_p, C.c_char_p, P(C.c_int), P(C.c_int), P(P(C.c_int))]
        lib.ref_list_of_mesh.restype = P(Triangle)
        lib.ref_load_textures.argtypes = [C.c_char_p, C.c_char_p, P(C.c_int), P(C.c_int)]
        lib.ref_load_textures.restype = P(Material)
        lib.ref_move_mesh.argtypes = [C.c_double, C.c_double, C.c_double, P(Triangle), C.c_int]
        lib.ref_free.argtypes = [C.c_void_p]
        _ref = lib
    return _ref


def ref_tracer():
    """The reference's own main.c:22-284 + denoiser.h:11-29 compiled verbatim
    (oracle/build_ref_tracer.sh), or None when /root/reference was absent."""
    global _ref_tracer
    if _ref_tracer is None:
        if not os.path.exists(REF_TRACER_SO):
            if os.path.exists("/root/reference/main.c"):
                build_oracle()
            if not os.path.exists(REF_TRACER_SO):
                return None
        lib = C.CDLL(REF_TRACER_SO)
        P = C.POINTER
        geo = [P(Sphere), C.c_int, P(Triangle), C.c_int, P(Material), C.c_int, C.c_int, P(C.c_int), P(Camera),
               C.c_int, C.c_int, C.c_int, C.c_int]
        lib.ref_fill_canva.argtypes = geo + [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.c_void_p, C.c_void_p, C.c_void_p]
        lib.ref_fill_canva.restype = C.c_int
        lib.ref_trace_rows.argtypes = geo + [C.c_double, C.c_double, C.c_double, C.c_int, C.c_double, C.c_int,
                                             C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.ref_trace_rows.restype = C.c_int
        lib.ref_tracer_srand.argtypes = [C.c_uint]
        _ref_tracer = lib
    return _ref_tracer


def ref_tracer_philox():
    """main.c:22-284 + denoiser.h:11-29 compiled verbatim with the GPU's
    stream spec in place of glibc rand() / libm (oracle/ref_tracer_stream.h),
    or None when /root/reference was absent."""
    global _ref_tracer_philox
    if _ref_tracer_philox is None:
        if not os.path.exists(REF_TRACER_PHILOX_SO):
            if os.path.exists("/root/reference/main.c"):
                build_oracle()
            if not os.path.exists(REF_TRACER_PHILOX_SO):
                return None
        lib = C.CDLL(REF_TRACER_PHILOX_SO)
        P = C.POINTER
        lib.ref_trace_rows_philox.argtypes = [P(Sphere), C.c_int, P(Triangle), C.c_int, P(Material), C.c_int,
                                              C.c_int, P(C.c_int), P(Camera), C.c_int, C.c_int, C.c_int, C.c_int,
                                              C.c_double, C.c_double, C.c_double, C.c_int, C.c_double,
                                              C.c_ulonglong, C.c_int, C.c_int, C.c_int,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.ref_trace_rows_philox.restype = C.c_int
        _ref_tracer_philox = lib
    return _ref_tracer_philox


def counters():
    return (C.c_ulonglong * RT_NCOUNTERS)()
