"""ctypes mirrors of include/rt/types.h and include/rt/rt.h (layout-identical
to the reference's vec3/material/sphere/triangle/camera/ThreadData)."""
import ctypes as C

RT_OK, RT_EINVAL, RT_EDEVICE, RT_ENOMEM, RT_EUNSUPPORTED = 0, -1, -2, -3, -4
RT_RNG_PHILOX, RT_RNG_GLIBC = 0, 1
RT_SPP_CHUNKS_AUTO, RT_SPP_CHUNKS_DEFAULT = -1, 32


def rt_resolve_spp_chunks(spp_chunks, spp):
    """rt.h rt_resolve_spp_chunks: the slice count a launch uses."""
    p = RT_SPP_CHUNKS_DEFAULT if spp_chunks == RT_SPP_CHUNKS_AUTO else spp_chunks
    return 1 if (p <= 1 or spp <= 1) else min(p, spp)


def rt_chunk_taper_levels(S, P):
    """rt.h rt_chunk_taper_levels: 5 (P >= 8, S >= 32 P), 3 (P >= 5, S >= 8 P) or 0."""
    if P >= 8 and S >= 32 * P:
        return 5
    if P >= 5 and S >= 8 * P:
        return 3
    return 0


def rt_chunk_bound(c, S, P):
    """rt.h rt_chunk_bound: first sample of slice c of S samples in P slices
    (equal slices, or P - L equal ones of weight 2^L then L tapered, weights
    2^(L-1) .. 1)."""
    L = rt_chunk_taper_levels(S, P)
    if not L:
        return c * S // P
    one, E = 1 << L, P - L
    U = E * one + one - 1
    w = one * c if c <= E else one * E + one - (one >> (c - E))
    return w * S // U


(RT_CNT_SAMPLES, RT_CNT_CASTS, RT_CNT_SPHERE_TESTS, RT_CNT_SPHERE_DISC,
 RT_CNT_TRI_TESTS, RT_CNT_SHADE, RT_CNT_TEX_HITS, RT_CNT_REFRACT,
 RT_CNT_RNG_DRAWS, RT_CNT_EXACT_RESCANS, RT_CNT_BVH_NODES, RT_CNT_BVH_TRI_TESTS,
 RT_CNT_BVH_LANE_SLOTS, RT_CNT_LEAF_LANE_SLOTS, RT_CNT_CAST_LANE_SLOTS, RT_CNT_SHADE_LANE_SLOTS,
 RT_CNT_BVH_STACK_OVER, RT_NCOUNTERS) = range(18)
COUNTER_NAMES = ["samples", "casts", "sphere_tests", "sphere_disc", "tri_tests",
                 "shade", "tex_hits", "refract", "rng_draws", "exact_rescans",
                 "bvh_nodes", "bvh_tri_tests", "bvh_lane_slots", "leaf_lane_slots", "cast_lane_slots",
                 "shade_lane_slots", "bvh_stack_over"]
RT_ACCEL_AUTO, RT_ACCEL_NONE = 0, 1
RT_SKY_OFF, RT_SKY_LAST_SPHERE = 0, 1
RT_SEM_MAIN_C, RT_SEM_CUDA = 0, 1
RT_PREC_FP64, RT_PREC_FP32 = 0, 1
RT_GATHER_RCCL, RT_GATHER_PEER = 0, 1
RT_ABI_VERSION = 4


class Vec3(C.Structure):
    _fields_ = [("e", C.c_double * 3)]

    def __init__(self, x=0.0, y=0.0, z=0.0):
        super().__init__()
        self.e[0], self.e[1], self.e[2] = x, y, z

    def tolist(self):
        return [self.e[0], self.e[1], self.e[2]]

    def __repr__(self):
        return "Vec3(%r, %r, %r)" % tuple(self.tolist())


class Ray(C.Structure):
    _fields_ = [("origin", Vec3), ("dir", Vec3)]


class Material(C.Structure):
    _fields_ = [("diffuseColor", Vec3), ("emissionColor", Vec3),
                ("emissionStrength", C.c_double), ("reflectionStrength", C.c_double),
                ("alpha", C.c_double), ("materialIndex", C.c_double)]


class Sphere(C.Structure):
    _fields_ = [("center", Vec3), ("radius", C.c_double), ("mat", Material)]


class UV(C.Structure):
    _fields_ = [("u", C.c_double), ("v", C.c_double)]


class Triangle(C.Structure):
    _fields_ = [("A", Vec3), ("B", Vec3), ("C", Vec3), ("mat", Material),
                ("uvA", UV), ("uvB", UV), ("uvC", UV)]


class Camera(C.Structure):
    _fields_ = [("origin", Vec3), ("horizontal", Vec3), ("vertical", Vec3),
                ("coin_bas_gauche", Vec3)]


class ThreadData(C.Structure):
    """main.c:22-46 struct ThreadData."""
    _fields_ = [("start_row", C.c_int), ("end_row", C.c_int),
                ("canva", C.POINTER(Vec3)), ("albedo_tab", C.POINTER(Vec3)),
                ("normal_tab", C.POINTER(Vec3)), ("tex_list", C.POINTER(Vec3)),
                ("mat_list", C.POINTER(Material)), ("sky_mat_list", C.POINTER(Material)),
                ("cam", Camera),
                ("largeur_image", C.c_int), ("hauteur_image", C.c_int),
                ("tex_width", C.c_int), ("tex_height", C.c_int),
                ("sky_width", C.c_int), ("sky_height", C.c_int),
                ("quelMatPourTri", C.POINTER(C.c_int)),
                ("nbRayonParPixel", C.c_int), ("nbRebondMax", C.c_int),
                ("total_pixels", C.c_int),
                ("sphere_list", C.POINTER(Sphere)), ("triangle_list", C.POINTER(Triangle)),
                ("nbSpheres", C.c_int), ("nbTriangles", C.c_int),
                ("ouverture_x", C.c_int), ("ouverture_y", C.c_int), ("focus_distance", C.c_int),
                ("AO_intensity", C.c_int), ("useAO", C.c_bool)]


class Scene(C.Structure):
    _fields_ = [("sphere_list", C.POINTER(Sphere)), ("nbSpheres", C.c_int),
                ("triangle_list", C.POINTER(Triangle)), ("nbTriangles", C.c_int),
                ("mat_list", C.POINTER(Material)),
                ("tex_width", C.c_int), ("tex_height", C.c_int), ("nbMaterials", C.c_int),
                ("quelMatPourTri", C.POINTER(C.c_int)),
                ("sky_mat_list", C.POINTER(Material)), ("sky_width", C.c_int), ("sky_height", C.c_int)]


class Params(C.Structure):
    _fields_ = [("largeur_image", C.c_int), ("hauteur_image", C.c_int),
                ("nbRayonParPixel", C.c_int), ("nbRebondMax", C.c_int),
                ("cam", Camera),
                ("focus_distance", C.c_double),
                ("ouverture_x", C.c_double), ("ouverture_y", C.c_double),
                ("AO_intensity", C.c_double), ("useAO", C.c_int),
                ("compat_int_truncation", C.c_int), ("rng", C.c_int),
                ("spp_chunks", C.c_int), ("seed", C.c_ulonglong), ("accel", C.c_int),
                ("sky_mode", C.c_int), ("semantics", C.c_int), ("precision", C.c_int),
                ("gather", C.c_int)]


class Tiling(C.Structure):
    _fields_ = [("row_base", C.c_int), ("tile_rows", C.c_int), ("tile_first", C.c_int),
                ("tile_step", C.c_int), ("n_tiles", C.c_int)]


class Frame(C.Structure):
    _fields_ = [("canva", C.c_void_p), ("albedo", C.c_void_p),
                ("normal", C.c_void_p), ("radiance", C.c_void_p)]


assert C.sizeof(Vec3) == 24 and C.sizeof(Material) == 80 and C.sizeof(Sphere) == 112
assert C.sizeof(Triangle) == 200 and C.sizeof(Camera) == 96 and C.sizeof(ThreadData) == 248
