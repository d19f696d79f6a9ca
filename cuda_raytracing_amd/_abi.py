"""ctypes mirror of include/rt_render.h, include/rt_host.h and include/rt_ref_layout.h.

The C-ABI is the product boundary.  This module only declares the structs
and loads the shared libraries; it contains no rendering logic.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_DIR = PKG_DIR / "lib"
# RT_HIP_LIB: another build of the render library (same-box A/B of two trees, tools/gpu_ab_env.sh); default in-tree
HIP_LIB = Path(os.environ["RT_HIP_LIB"]) if os.environ.get("RT_HIP_LIB") else LIB_DIR / "librt_hip.so"
HOST_LIB = LIB_DIR / "librt_host.so"
ORACLE_LIB = REPO_DIR / "oracle" / "_build" / "liboracle_rt.so"

RT_OK = 0
RT_ERR_INVALID_ARG = -1
RT_ERR_SCENE = -2
RT_ERR_HIP = -3
RT_ERR_NO_DEVICE = -4
RT_ERR_STACK = -5
RT_ERR_UNSUPPORTED = -6
RT_ERR_DEVICE_CHECK = -7

RT_FLAG_COUNT = 0x1
RT_FLAG_GLOBAL_SCENE = 0x2
RT_FLAG_NO_JIT = 0x4
RT_FLAG_FORCE_LANE, RT_FLAG_FORCE_PACKET, RT_FLAG_FORCE_STATIC = 0x8, 0x10, 0x20
RT_FLAG_NO_FOLD = 0x40
RT_FLAG_FORCE_ACCEL, RT_FLAG_NO_ACCEL = 0x80, 0x100
RT_FLAG_RC_AUDIT = 0x200
RT_FLAG_FORCE_MIXED, RT_FLAG_NO_MIXED = 0x400, 0x800
RT_TRAV_LANE, RT_TRAV_PACKET, RT_TRAV_STATIC, RT_TRAV_ACCEL, RT_TRAV_MIXED = 0, 1, 2, 3, 4

CNT_NAMES = [
    "visit_sphere", "visit_bvh", "visit_triangle", "visit_quad", "visit_translate",
    "visit_yrotate", "visit_group", "bounces", "shades", "perlin", "rng_draws", "samples",
    "max_stack", "stack_overflow", "exec_node", "exec_prim",
]

RT_XF_NONE, RT_XF_TRANSLATE, RT_XF_YROTATE, RT_XF_YROTATE_TRANSLATE = 0, 1, 2, 3
RT_SCENE_COUNT = 21
RT_SCENE_RANDOM_10K = 20
HITTABLE_BYTES = 120
TEXTURE_BYTES = 32


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]

    def tolist(self):
        return [self.x, self.y, self.z]


def vec3(x, y, z) -> Vec3:
    return Vec3(float(x), float(y), float(z))


class Material(C.Structure):
    """rtr_material: 24 bytes (raytracing.cu:86-99); treated as an opaque value here."""
    _fields_ = [("kind", C.c_uint32), ("pad_", C.c_uint32), ("payload", C.c_uint8 * 16)]


class Scene(C.Structure):
    _fields_ = [
        ("hittables", C.c_void_p), ("hittable_count", C.c_uint32),
        ("refs", C.POINTER(C.c_uint16)), ("ref_count", C.c_uint32),
        ("root", C.c_uint16), ("pad_", C.c_uint16),
        ("textures", C.POINTER(C.c_uint8)), ("texture_bytes", C.c_uint64),
    ]


class Camera(C.Structure):
    _fields_ = [
        ("pixel00", Vec3), ("delta_u", Vec3), ("delta_v", Vec3), ("center", Vec3),
        ("defocus_u", Vec3), ("defocus_v", Vec3), ("defocus_angle", C.c_float),
    ]


class Params(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("row_offset", C.c_int32), ("row_stride", C.c_int32), ("row_count", C.c_int32),
        ("samples_per_pixel", C.c_int32), ("max_bounces", C.c_int32),
        ("background", Vec3), ("seed", C.c_uint64), ("flags", C.c_uint32), ("pad_", C.c_uint32),
    ]


class KernelInfo(C.Structure):
    """rt_kernel_info (ABI 6): a render kernel as the register allocator built it."""
    _fields_ = [
        ("vgprs", C.c_int32), ("agprs", C.c_int32), ("sgprs", C.c_int32), ("scratch_bytes", C.c_int32),
        ("vgpr_spills", C.c_int32), ("sgpr_spills", C.c_int32), ("blocks_per_cu", C.c_int32), ("run_time", C.c_int32),
        ("compiler", C.c_char * 128), ("loader", C.c_char * 128),
    ]

    def as_dict(self):
        return {"vgprs": self.vgprs, "agprs": self.agprs, "sgprs": self.sgprs, "scratch_bytes": self.scratch_bytes,
                "vgpr_spills": self.vgpr_spills, "sgpr_spills": self.sgpr_spills, "blocks_per_cu": self.blocks_per_cu,
                "run_time": self.run_time, "compiler": self.compiler.decode(errors="replace"),
                "loader": self.loader.decode(errors="replace")}


class Stats(C.Structure):
    _fields_ = [
        ("init_ms", C.c_double), ("render_ms", C.c_double), ("total_ms", C.c_double),
        ("samples", C.c_uint64), ("counters", C.c_uint64 * 16),
        ("stack_needed", C.c_int32), ("scene_in_lds", C.c_int32),
        ("traversal", C.c_int32), ("jit_visits", C.c_int32),
        ("sched_ms", C.c_double),
        ("folded", C.c_int32), ("fold_rerenders", C.c_int32),
        ("accel_spheres", C.c_int32), ("accel_depth", C.c_int32),
        ("accel_fallbacks", C.c_uint32), ("jit_source", C.c_int32), ("jit_ms", C.c_double),
        ("rc_hbm_slots", C.c_uint64), ("rc_lds_levels", C.c_int32), ("mix_macros", C.c_int32),
        ("mix_fallbacks", C.c_uint32), ("tiled_out", C.c_int32),
        ("render_kernel_ms", C.c_double), ("gather_ms", C.c_double), ("devices", C.c_int32), ("rc_pool_chunks", C.c_int32),
        ("kernel", KernelInfo),
    ]

    def counter_dict(self):
        return {n: int(self.counters[i]) for i, n in enumerate(CNT_NAMES) if not n.startswith("reserved")}


class Settings(C.Structure):
    _fields_ = [
        ("img_ratio", C.c_float), ("img_width", C.c_int32), ("samples_per_pixel", C.c_int32),
        ("max_bounces", C.c_int32), ("vfov", C.c_float),
        ("lookfrom", Vec3), ("lookat", Vec3), ("view_up", Vec3),
        ("defocus_angle", C.c_float), ("background", Vec3), ("img_name", C.c_char * 64),
    ]


def _sig(fn, restype, *argtypes):
    fn.restype = restype
    fn.argtypes = list(argtypes)
    return fn


_host = None
_hip = None
_oracle = None


def check_build_stamp(L, prefix: str, path: Path) -> None:
    """Refuse a library built from other sources than this tree's (Makefile `stamp`): it records the files it was built
    from and the sha256 of their bytes; recompute both here.  build() (make) is the only producer of the libraries the
    tests, smoke() and bench.py load, so a stale prebuilt library fails loudly instead of being measured.
    (RT_HIP_LIB — another build for a same-box A/B — is exempt.)"""
    import hashlib
    h = getattr(L, prefix + "_build_hash", None)
    f = getattr(L, prefix + "_build_files", None)
    if h is None or f is None:
        raise RuntimeError(f"{path} carries no build stamp: rebuild with `make` / __graft_entry__.build()")
    h.restype = C.c_char_p
    f.restype = C.c_char_p
    want, files = h().decode(), f().decode().split()
    if want == "unstamped" or not files:
        raise RuntimeError(f"{path} was built without a source stamp: rebuild with `make` / __graft_entry__.build()")
    d = hashlib.sha256()
    for name in files:
        d.update((REPO_DIR / name).read_bytes())
    got = d.hexdigest()[:16]
    if got != want:
        raise RuntimeError(f"{path} was built from other sources (stamp {want}, tree {got}): stale library; rebuild with "
                           "`make` / __graft_entry__.build()")


def host_lib():
    global _host
    if _host is None:
        if not HOST_LIB.exists():
            raise RuntimeError(f"{HOST_LIB} missing: run `make host` (or __graft_entry__.build())")
        L = C.CDLL(str(HOST_LIB))
        check_build_stamp(L, "rt_host", HOST_LIB)
        P = C.c_void_p
        _sig(L.rt_world_create, P, C.c_uint32, C.c_uint64)
        _sig(L.rt_world_destroy, None, P)
        _sig(L.rt_settings_default, None, C.POINTER(Settings))
        _sig(L.rt_world_build_scene, C.c_int, P, C.c_int, C.POINTER(Settings))
        _sig(L.rt_world_build_bvh, C.c_int, P, C.POINTER(C.c_uint16))
        _sig(L.rt_world_scene, C.c_int, P, C.c_uint16, C.POINTER(Scene))
        _sig(L.rt_world_hittable_count, C.c_uint32, P)
        _sig(L.rt_world_ref_count, C.c_uint32, P)
        _sig(L.rt_world_texture_bytes, C.c_uint64, P)
        _sig(L.rt_world_rand, C.c_int32, P)
        _sig(L.rt_scene_name, C.c_char_p, C.c_int)
        for name in ("rt_mat_lambert_solid", "rt_mat_light_solid"):
            _sig(getattr(L, name), Material, P, Vec3)
        _sig(L.rt_mat_lambert_image, Material, P, C.c_char_p)
        _sig(L.rt_mat_lambert_image_pixels, Material, P, P, C.c_int32, C.c_int32)
        _sig(L.rt_world_status, C.c_int, P)
        _sig(L.rt_image_load, C.c_int, C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_int32),
             C.POINTER(C.c_int32))
        _sig(L.rt_image_free, None, C.POINTER(C.c_float))
        _sig(L.rt_mat_lambert_noise, Material, P, C.c_float)
        _sig(L.rt_mat_metal, Material, Vec3, C.c_float)
        _sig(L.rt_mat_dielectric, Material, C.c_float)
        _sig(L.rt_mat_lambert_checker, Material, P, C.c_float, Vec3, Vec3)
        xf = (P, C.c_int, C.c_float, Vec3)
        _sig(L.rt_add_sphere, C.c_int, *xf, Vec3, C.c_float, Material)
        _sig(L.rt_add_moving_sphere, C.c_int, *xf, Vec3, Vec3, C.c_float, Material)
        _sig(L.rt_add_quad, C.c_int, *xf, Vec3, Vec3, Vec3, Material)
        _sig(L.rt_add_triangle, C.c_int, *xf, Vec3, Vec3, Vec3, Material)
        _sig(L.rt_add_box, C.c_int, *xf, Vec3, Vec3, Material)
        _sig(L.rt_add_pyramid, C.c_int, *xf, Vec3, Vec3, Vec3, Material)
        _sig(L.rt_camera_from_settings, C.c_int, C.POINTER(Settings), C.c_int32, C.c_int32,
             C.POINTER(Camera), C.POINTER(C.c_int32), C.POINTER(C.c_int32))
        _sig(L.rt_reference_stack_depth, C.c_int, C.POINTER(Scene), C.POINTER(C.c_uint32))
        _sig(L.rt_tonemap, None, C.c_void_p, C.c_size_t, C.c_void_p)
        _sig(L.rt_write_ppm, C.c_int, C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32)
        _host = L
    return _host


HIP_SYMBOLS = ["rt_render", "rt_context_create", "rt_context_render", "rt_context_render_ppm", "rt_context_timing",
               "rt_context_destroy", "rt_status_string", "rt_device_count", "rt_abi_version",
               "rt_static_source", "rt_static_compile", "rt_context_note", "rt_tonemap_device", "rt_accel_build",
               "rt_seed_states", "rt_kernel_source", "rt_mixed_build", "rt_multi_create", "rt_multi_render",
               "rt_multi_destroy", "rt_render_devices", "rt_multi_row_map", "rt_accel_build_wide", "rt_rng_table_states",
               "rt_accel_build_quant", "rt_prim_lists", "rt_multi_unpermute", "rt_kernel_build",
               "rt_hip_build_hash", "rt_hip_build_files"]


def _bind_single_hip_runtime():
    """Keep ONE HIP runtime per process.

    PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7, the same as /opt/rocm's).  If
    torch's copy is loaded first, librt_hip.so's DT_NEEDED resolves to it by SONAME and the process has
    one runtime.  If ours were loaded first, torch would later map a second runtime and see no GPUs.
    So when torch is installed we import it before dlopen-ing the render library.
    """
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def hip_lib():
    """The MI355X render library.  Raises (never falls back) when it is missing."""
    global _hip
    if _hip is None:
        if not HIP_LIB.exists():
            raise RuntimeError(f"{HIP_LIB} missing: the HIP render path is not built "
                               "(run `make hip` / __graft_entry__.build()); there is no CPU fallback")
        _bind_single_hip_runtime()
        L = C.CDLL(str(HIP_LIB))
        if not os.environ.get("RT_HIP_LIB"):
            check_build_stamp(L, "rt_hip", HIP_LIB)
        P = C.c_void_p

        # (entry points added in ABI 5 are bound when present: RT_HIP_LIB may name an older build for an A/B)
        def opt(name, restype, *argtypes):
            if hasattr(L, name):
                _sig(getattr(L, name), restype, *argtypes)
        _sig(L.rt_render, C.c_int, C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params), P,
             C.POINTER(Stats))
        _sig(L.rt_context_create, C.c_int, C.POINTER(Scene), C.c_int, C.POINTER(C.c_void_p))
        _sig(L.rt_context_render, C.c_int, P, C.POINTER(Camera), C.POINTER(Params), P, P)
        _sig(L.rt_context_render_ppm, C.c_int, P, C.POINTER(Camera), C.POINTER(Params), P, P, P)
        _sig(L.rt_context_timing, C.c_int, P, C.POINTER(Stats))
        _sig(L.rt_context_destroy, None, P)
        _sig(L.rt_status_string, C.c_char_p, C.c_int)
        _sig(L.rt_device_count, C.c_int, C.POINTER(C.c_int))
        _sig(L.rt_abi_version, C.c_int)
        _sig(L.rt_static_source, C.c_int, C.POINTER(Scene), C.c_uint32, C.c_char_p, C.c_uint64,
             C.POINTER(C.c_uint32))
        _sig(L.rt_static_compile, C.c_int, C.POINTER(Scene), C.c_uint32, C.c_char_p, C.c_char_p,
             C.c_uint64)
        _sig(L.rt_context_note, C.c_char_p, P)
        _sig(L.rt_tonemap_device, C.c_int, P, C.c_uint64, P, P)
        _sig(L.rt_accel_build, C.c_int, C.POINTER(Scene), P, C.c_uint64, C.POINTER(C.c_uint32))
        _sig(L.rt_mixed_build, C.c_int, C.POINTER(Scene), C.POINTER(C.c_uint32))
        opt("rt_accel_build_wide", C.c_int, C.POINTER(Scene), P, C.c_uint64, C.POINTER(C.c_uint32))
        opt("rt_accel_build_quant", C.c_int, C.POINTER(Scene), P, C.c_uint64, C.POINTER(C.c_uint32))
        opt("rt_prim_lists", C.c_int, C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params), C.c_uint32, P, P,
            C.POINTER(C.c_float))
        opt("rt_rng_table_states", C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, P)
        _sig(L.rt_seed_states, C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, P)
        _sig(L.rt_kernel_source, C.c_int, C.POINTER(Scene), C.c_int, C.c_int32, C.c_char_p, C.c_uint64)
        opt("rt_kernel_build", C.c_int, C.POINTER(Scene), C.c_int, C.c_int32, C.POINTER(KernelInfo))
        opt("rt_multi_create", C.c_int, C.POINTER(Scene), C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p))
        opt("rt_multi_render", C.c_int, P, C.POINTER(Camera), C.POINTER(Params), P, P, C.POINTER(Stats))
        opt("rt_multi_destroy", None, P)
        opt("rt_render_devices", C.c_int, C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params), C.POINTER(C.c_int),
            C.c_int, P, P, C.POINTER(Stats))
        i32p = C.POINTER(C.c_int32)
        opt("rt_multi_row_map", C.c_int, C.c_int32, C.c_int32, C.c_int32, i32p, i32p, i32p, i32p)
        opt("rt_multi_unpermute", C.c_int, P, P, C.c_int32, C.c_int32, C.c_int32, C.c_uint32, P)
        _hip = L
    return _hip


_oracle_builds: dict = {}


def oracle_lib(path=None):
    """CPU oracle — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).

    path: another build of oracle/oracle_rt.c (bench.py's -O3 -march=native CPU-baseline build)."""
    global _oracle
    if path is None and _oracle is not None:
        return _oracle
    lib_path = ORACLE_LIB if path is None else Path(path)
    if str(lib_path) in _oracle_builds:
        return _oracle_builds[str(lib_path)]
    if not lib_path.exists():
        raise RuntimeError(f"{lib_path} missing: run `make oracle`")
    L = C.CDLL(str(lib_path))
    _sig(L.rt_render_cpu, C.c_int, C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params),
         C.c_void_p, C.POINTER(Stats))
    _sig(L.rt_oracle_sinf, C.c_float, C.c_float)
    _sig(L.rt_oracle_pow5f, C.c_float, C.c_float)
    _sig(L.rt_oracle_atan2f, C.c_float, C.c_float, C.c_float)
    _sig(L.rt_oracle_acosf, C.c_float, C.c_float)
    _sig(L.rt_oracle_uniforms, C.c_int, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int)
    _sig(L.rt_oracle_threads, C.c_int)
    _sig(L.rt_oracle_set_threads, C.c_int, C.c_int)
    _oracle_builds[str(lib_path)] = L
    if path is None:
        _oracle = L
    return L


def status_string(code: int) -> str:
    names = {0: "ok", -1: "invalid argument", -2: "malformed scene", -3: "HIP runtime error",
             -4: "no HIP device", -5: "traversal stack too deep", -6: "unsupported", -7: "device check failed"}
    return names.get(code, f"status {code}")


def env_threads() -> int:
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
