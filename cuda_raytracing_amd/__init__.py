"""cuda_raytracing_amd — MI355X-native drop-in for luk-zm/cuda_raytracing's per-pixel render path.

Layers:
  host (librt_host.so, C++)   scene catalog + builder API, BVH, camera, tonemap/PPM
  device (librt_hip.so, HIP)  rt_render / rt_context_*: RNG seeding + the render kernel on gfx950
  this module                 thin Python mirror of the reference's surface for tests and bench

The render entry points call the HIP library only; a missing library is an error, never a fallback.
"""
from __future__ import annotations

import ctypes as C
import numpy as np

from . import _abi
from ._abi import (Camera, Params, Scene, Settings, Stats, Vec3, vec3, RT_FLAG_COUNT,
                   RT_FLAG_GLOBAL_SCENE, RT_FLAG_NO_JIT, RT_FLAG_FORCE_LANE, RT_FLAG_FORCE_PACKET,
                   RT_FLAG_FORCE_STATIC, RT_FLAG_NO_FOLD, RT_FLAG_FORCE_ACCEL, RT_FLAG_NO_ACCEL, RT_FLAG_RC_AUDIT, RT_FLAG_FORCE_MIXED, RT_FLAG_NO_MIXED, RT_TRAV_MIXED, RT_TRAV_LANE, RT_TRAV_PACKET, RT_TRAV_STATIC, RT_TRAV_ACCEL, RT_SCENE_COUNT, RT_SCENE_RANDOM_10K, RT_XF_NONE,
                   RT_XF_TRANSLATE, RT_XF_YROTATE, RT_XF_YROTATE_TRANSLATE)

__all__ = [
    "World", "Camera", "Params", "Scene", "Settings", "Stats", "vec3", "build_scene",
    "camera_from_settings", "make_params", "render", "RenderContext", "tonemap", "write_ppm",
    "scene_name", "BlobScene", "shard_rows", "unshard", "RT_FLAG_COUNT", "RT_FLAG_GLOBAL_SCENE",
    "RT_FLAG_NO_JIT", "RT_FLAG_RC_AUDIT", "RT_FLAG_FORCE_MIXED", "RT_FLAG_NO_MIXED", "RT_TRAV_MIXED", "RT_FLAG_FORCE_LANE", "RT_FLAG_FORCE_PACKET", "RT_FLAG_FORCE_STATIC", "RT_FLAG_NO_FOLD", "RT_FLAG_FORCE_ACCEL", "RT_FLAG_NO_ACCEL", "RT_TRAV_ACCEL", "RT_TRAV_LANE",
    "RT_TRAV_PACKET", "RT_TRAV_STATIC", "static_source", "static_compile", "accel_build", "tonemap_device", "RT_SCENE_COUNT", "RT_SCENE_RANDOM_10K",
    "RT_XF_NONE", "RT_XF_TRANSLATE", "RT_XF_YROTATE", "RT_XF_YROTATE_TRANSLATE", "RenderError", "load_image",
    "render_devices", "multi_row_map", "kernel_build",
]


class RenderError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {_abi.status_string(code)} ({code})")
        self.code = code


def _check(code: int, what: str) -> None:
    if code != _abi.RT_OK:
        raise RenderError(code, what)


def scene_name(index: int) -> str:
    n = _abi.host_lib().rt_scene_name(index)
    return n.decode() if n else ""


class World:
    """Owns a reference-layout scene (records, refs, texture arena) built on the host.

    Mirrors `World` + the `add_*` builder API of raytracing.cu:1608-1612,1775-1977.  Each World has
    its own glibc-rand stream seeded with 1, like a fresh reference process.
    """

    def __init__(self, capacity: int = 8000, arena_bytes: int = 10 << 20):
        self._L = _abi.host_lib()
        self._w = self._L.rt_world_create(capacity, arena_bytes)
        if not self._w:
            raise MemoryError("rt_world_create failed")
        self.root: int | None = None

    def __del__(self):
        w = getattr(self, "_w", None)
        if w:
            self._L.rt_world_destroy(w)
            self._w = None

    # --- catalog (main.cu:52-117) ---
    def build_scene(self, index: int) -> Settings:
        s = Settings()
        _check(self._L.rt_world_build_scene(self._w, index, C.byref(s)), f"build scene {index}")
        return s

    # --- materials ---
    def lambert(self, rgb) -> _abi.Material:
        return self._L.rt_mat_lambert_solid(self._w, vec3(*rgb))

    def light(self, rgb) -> _abi.Material:
        return self._L.rt_mat_light_solid(self._w, vec3(*rgb))

    def noise(self, scale: float) -> _abi.Material:
        return self._L.rt_mat_lambert_noise(self._w, scale)

    def checker(self, scale: float, even, odd) -> _abi.Material:
        return self._L.rt_mat_lambert_checker(self._w, scale, vec3(*even), vec3(*odd))

    def image(self, name: str = "earthmap.jpg") -> _abi.Material:
        """Image texture from a file (stbi_loadf semantics, load_image); a missing or undecodable file
        renders magenta like the reference's failed load."""
        return self._L.rt_mat_lambert_image(self._w, name.encode())

    def status(self) -> int:
        return int(self._L.rt_world_status(self._w))

    def image_pixels(self, rgb) -> _abi.Material:
        """Image texture with texels (float32 [H, W, 3], like stbi_loadf) — copied into the arena."""
        a = np.ascontiguousarray(rgb, dtype=np.float32)
        self._keep = getattr(self, "_keep", []) + [a]
        return self._L.rt_mat_lambert_image_pixels(self._w, a.ctypes.data_as(C.c_void_p), a.shape[1], a.shape[0])

    def metal(self, rgb, fuzz: float) -> _abi.Material:
        return self._L.rt_mat_metal(vec3(*rgb), fuzz)

    def dielectric(self, ior: float) -> _abi.Material:
        return self._L.rt_mat_dielectric(ior)

    # --- primitives; xf = RT_XF_* transform ---
    def sphere(self, center, radius, mat, xf=RT_XF_NONE, angle=0.0, offset=(0, 0, 0)) -> int:
        return self._L.rt_add_sphere(self._w, xf, angle, vec3(*offset), vec3(*center), radius, mat)

    def moving_sphere(self, center, motion, radius, mat, xf=RT_XF_NONE, angle=0.0, offset=(0, 0, 0)) -> int:
        return self._L.rt_add_moving_sphere(self._w, xf, angle, vec3(*offset), vec3(*center),
                                            vec3(*motion), radius, mat)

    def quad(self, q, u, v, mat, xf=RT_XF_NONE, angle=0.0, offset=(0, 0, 0)) -> int:
        return self._L.rt_add_quad(self._w, xf, angle, vec3(*offset), vec3(*q), vec3(*u), vec3(*v), mat)

    def triangle(self, q, u, v, mat, xf=RT_XF_NONE, angle=0.0, offset=(0, 0, 0)) -> int:
        return self._L.rt_add_triangle(self._w, xf, angle, vec3(*offset), vec3(*q), vec3(*u), vec3(*v), mat)

    def box(self, a, b, mat, xf=RT_XF_NONE, angle=0.0, offset=(0, 0, 0)) -> int:
        return self._L.rt_add_box(self._w, xf, angle, vec3(*offset), vec3(*a), vec3(*b), mat)

    def pyramid(self, a, b, tip, mat, xf=RT_XF_NONE, angle=0.0, offset=(0, 0, 0)) -> int:
        return self._L.rt_add_pyramid(self._w, xf, angle, vec3(*offset), vec3(*a), vec3(*b), vec3(*tip), mat)

    def rand(self) -> int:
        return self._L.rt_world_rand(self._w)

    # --- BVH + export ---
    def build_bvh(self) -> int:
        root = C.c_uint16()
        _check(self._L.rt_world_build_bvh(self._w, C.byref(root)), "make_bvh")
        self.root = root.value
        return self.root

    def scene(self) -> Scene:
        if self.root is None:
            self.build_bvh()
        sc = Scene()
        _check(self._L.rt_world_scene(self._w, self.root, C.byref(sc)), "scene view")
        sc._owner = self   # keep the world alive while the view is used
        return sc

    def blobs(self) -> dict:
        """Copies of the scene bytes: records, refs, arena (fixtures, tests)."""
        sc = self.scene()
        rec = C.string_at(sc.hittables, sc.hittable_count * _abi.HITTABLE_BYTES)
        refs = np.ctypeslib.as_array(sc.refs, shape=(sc.ref_count,)).copy()
        tex = C.string_at(sc.textures, sc.texture_bytes) if sc.texture_bytes else b""
        return {"hittables": rec, "refs": refs, "textures": tex, "root": sc.root}

    def reference_stack_depth(self) -> int:
        sc = self.scene()
        d = C.c_uint32()
        _check(self._L.rt_reference_stack_depth(C.byref(sc), C.byref(d)), "stack depth")
        return d.value


class BlobScene:
    """A scene held as raw reference-layout bytes (e.g. loaded from tests/golden fixtures)."""

    def __init__(self, hittables: bytes, refs, textures: bytes, root: int):
        self._rec = C.create_string_buffer(bytes(hittables), len(hittables) or 1)
        self._refs = np.ascontiguousarray(np.asarray(refs, dtype=np.uint16))
        self._tex = C.create_string_buffer(bytes(textures), len(textures) or 1)
        self.count = len(hittables) // _abi.HITTABLE_BYTES
        self.ntex = len(textures)
        self.root = int(root)

    def scene(self) -> Scene:
        sc = Scene()
        sc.hittables = C.cast(self._rec, C.c_void_p)
        sc.hittable_count = self.count
        sc.refs = self._refs.ctypes.data_as(C.POINTER(C.c_uint16))
        sc.ref_count = len(self._refs)
        sc.root = self.root
        sc.textures = C.cast(self._tex, C.POINTER(C.c_uint8))
        sc.texture_bytes = self.ntex
        sc._owner = self
        return sc


def shard_rows(height: int, rank: int, world: int) -> tuple[int, int, int]:
    """Row-interleaved shard of `rank` in `world`: (row_offset, row_stride, row_count).

    Row r goes to GPU r mod G: interleaving balances the sky-heavy top rows against the
    expensive ground rows.  The RNG subsequence is the global pixel index, so any sharding reproduces
    the single-GPU image bit for bit."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad shard geometry")
    return rank, world, len(range(rank, height, world))


def unshard(shards: list, height: int, width: int) -> np.ndarray:
    """Inverse of shard_rows: list of [rows_k, W, 3] arrays (rank order) -> [H, W, 3]."""
    world = len(shards)
    img = np.empty((height, width, 3), dtype=np.float32)
    for r, sh in enumerate(shards):
        img[r::world] = sh
    return img


def build_scene(index: int, capacity: int | None = None):
    """Catalog scene -> (World, Settings) with the BVH built (the reference's main + make_bvh)."""
    if capacity is None:
        capacity = 24000 if index == RT_SCENE_RANDOM_10K else 8000
    w = World(capacity=capacity)
    s = w.build_scene(index)
    w.build_bvh()
    return w, s


def load_image(path: str):
    """rt_image_load: float32 [H, W, 3] texels as stbi_loadf(path, .., 3) returns them (row 0 = top; JPEG,
    PNG, BMP, TGA, GIF, PSD, Softimage PIC, PNM with 8-bit channels as powf(c/255, 2.2); Radiance HDR as
    stored), or None when the file does not exist or stb would fail to load it (the reference's failed load:
    a magenta texture)."""
    L = _abi.host_lib()
    p = C.POINTER(C.c_float)()
    w, h = C.c_int32(0), C.c_int32(0)
    rc = L.rt_image_load(str(path).encode(), C.byref(p), C.byref(w), C.byref(h))
    if rc == 1:   # RT_IMAGE_MISSING
        return None
    _check(rc, f"load image {path}")
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        L.rt_image_free(p)


def camera_from_settings(settings: Settings, width: int = 0, height: int = 0):
    """raytracing.cu:1657-1692.  width/height 0 => the reference's W and (int)(W/ratio)."""
    cam = Camera()
    W, H = C.c_int32(), C.c_int32()
    _check(_abi.host_lib().rt_camera_from_settings(C.byref(settings), width, height, C.byref(cam),
                                                   C.byref(W), C.byref(H)), "camera")
    return cam, W.value, H.value


def make_params(settings: Settings, width: int, height: int, spp: int | None = None,
                bounces: int | None = None, row_offset: int = 0, row_stride: int = 1,
                row_count: int | None = None, seed: int = 1234, flags: int = 0) -> Params:
    p = Params()
    p.width, p.height = width, height
    p.row_offset, p.row_stride = row_offset, row_stride
    p.row_count = row_count if row_count is not None else len(range(row_offset, height, row_stride))
    p.samples_per_pixel = settings.samples_per_pixel if spp is None else spp
    p.max_bounces = settings.max_bounces if bounces is None else bounces
    p.background = settings.background
    p.seed = seed
    p.flags = flags
    return p


def render(scene: Scene, camera: Camera, params: Params, with_stats: bool = False):
    """One-shot GPU render (rt_render): float32 array [row_count, width, 3], linear RGB."""
    out = np.zeros((params.row_count, params.width, 3), dtype=np.float32)
    st = Stats()
    _check(_abi.hip_lib().rt_render(C.byref(scene), C.byref(camera), C.byref(params),
                                    out.ctypes.data_as(C.c_void_p), C.byref(st)), "rt_render")
    return (out, st) if with_stats else out


def kernel_build(scene: Scene, traversal: int, max_bounces: int) -> dict:
    """rt_kernel_build: the render kernel a render of `scene` with `traversal` would build, compiled here by the run-time
    compiler (no device): VGPRs, SGPRs, scratch bytes, spill counts, the compiler and where its hipRTC came from."""
    k = _abi.KernelInfo()
    _check(_abi.hip_lib().rt_kernel_build(C.byref(scene), traversal, max_bounces, C.byref(k)), "rt_kernel_build")
    return k.as_dict()


def render_devices(scene: Scene, camera: Camera, params: Params, devices, rgb: bool = True, ppm: bool = True,
                   with_stats: bool = False):
    """One process, several devices (rt_render_devices): rows dealt round-robin over `devices`, one RCCL gather
    to devices[0], un-permuted there.  Returns (float32 [rows, W, 3] or None, uint8 [rows, W, 3] or None[, Stats])."""
    devs = (C.c_int * len(devices))(*devices)
    shape = (params.row_count, params.width, 3)
    f = np.zeros(shape, dtype=np.float32) if rgb else None
    b = np.zeros(shape, dtype=np.uint8) if ppm else None
    st = Stats()
    _check(_abi.hip_lib().rt_render_devices(C.byref(scene), C.byref(camera), C.byref(params), devs, len(devices),
                                            None if f is None else f.ctypes.data_as(C.c_void_p),
                                            None if b is None else b.ctypes.data_as(C.c_void_p), C.byref(st)),
           "rt_render_devices")
    return (f, b, st) if with_stats else (f, b)


def multi_row_map(row_count: int, n_devices: int, k: int):
    """rt_multi_row_map: (device, row in its shard, that shard's rows, longest shard) of frame row k."""
    o = [C.c_int32() for _ in range(4)]
    _check(_abi.hip_lib().rt_multi_row_map(row_count, n_devices, k, *(C.byref(x) for x in o)), "rt_multi_row_map")
    return tuple(x.value for x in o)


class RenderContext:
    """Device-resident scene (rt_context_*): render into caller device buffers on a HIP stream."""

    def __init__(self, scene: Scene, device: int = 0):
        self._L = _abi.hip_lib()
        h = C.c_void_p()
        _check(self._L.rt_context_create(C.byref(scene), device, C.byref(h)), "rt_context_create")
        self._h = h
        self._scene = scene

    def render_into(self, camera: Camera, params: Params, out_device_ptr: int, stream: int = 0,
                    out_ppm_device_ptr: int = 0) -> None:
        """Render into a device float buffer; with out_ppm_device_ptr also the P6 payload bytes, written
        by the render kernel as it finishes each pixel (rt_context_render_ppm)."""
        if out_ppm_device_ptr:
            _check(self._L.rt_context_render_ppm(self._h, C.byref(camera), C.byref(params), C.c_void_p(out_device_ptr),
                                                 C.c_void_p(out_ppm_device_ptr), C.c_void_p(stream)),
                   "rt_context_render_ppm")
            return
        _check(self._L.rt_context_render(self._h, C.byref(camera), C.byref(params),
                                         C.c_void_p(out_device_ptr), C.c_void_p(stream)), "rt_context_render")

    def timing(self) -> Stats:
        st = Stats()
        _check(self._L.rt_context_timing(self._h, C.byref(st)), "rt_context_timing")
        return st

    def note(self) -> str:
        """Why the last render did not use the scene-specialised traversal ("" if it did)."""
        n = self._L.rt_context_note(self._h)
        return n.decode() if n else ""

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.rt_context_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def static_source(scene: Scene, max_visits: int = 256) -> tuple[str, int]:
    """(hipRTC source of the scene-specialised traversal, node visits); RenderError over budget."""
    buf = C.create_string_buffer(1 << 22)
    v = C.c_uint32()
    _check(_abi.hip_lib().rt_static_source(C.byref(scene), max_visits, buf, len(buf), C.byref(v)),
           "rt_static_source")
    return buf.value.decode(), v.value


def accel_build(scene: Scene):
    """SAH tree of the verified sphere traversal (no device needed): (info dict, node words, prim words)
    as uint32 arrays, or None when the world is not an all-sphere BVH/group tree."""
    import numpy as np
    L = _abi.hip_lib()
    info = (C.c_uint32 * 4)()
    rc = L.rt_accel_build(C.byref(scene), None, 0, info)
    if rc == _abi.RT_ERR_UNSUPPORTED:
        return None
    _check(rc, "rt_accel_build")
    nw = info[3]
    total = nw + info[2] * 16
    buf = np.zeros(total, np.uint32)
    _check(L.rt_accel_build(C.byref(scene), buf.ctypes.data_as(C.c_void_p), total, info), "rt_accel_build")
    return {"root": info[0], "depth": info[1], "spheres": info[2]}, buf[:nw], buf[nw:]


def accel_build_wide(scene: Scene, quant: bool = False):
    """4-wide form of the verified walk's tree (no device needed): (info dict, node words as uint32), or None.
    quant: the quantised 64-B nodes (rt_accel_build_quant) instead of the float 128-B ones."""
    L = _abi.hip_lib()
    fn = L.rt_accel_build_quant if quant else L.rt_accel_build_wide
    info = (C.c_uint32 * 4)()
    rc = fn(C.byref(scene), None, 0, info)
    if rc == _abi.RT_ERR_UNSUPPORTED:
        return None
    _check(rc, fn.__name__)
    buf = np.zeros(info[3], np.uint32)
    _check(fn(C.byref(scene), buf.ctypes.data_as(C.c_void_p), len(buf), info), fn.__name__)
    return {"nodes": info[0], "depth": info[1], "stack": info[2]}, buf


def prim_lists(scene: Scene, camera: Camera, params: Params, cap: int = 128):
    """The verified sphere walk's primary-ray candidate lists of a frame, built on the host (no device needed):
    (counts [tiles] uint32 with 0xffffffff = no list, lists [tiles, cap, 2] uint32 {SAH prim index, axial bound
    bits}, rho), or None when the world is not eligible."""
    L = _abi.hip_lib()
    tiles = ((params.width + 7) // 8) * ((params.row_count + 7) // 8)
    counts = np.zeros(tiles, np.uint32)
    lists = np.zeros((tiles, cap, 2), np.uint32)
    rho = C.c_float()
    rc = L.rt_prim_lists(C.byref(scene), C.byref(camera), C.byref(params), cap, counts.ctypes.data_as(C.c_void_p),
                         lists.ctypes.data_as(C.c_void_p), C.byref(rho))
    if rc == _abi.RT_ERR_UNSUPPORTED:
        return None
    _check(rc, "rt_prim_lists")
    return counts, lists, rho.value


def mixed_build(scene: Scene):
    """Macro roots of the verified mixed-world traversal (no device needed): dict, or None when no
    transform-free subtree qualifies."""
    info = (C.c_uint32 * 4)()
    rc = _abi.hip_lib().rt_mixed_build(C.byref(scene), info)
    if rc == _abi.RT_ERR_UNSUPPORTED:
        return None
    _check(rc, "rt_mixed_build")
    return {"macros": info[0], "dynamic": info[1], "prims": info[2], "depth": info[3]}


def static_compile(scene: Scene, arch: str = "gfx950", max_visits: int = 256) -> str:
    """Compile the scene-specialised kernels with hipRTC (no device needed); returns the log."""
    log = C.create_string_buffer(1 << 16)
    rc = _abi.hip_lib().rt_static_compile(C.byref(scene), max_visits, arch.encode(), log, len(log))
    if rc != 0:
        raise RenderError(rc, "rt_static_compile: " + log.value.decode(errors="replace")[:4000])
    return log.value.decode(errors="replace")


def seed_states(seed: int, width: int, row_offset: int, row_stride: int, rows: int) -> np.ndarray:
    """Device-seeded per-pixel XORWOW states [6, rows*width] (d, x0..x4) — rt_seed_states."""
    out = np.empty((6, rows * width), dtype=np.uint32)
    _check(_abi.hip_lib().rt_seed_states(seed, width, row_offset, row_stride, rows, out.ctypes.data_as(C.c_void_p)),
           "rt_seed_states")
    return out


def tonemap(rgb: np.ndarray) -> np.ndarray:
    """raytracing.cu:1391-1395,1419-1433: sqrt gamma, clamp [0,0.999], x256 -> u8."""
    src = np.ascontiguousarray(rgb, dtype=np.float32)
    out = np.empty(src.shape, dtype=np.uint8)
    _abi.host_lib().rt_tonemap(src.ctypes.data_as(C.c_void_p), src.size // 3, out.ctypes.data_as(C.c_void_p))
    return out


def tonemap_device(rgb, out=None, stream: int = 0):
    """GPU tonemap (rt_tonemap_device) of a float32 CUDA tensor [..., 3] -> uint8 tensor, same shape."""
    import torch
    if not (rgb.is_cuda and rgb.dtype == torch.float32 and rgb.is_contiguous()):
        raise ValueError("tonemap_device expects a contiguous float32 device tensor")
    if out is None:
        out = torch.empty(rgb.shape, dtype=torch.uint8, device=rgb.device)
    _check(_abi.hip_lib().rt_tonemap_device(C.c_void_p(rgb.data_ptr()), rgb.numel() // 3,
                                            C.c_void_p(out.data_ptr()), C.c_void_p(stream)), "rt_tonemap_device")
    return out


def write_ppm(path: str, rgb: np.ndarray) -> None:
    src = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = src.shape[:2]
    _check(_abi.host_lib().rt_write_ppm(path.encode(), src.ctypes.data_as(C.c_void_p), w, h), "write_ppm")
