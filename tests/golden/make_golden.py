"""Regenerate tests/golden/{scenes.npz,frames.npz,manifest.json}.

Run from the repo root after `make host oracle`:  python tests/golden/make_golden.py

What the fixtures are:
  * scenes.npz  — reference-layout scene bytes (Hittable records, u16 refs, texture arena, root) that
                  the host builder produces for the catalog scenes used in parity tests.  The 10k scene
                  is stored by SHA-256 only (2.6 MB).
  * frames.npz  — float32 framebuffers rendered by the CPU oracle (oracle/oracle_rt.c) from those bytes
                  at small sizes, plus the tonemapped 8-bit P6 bytes.
  * manifest.json — per case: scene, resolution, spp, bounces, camera, SHA-256 of every array.

Provenance / pinning: the reference (CUDA + cuRAND) cannot be built here, so these
frames pin the oracle and the HIP kernel to each other and to themselves over time; the oracle's own
dependencies are pinned separately (rng_kat.json from rocRAND, glibc rand from libc).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
import cuda_raytracing_amd as rt  # noqa: E402
from cuda_raytracing_amd import _abi  # noqa: E402

OUT = Path(__file__).resolve().parent

# (name, scene, W, H, spp, bounces)
CASES = [
    ("scene0_cfg1", 0, 256, 144, 4, 4),        # BASELINE config 1 exactly (./raytracing 0 s4 b4 at 256x144)
    ("scene0_96x54_s16_b16", 0, 96, 54, 16, 16),
    ("scene1_cornell_48x48_s16_b50", 1, 48, 48, 16, 50),
    ("scene17_perlin_96x54_s16_b50", 17, 96, 54, 16, 50),
    ("scene2_bouncing_64x36_s8_b16", 2, 64, 36, 8, 16),
    ("scene20_random10k_64x36_s4_b16", 20, 64, 36, 4, 16),
    ("scene8_refract1_48x27_s8_b16", 8, 48, 27, 8, 16),
    ("scene12_refract5_48x27_s8_b16", 12, 48, 27, 8, 16),
    ("scene13_motion_blur_48x27_s8_b16", 13, 48, 27, 8, 16),
    ("scene14_light_test_48x27_s8_b16", 14, 48, 27, 8, 16),
    ("scene15_checkered_48x27_s8_b16", 15, 48, 27, 8, 16),
    ("scene19_simple_light_48x27_s8_b50", 19, 48, 27, 8, 50),
]
STORE_BLOB = {0, 1, 17, 2, 8, 12, 13, 14, 15, 19}


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def oracle_render(sc, cam, p):
    out = np.zeros((p.row_count, p.width, 3), np.float32)
    st = _abi.Stats()
    rc = _abi.oracle_lib().rt_render_cpu(C.byref(sc), C.byref(cam), C.byref(p),
                                         out.ctypes.data_as(C.c_void_p), C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle failed: {rc}")
    return out, st


def main():
    scenes, frames, manifest = {}, {}, {"cases": [], "scenes": {}}
    for name, idx, W, H, spp, b in CASES:
        w, s = rt.build_scene(idx)
        blobs = w.blobs()
        key = f"s{idx}"
        if key not in manifest["scenes"]:
            manifest["scenes"][key] = {
                "index": idx, "name": rt.scene_name(idx), "root": int(blobs["root"]),
                "hittable_count": len(blobs["hittables"]) // 120, "ref_count": int(len(blobs["refs"])),
                "texture_bytes": len(blobs["textures"]),
                "sha256_hittables": sha(blobs["hittables"]), "sha256_refs": sha(blobs["refs"].tobytes()),
                "sha256_textures": sha(blobs["textures"]),
                "reference_stack_depth": w.reference_stack_depth(),
                "settings": {"img_ratio": s.img_ratio, "img_width": s.img_width, "spp": s.samples_per_pixel,
                             "max_bounces": s.max_bounces, "vfov": s.vfov, "defocus_angle": s.defocus_angle,
                             "background": s.background.tolist(), "img_name": s.img_name.decode()},
            }
            if idx in STORE_BLOB:
                scenes[f"{key}_hittables"] = np.frombuffer(blobs["hittables"], np.uint8)
                scenes[f"{key}_refs"] = blobs["refs"]
                scenes[f"{key}_textures"] = np.frombuffer(blobs["textures"], np.uint8)
                scenes[f"{key}_root"] = np.array([blobs["root"]], np.uint16)
        cam, W2, H2 = rt.camera_from_settings(s, W, H)
        p = rt.make_params(s, W2, H2, spp=spp, bounces=b)
        fb, st = oracle_render(w.scene(), cam, p)
        frames[f"{name}_fb"] = fb
        frames[f"{name}_u8"] = rt.tonemap(fb)
        cam_d = {f: [getattr(cam, f).x, getattr(cam, f).y, getattr(cam, f).z]
                 for f in ("pixel00", "delta_u", "delta_v", "center", "defocus_u", "defocus_v")}
        cam_d["defocus_angle"] = cam.defocus_angle
        manifest["cases"].append({
            "name": name, "scene": idx, "width": W2, "height": H2, "spp": spp, "bounces": b,
            "camera": cam_d, "sha256_fb": sha(fb.tobytes()), "counters": st.counter_dict(),
        })
        print(name, "ok", st.counter_dict()["samples"], flush=True)
    np.savez_compressed(OUT / "scenes.npz", **scenes)
    np.savez_compressed(OUT / "frames.npz", **frames)
    (OUT / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
