"""Regenerate tests/golden/images: small image files of every decoded format plus the SHA-256 of the
float texels the reference's own loader (stb_image v2.30's stbi_loadf(file, .., 3), compiled from
/root/reference into oracle/_ref by `make ref`) returns for them, or null where it fails.
Run from the repo root in the container that has /root/reference:  python tools/gen_image_golden.py
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import image_corpus as corpus  # noqa: E402
from test_image_load import stbi_loadf  # noqa: E402

PICKS = ["ss2_q75.jpg", "ss0_q100.jpg", "progressive_420.jpg", "restart.jpg", "cmyk.jpg", "grey_progressive.jpg",
         "rgb16_adam7.png", "pal4_flat.png", "grey2_adam7.png", "ga16_flat.png", "rgb8_fixed.png", "rgb8_stored.png",
         "rgb565_bitfields.bmp", "pal4.bmp", "os2_24.bmp", "pal1_topdown.bmp", "v5_32.bmp", "pil_P_tga_rle.tga", "cmap16.tga",
         "rgb15_topdown_id.tga", "rle.hdr", "flat_wide.hdr", "g_local_interlaced.gif", "g_transparent_bg.gif",
         "g_clears.gif", "p_rgba_rle.psd", "p_rgb16.psd", "mixed.pic", "split_channels.pic"]


def main():
    out = ROOT / "tests" / "golden" / "images"
    out.mkdir(parents=True, exist_ok=True)
    files = corpus.corpus(4, 11, 19)
    chosen = {name: files[name] for name in PICKS}
    jpg = files["ss1_q75.jpg"]
    for frac in (0.66, 0.7, 0.75, 0.8, 0.85, 0.9):               # decodes: zero bits after the data
        t = out / "truncated.jpg"
        t.write_bytes(jpg[: int(len(jpg) * frac)])
        z = stbi_loadf(t, "_zero")
        if z is not None and np.array_equal(z, stbi_loadf(t, "_pattern")):
            chosen["truncated.jpg"] = t.read_bytes()
            break
    png = bytearray(files["rgb8_flat.png"])
    png[60] ^= 0x55                                               # corrupt DEFLATE data: a failed load
    chosen["corrupt.png"] = bytes(png)
    manifest = {}
    for name, data in chosen.items():
        f = out / name
        f.write_bytes(data)
        ref = stbi_loadf(f)
        if not (ref is None) == (stbi_loadf(f, "_zero") is None) or (
                ref is not None and not np.array_equal(stbi_loadf(f, "_zero"), stbi_loadf(f, "_pattern"))):
            raise SystemExit(f"{name}: the reference's output depends on uninitialised memory; pick another")
        manifest[name] = None if ref is None else {
            "shape": list(ref.shape), "sha256": hashlib.sha256(np.ascontiguousarray(ref, np.float32).tobytes()).hexdigest()}
    (out / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True) + "\n")
    print(f"{len(manifest)} fixtures, {sum(len(v) for v in chosen.values())} bytes")


if __name__ == "__main__":
    main()
