"""Image files for image textures (make_image_texture's stbi_loadf, raytracing.cu:332-341), no GPU needed.

rt_image_load decodes binary PNM (P5/P6), BMP (24/32 bit BI_RGB) and TGA (uncompressed 8/24/32 bit) the
way stbi_loadf(file, .., 3) returns them: float RGB, row 0 = top of the picture, grey replicated, alpha
dropped, 8-bit channels as powf(c / 255.0f, 2.2f) (stb_image's LDR->float rule).  Expected texels are
built here from the same picture the file encodes.  The rule's powf is checked against the correctly
rounded pow of the same float operands (tolerance: 0 ulp).
"""
from __future__ import annotations

import ctypes as C
import struct
from pathlib import Path

import numpy as np
import pytest

import cuda_raytracing_amd as rt
from cuda_raytracing_amd import _abi


REF_STBI = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "libstbi_ref.so"


def stbi_loadf(path):
    """The reference's own loader (stb_image v2.30 compiled where it lies, oracle/stbi_ref.cpp)."""
    L = C.CDLL(str(REF_STBI))
    L.rt_ref_stbi_loadf.restype = C.POINTER(C.c_float)
    L.rt_ref_stbi_loadf.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.rt_ref_stbi_free.argtypes = [C.c_void_p]
    w, h = C.c_int(0), C.c_int(0)
    p = L.rt_ref_stbi_loadf(str(path).encode(), C.byref(w), C.byref(h))
    if not p:
        return None
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        L.rt_ref_stbi_free(p)


def check_vs_stb(path, got):
    """Pinned against the reference's stb_image when oracle/_ref is built (make ref, needs /root/reference)."""
    if not REF_STBI.exists():
        return
    ref = stbi_loadf(path)
    assert (ref is None) == (got is None)
    if ref is not None:
        assert ref.shape == got.shape and np.array_equal(ref.view(np.uint32), got.view(np.uint32))


def ldr_to_float(px: np.ndarray) -> np.ndarray:
    # (float) powf(c / 255.0f, 2.2f): the float quotient, then the correctly rounded float power
    q = px.astype(np.float32) / np.float32(255.0)
    return np.power(q.astype(np.float64), np.float64(np.float32(2.2))).astype(np.float32)


@pytest.fixture(scope="module")
def picture():
    rng = np.random.default_rng(7)
    return rng.integers(0, 256, size=(5, 7, 3), dtype=np.uint8)   # rows top first


def expect(pic):
    if pic.ndim == 2:
        pic = np.repeat(pic[:, :, None], 3, axis=2)
    return ldr_to_float(pic[:, :, :3])


def test_every_byte_value_converts_like_stb(tmp_path):
    pic = np.arange(256, dtype=np.uint8).reshape(16, 16)
    f = tmp_path / "ramp.pgm"
    f.write_bytes(b"P5\n16 16\n255\n" + pic.tobytes())
    got = rt.load_image(f)
    check_vs_stb(f, got)
    assert got.shape == (16, 16, 3) and got.dtype == np.float32
    assert np.array_equal(got.view(np.uint32), expect(pic).view(np.uint32))
    assert got[0, 0, 0] == 0.0 and got[-1, -1, 0] == 1.0


def test_ppm_p6_with_comments(tmp_path, picture):
    f = tmp_path / "a.ppm"
    f.write_bytes(b"P6\n# a comment\n7 5\n# another\n255\n" + picture.tobytes())
    got = rt.load_image(f)
    check_vs_stb(f, got)
    assert np.array_equal(got.view(np.uint32), expect(picture).view(np.uint32))


@pytest.mark.parametrize("maxval", [0, 100, 256, 65535])
def test_pnm_samples_are_taken_as_stored(tmp_path, picture, maxval):
    # stb does not rescale by maxval; 16-bit samples (maxval > 255) come out as their second byte
    if maxval > 255:
        hi = np.random.default_rng(3).integers(0, 256, size=picture.shape, dtype=np.uint8)
        body = np.stack([hi, picture], axis=-1).tobytes()
    else:
        body = picture.tobytes()
    f = tmp_path / "a.ppm"
    f.write_bytes(b"P6\n7 5\n%d\n" % maxval + body)
    got = rt.load_image(f)
    check_vs_stb(f, got)
    assert np.array_equal(got.view(np.uint32), expect(picture).view(np.uint32))


def bmp_bytes(pic: np.ndarray, bpp: int, top_down: bool) -> bytes:
    h, w, _ = pic.shape
    bypp = bpp // 8
    stride = (w * bypp + 3) & ~3
    rows = []
    order = range(h) if top_down else range(h - 1, -1, -1)
    for y in order:
        row = bytearray()
        for x in range(w):
            r, g, b = (int(v) for v in pic[y, x])
            row += bytes([b, g, r] + ([0xAB] if bypp == 4 else []))
        row += b"\0" * (stride - len(row))
        rows.append(bytes(row))
    data = b"".join(rows)
    header = struct.pack("<2sIHHI", b"BM", 54 + len(data), 0, 0, 54)
    info = struct.pack("<IiiHHIIiiII", 40, w, -h if top_down else h, 1, bpp, 0, len(data), 2835, 2835, 0, 0)
    return header + info + data


@pytest.mark.parametrize("bpp,top_down", [(24, False), (32, True), (24, True)])
def test_bmp(tmp_path, picture, bpp, top_down):
    f = tmp_path / "a.bmp"
    f.write_bytes(bmp_bytes(picture, bpp, top_down))
    got = rt.load_image(f)
    check_vs_stb(f, got)
    assert np.array_equal(got.view(np.uint32), expect(picture).view(np.uint32))


@pytest.mark.parametrize("grey,top_first", [(False, False), (False, True), (True, False)])
def test_tga(tmp_path, picture, grey, top_first):
    h, w, _ = picture.shape
    pic = picture[:, :, 0] if grey else picture
    hdr = struct.pack("<BBBHHBHHHHBB", 0, 0, 3 if grey else 2, 0, 0, 0, 0, 0, w, h, 8 if grey else 24,
                      0x20 if top_first else 0)
    rows = [pic[y] for y in (range(h) if top_first else range(h - 1, -1, -1))]
    body = b"".join(r.tobytes() if grey else r[:, ::-1].tobytes() for r in rows)   # BGR
    f = tmp_path / "a.tga"
    f.write_bytes(hdr + body)
    got = rt.load_image(f)
    check_vs_stb(f, got)
    assert np.array_equal(got.view(np.uint32), expect(pic).view(np.uint32))


def test_missing_file_is_the_reference_failed_load(tmp_path):
    assert rt.load_image(tmp_path / "earthmap.jpg") is None
    check_vs_stb(tmp_path / "earthmap.jpg", None)
    w = rt.World()
    m = w.image(str(tmp_path / "earthmap.jpg"))
    assert w.status() == 0 and m.kind == 0


@pytest.mark.parametrize("payload", [b"\xff\xd8\xff\xe0\x00\x10JFIF\x00", b"\x89PNG\r\n\x1a\n\x00\x00", b"P3\n1 1\n255\n0 0 0\n",
                                     b"P6\n1 1\n65536\n\0\0\0\0\0\0", b"P6\n2 1\n255\n\0\0\0"])
def test_other_formats_are_unsupported(tmp_path, payload):
    f = tmp_path / "earthmap.jpg"
    f.write_bytes(payload)
    with pytest.raises(rt.RenderError) as e:
        rt.load_image(f)
    assert e.value.code == -6
    w = rt.World()
    w.image(str(f))
    assert w.status() == -6


def test_earth_scene_loads_its_texture(tmp_path, monkeypatch, picture):
    # the catalog's earth scene (raytracing.cu:2042-2052) names earthmap.jpg relative to the working
    # directory: absent -> magenta texture (the reference's run), a JPEG -> unsupported, and the texels
    # of a decodable file end up in the texture arena behind the image Texture record (:270-279)
    monkeypatch.chdir(tmp_path)
    idx = [rt.scene_name(i) for i in range(rt.RT_SCENE_COUNT)].index("earth")
    w = rt.World()
    w.build_scene(idx)
    assert w.status() == 0
    (tmp_path / "earthmap.jpg").write_bytes(b"\xff\xd8\xff\xe0")
    with pytest.raises(rt.RenderError):
        rt.World().build_scene(idx)
    (tmp_path / "earthmap.jpg").write_bytes(b"P6 7 5 255\n" + picture.tobytes())
    w2 = rt.World()
    w2.build_scene(idx)
    sc = w2.scene()
    arena = np.frombuffer(C.string_at(sc.textures, sc.texture_bytes), np.uint8)
    want = expect(picture).tobytes()
    assert arena.tobytes().find(want) > 0


@pytest.mark.skipif(not REF_STBI.exists(), reason="oracle/_ref not built (needs /root/reference)")
def test_reference_loader_is_pinned_on_random_images(tmp_path):
    # random sizes and pixels through every decoded format, against stbi_loadf itself
    rng = np.random.default_rng(11)
    for case in range(12):
        h, w = (int(x) for x in rng.integers(1, 40, size=2))
        pic = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        files = {
            "a.ppm": b"P6 %d %d 255\n" % (w, h) + pic.tobytes(),
            "a.pgm": b"P5\n%d %d\n255\n" % (w, h) + pic[:, :, 1].tobytes(),
            "a.bmp": bmp_bytes(pic, 24 if case % 2 else 32, bool(case % 3 == 0)),
        }
        for name, data in files.items():
            f = tmp_path / f"{case}_{name}"
            f.write_bytes(data)
            got = rt.load_image(f)
            ref = stbi_loadf(f)
            assert ref is not None and np.array_equal(ref.view(np.uint32), got.view(np.uint32)), f
