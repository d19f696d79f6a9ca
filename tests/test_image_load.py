"""Image files for image textures (make_image_texture's stbi_loadf, raytracing.cu:332-341), no GPU needed.

rt_image_load returns what stbi_loadf(file, .., 3) (stb_image v2.30, vendored by the reference) returns:
float RGB, row 0 = top of the picture, grey replicated, alpha dropped, 8-bit channels as
powf(c / 255.0f, 2.2f), Radiance HDR as stored; a missing, unknown or corrupt file is the reference's failed
load (None: a magenta texture).  Tolerance everywhere: 0 ulp.

Pinning: the reference's own loader is compiled from /root/reference into oracle/_ref (make ref) as-is and
twice with its uninitialised memory made explicit (zeros / a pattern: oracle/stbi_ref.cpp).  Every file of
tests/image_corpus.py (JPEG baseline / progressive / restart / grey / CMYK, PNG of every colour type and bit
depth, Adam7, all filters and DEFLATE block types, BMP 1-32 bit with bit fields and V4 / V5 / OS/2 headers,
TGA raw / RLE / colour-mapped / 16-bit, HDR flat / RLE, GIF global / local / interlaced / transparent / with
table clears, PSD raw / RLE at 8 and 16 bits with 1-5 channels, Softimage PIC raw / pure / mixed RLE packets) and thousands of truncated or corrupted copies must
decode to the same bits as the zero build, and as the as-is build wherever the two explicit builds agree.
Without /root/reference (the GPU box) the committed fixtures under tests/golden/images pin the same path:
files plus the SHA-256 of the reference loader's output (tools/gen_image_golden.py).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import struct
from pathlib import Path

import numpy as np
import pytest

import cuda_raytracing_amd as rt
from cuda_raytracing_amd import _abi


import image_corpus as corpus

REF_DIR = Path(__file__).resolve().parents[1] / "oracle" / "_ref"
REF_STBI = REF_DIR / "libstbi_ref.so"
GOLDEN = Path(__file__).resolve().parent / "golden" / "images"
_LIBS: dict = {}
needs_ref = pytest.mark.skipif(not REF_STBI.exists(), reason="oracle/_ref not built (needs /root/reference)")


def _ref_lib(variant: str):
    if variant not in _LIBS:
        L = C.CDLL(str(REF_DIR / f"libstbi_ref{variant}.so"))
        L.rt_ref_stbi_loadf.restype = C.POINTER(C.c_float)
        L.rt_ref_stbi_loadf.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.rt_ref_stbi_free.argtypes = [C.c_void_p]
        _LIBS[variant] = L
    return _LIBS[variant]


def stbi_loadf(path, variant: str = ""):
    """The reference's own loader (stb_image v2.30 compiled where it lies, oracle/stbi_ref.cpp); variant
    "_zero" / "_pattern": the builds with uninitialised memory set to zeros / a pattern."""
    L = _ref_lib(variant)
    w, h = C.c_int(0), C.c_int(0)
    p = L.rt_ref_stbi_loadf(str(path).encode(), C.byref(w), C.byref(h))
    if not p:
        return None
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        L.rt_ref_stbi_free(p)


def load_or_code(path):
    """rt_image_load through the package: texels, None (failed load) or the error code."""
    try:
        return rt.load_image(path)
    except rt.RenderError as e:
        return e.code


def same(a, b) -> bool:
    if a is None or b is None or isinstance(a, int) or isinstance(b, int):
        return (a is None and b is None) or (isinstance(a, int) and a is b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def agrees_with_reference(path) -> tuple[bool, bool]:
    """(rt_image_load == the reference loader, the reference's output depends on memory it never wrote).
    A zero-area image, which stb returns for some corrupt headers, is a failed load here (image_load.cpp), and so
    is a corrupt PIC file on which stb faults (the checker reports the fault as a failed load: oracle/stbi_ref.cpp)."""
    got = load_or_code(path)
    zero, pattern, asis = (stbi_loadf(path, v) for v in ("_zero", "_pattern", ""))
    if zero is not None and zero.size == 0:
        zero = pattern = asis = None
    uninit = not same(zero, pattern)
    return same(got, zero) and (uninit or same(got, asis)), uninit


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
                                     b"P6\n1 1\n65536\n\0\0\0\0\0\0", b"", b"hello world", b"BM\0\0"])
def test_corrupt_and_unknown_files_are_the_reference_failed_load(tmp_path, payload):
    # stbi_loadf returns NULL: the texture renders magenta, the world stays valid
    f = tmp_path / "earthmap.jpg"
    f.write_bytes(payload)
    assert rt.load_image(f) is None
    check_vs_stb(f, None)
    w = rt.World()
    m = w.image(str(f))
    assert w.status() == 0 and m.kind == 0


@pytest.mark.parametrize("payload", [b"GIF89a\x01\x00\x01\x00\x00\x00\x00;", b"8BPS\x00\x01" + b"\0" * 30,
                                     b"\x53\x80\xF6\x34" + b"\0" * 84 + b"PICT" + b"\0" * 16])
def test_gif_psd_pic_headers_without_a_picture_are_failed_loads(tmp_path, payload):
    # a GIF with no colour table and no image, a PSD of version 0, a PIC of zero area: stb fails (or returns a
    # zero-area image, which this build treats as a failed load) — a magenta texture, the world stays valid
    f = tmp_path / "earthmap.jpg"
    f.write_bytes(payload)
    assert rt.load_image(f) is None
    w = rt.World()
    m = w.image(str(f))
    assert w.status() == 0 and m.kind == 0


def _rgb_float(rgb8: np.ndarray) -> np.ndarray:
    return ldr_to_float(rgb8)


def test_gif_decodes_the_picture_it_encodes(tmp_path):
    # independent of stb: palette entries of the raster's indices, interlaced or not, global or local table,
    # with table clears, and the image at an offset of a larger screen (texels outside it: black, or the
    # background entry's bytes in stored order when its index is not 0)
    rng = np.random.default_rng(4)
    idx = rng.integers(0, 256, size=(11, 19), dtype=np.uint8)
    pal = rng.integers(0, 256, size=(256, 3), dtype=np.uint8)
    for kw in ({}, {"interlace": True}, {"local": True, "interlace": True}, {"clear_every": 5}):
        f = tmp_path / "a.gif"
        f.write_bytes(corpus.gif_bytes(idx, pal, **kw))
        got = rt.load_image(f)
        check_vs_stb(f, got)
        assert np.array_equal(got.view(np.uint32), _rgb_float(pal[idx]).view(np.uint32)), kw
    f = tmp_path / "b.gif"
    f.write_bytes(corpus.gif_bytes(idx & 7, pal, bits=3, screen=(22, 13), offset=(2, 1), bgindex=5))
    got = rt.load_image(f)
    check_vs_stb(f, got)
    want = np.empty((13, 22, 3), np.uint8)
    want[:] = pal[5][::-1]                       # the background entry as stb copies it: blue, green, red
    want[1:12, 2:21] = pal[idx & 7]
    assert np.array_equal(got.view(np.uint32), _rgb_float(want).view(np.uint32))
    f.write_bytes(corpus.gif_bytes(idx & 7, pal, bits=3, transparent=2))
    got = rt.load_image(f)
    check_vs_stb(f, got)
    want = pal[idx & 7].copy()
    want[(idx & 7) == 2] = 0                     # transparent texels are not written
    assert np.array_equal(got.view(np.uint32), _rgb_float(want).view(np.uint32))


def test_psd_and_pic_decode_the_picture_they_encode(tmp_path):
    # independent of stb: planar RGB (raw / PackBits, 8 / 16 bits), PIC raw and RLE packets; PSD alpha below 255
    # removes the white matte in float arithmetic (c / a + 255 (1 - 1 / a), truncated)
    pic = corpus.picture(9, 14, seed=6, smooth=False)
    planes = np.moveaxis(pic, 2, 0)
    cases = {"a.psd": corpus.psd_bytes(planes), "b.psd": corpus.psd_bytes(planes, rle=True),
             "c.psd": corpus.psd_bytes(planes.astype(np.uint16) * 256 + 255, depth=16),
             "d.pic": corpus.pic_bytes(np.concatenate([pic, pic[:, :, :1]], 2), [(0xE0, 0)]),
             "e.pic": corpus.pic_bytes(np.concatenate([pic, pic[:, :, :1]], 2), [(0x80, 1), (0x60, 2)])}
    for name, data in cases.items():
        f = tmp_path / name
        f.write_bytes(data)
        got = rt.load_image(f)
        check_vs_stb(f, got)
        assert np.array_equal(got.view(np.uint32), _rgb_float(pic).view(np.uint32)), name
    a = np.full((1, 9, 14), 128, np.uint8)
    f = tmp_path / "f.psd"
    f.write_bytes(corpus.psd_bytes(np.concatenate([planes, a])))
    got = rt.load_image(f)
    check_vs_stb(f, got)
    ra = np.float32(1) / (np.float32(128) / np.float32(255))
    v = (pic.astype(np.float32) * ra + np.float32(255) * (np.float32(1) - ra)).astype(np.int32).astype(np.uint8)
    assert np.array_equal(got.view(np.uint32), _rgb_float(v).view(np.uint32))
    f = tmp_path / "g.pic"
    f.write_bytes(corpus.pic_bytes(np.concatenate([pic, pic[:, :, :1]], 2), [(0x40, 0)]))   # green only: others 255
    want = np.full_like(pic, 255)
    want[:, :, 1] = pic[:, :, 1]
    got = rt.load_image(f)
    check_vs_stb(f, got)
    assert np.array_equal(got.view(np.uint32), _rgb_float(want).view(np.uint32))


def test_earth_scene_loads_its_texture(tmp_path, monkeypatch, picture):
    # the catalog's earth scene (raytracing.cu:2042-2052) names earthmap.jpg relative to the working
    # directory: absent or corrupt -> magenta texture (the reference's run), and the texels of a
    # decodable file (a real JPEG here) end up in the texture arena behind the image Texture record
    # (:270-279)
    monkeypatch.chdir(tmp_path)
    idx = [rt.scene_name(i) for i in range(rt.RT_SCENE_COUNT)].index("earth")
    w = rt.World()
    w.build_scene(idx)
    assert w.status() == 0
    (tmp_path / "earthmap.jpg").write_bytes(b"\xff\xd8\xff\xe0")
    w1 = rt.World()
    w1.build_scene(idx)
    assert w1.status() == 0
    pic = corpus.picture(64, 128, seed=3)
    (tmp_path / "earthmap.jpg").write_bytes(corpus.pil_bytes(pic, "JPEG", quality=90))
    texels = rt.load_image(tmp_path / "earthmap.jpg")
    check_vs_stb(tmp_path / "earthmap.jpg", texels)
    assert texels.shape == (64, 128, 3)
    w2 = rt.World()
    w2.build_scene(idx)
    sc = w2.scene()
    arena = np.frombuffer(C.string_at(sc.textures, sc.texture_bytes), np.uint8)
    assert arena.tobytes().find(texels.tobytes()) > 0


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


# ---------------------------------------------------------------- every format stb reads

CORPUS_SIZES = [(1, 1), (2, 3), (8, 8), (16, 17), (37, 53), (3, 200), (70, 9)]


@needs_ref
@pytest.mark.parametrize("size", CORPUS_SIZES, ids=lambda s: f"{s[0]}x{s[1]}")
def test_corpus_matches_the_reference_loader(tmp_path, size):
    files = corpus.corpus(CORPUS_SIZES.index(size), *size)
    assert len(files) >= 90
    bad = []
    for name, data in files.items():
        f = tmp_path / name
        f.write_bytes(data)
        ok, _ = agrees_with_reference(f)
        if not ok:
            bad.append(name)
    assert not bad, bad


@needs_ref
@pytest.mark.parametrize("seed", [1, 2])
def test_truncated_and_corrupted_files_match_the_reference_loader(tmp_path, seed):
    # truncations, random byte stores, bit flips in the headers and random runs, over the whole corpus:
    # success / failure and every texel as the reference loader (its zero build where it reads memory
    # it never wrote — rt_image_load reads zeros there)
    rng = np.random.default_rng(seed)
    files = corpus.corpus(seed, int(rng.integers(1, 40)), int(rng.integers(1, 60)))
    bad, n, uninit = [], 0, 0
    for name, data in files.items():
        for trial in range(8):
            d = bytearray(data)
            kind = trial % 4
            if kind == 0:
                d = d[:int(rng.integers(0, len(d)))]
            elif kind == 1:
                for _ in range(int(rng.integers(1, 4))):
                    d[int(rng.integers(0, len(d)))] = int(rng.integers(0, 256))
            elif kind == 2:
                d[int(rng.integers(0, min(len(d), 300)))] ^= 1 << int(rng.integers(0, 8))
            else:
                i = int(rng.integers(0, len(d)))
                j = min(len(d), i + int(rng.integers(1, 64)))
                d[i:j] = rng.integers(0, 256, j - i, dtype=np.uint8).tobytes()
            f = tmp_path / ("x." + name.rsplit(".", 1)[1])
            f.write_bytes(bytes(d))
            ok, u = agrees_with_reference(f)
            n += 1
            uninit += u
            if not ok:
                bad.append((name, trial))
    assert n >= 800 and not bad, bad


def test_hdr_texels_are_the_stored_rgbe_values(tmp_path):
    # independent of stb: mantissa * 2^(exponent - 136), a zero exponent is black; flat and RLE scanlines
    for seed, rle, (h, w) in [(0, False, (6, 5)), (1, True, (9, 40)), (2, True, (3, 9))]:
        rgbe = corpus._rgbe(h, w, seed)
        f = tmp_path / f"{seed}.hdr"
        f.write_bytes(corpus.hdr_bytes(rgbe, rle))
        got = rt.load_image(f)
        check_vs_stb(f, got)
        want = corpus.hdr_expected(rgbe)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        assert got[0, 0].tolist() == [0.0, 0.0, 0.0]


def test_png_and_bmp_decode_the_picture_they_encode(tmp_path):
    # independent of stb: lossless formats give back the picture they were written from
    pic = corpus.picture(13, 21, seed=9, smooth=False)
    cases = {"a.png": corpus.png_bytes(pic, 2, 8, interlace=True), "b.png": corpus.png_bytes(pic, 2, 8, level=0),
             "c.bmp": corpus.bmp_variants(pic)["v5_24.bmp"], "d.bmp": corpus.bmp_variants(pic)["os2_24.bmp"]}
    for name, data in cases.items():
        f = tmp_path / name
        f.write_bytes(data)
        got = rt.load_image(f)
        assert np.array_equal(got.view(np.uint32), expect(pic).view(np.uint32)), name


def test_golden_fixtures(tmp_path):
    # committed files + the SHA-256 of the reference loader's float texels (tools/gen_image_golden.py):
    # pins the decoders where /root/reference is absent (the GPU box)
    manifest = json.loads((GOLDEN / "manifest.json").read_text())
    assert len(manifest) >= 12
    for name, want in manifest.items():
        got = rt.load_image(GOLDEN / name)
        if want is None:
            assert got is None, name
            continue
        assert list(got.shape) == want["shape"], name
        assert hashlib.sha256(np.ascontiguousarray(got, np.float32).tobytes()).hexdigest() == want["sha256"], name
