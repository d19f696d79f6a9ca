"""Image files for the rt_image_load tests: every format and variant stb_image's stbi_loadf reads
(stb_image.h v2.30, vendored by the reference; make_image_texture, raytracing.cu:332-341).

JPEG and most PNG / BMP / TGA files come from Pillow; the variants Pillow does not write (Adam7 PNG,
chosen PNG filters and bit depths, DEFLATE block types, BMP bit-field / V4 / V5 / OS/2 headers, 16-bit
and colour-mapped TGA, Radiance HDR, GIF with chosen tables / interlace / transparency / clears, Photoshop PSD
raw and RLE at 8 and 16 bits, Softimage PIC raw / pure / mixed RLE packets) are encoded here from the format
specifications.
"""
from __future__ import annotations

import io
import struct
import zlib

import numpy as np

try:
    from PIL import Image
except ImportError:   # pragma: no cover - Pillow is in this image; the hand-made files still work
    Image = None


def picture(h: int, w: int, seed: int = 0, smooth: bool = True) -> np.ndarray:
    """uint8 [h, w, 3], rows top first: gradients plus noise (JPEG-friendly) or plain noise."""
    rng = np.random.default_rng(seed)
    if not smooth:
        return rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 5 + seed) % 256, (yy * 7) % 256, ((xx + yy) * 3) % 256], -1)
    return np.clip(base + rng.integers(-20, 21, base.shape), 0, 255).astype(np.uint8)


# ---------------------------------------------------------------- Pillow-written files

def pil_bytes(arr: np.ndarray, fmt: str, mode: str | None = None, **kw) -> bytes:
    im = Image.fromarray(arr)
    if mode:
        im = im.convert(mode)
    b = io.BytesIO()
    im.save(b, format=fmt, **kw)
    return b.getvalue()


def jpeg_variants(arr: np.ndarray) -> dict[str, bytes]:
    out = {}
    for ss in (0, 1, 2):
        for q in (25, 75, 100):
            out[f"ss{ss}_q{q}.jpg"] = pil_bytes(arr, "JPEG", quality=q, subsampling=ss)
    out["progressive.jpg"] = pil_bytes(arr, "JPEG", quality=80, progressive=True)
    out["progressive_420.jpg"] = pil_bytes(arr, "JPEG", quality=60, progressive=True, subsampling=2)
    out["optimized.jpg"] = pil_bytes(arr, "JPEG", quality=85, optimize=True)
    out["grey.jpg"] = pil_bytes(arr, "JPEG", mode="L")
    out["grey_progressive.jpg"] = pil_bytes(arr, "JPEG", mode="L", progressive=True)
    out["cmyk.jpg"] = pil_bytes(arr, "JPEG", mode="CMYK")
    out["restart.jpg"] = jpeg_with_restarts(pil_bytes(arr, "JPEG", quality=90, subsampling=2))
    return out


def jpeg_with_restarts(jpg: bytes) -> bytes:
    """Re-encode with restart markers every MCU row (Pillow: restart_marker_rows) when available."""
    try:
        im = Image.open(io.BytesIO(jpg))
        b = io.BytesIO()
        im.save(b, format="JPEG", quality=90, subsampling=2, restart_marker_rows=1)
        return b.getvalue()
    except (TypeError, ValueError, OSError):
        return jpg


def pil_png_variants(arr: np.ndarray) -> dict[str, bytes]:
    out = {f"pil_{m}.png": pil_bytes(arr, "PNG", mode=m) for m in ("RGB", "RGBA", "L", "LA", "P", "1")}
    out["pil_I16.png"] = pil_bytes((arr[:, :, 0].astype(np.uint16) * 257), "PNG")
    return out


def pil_bmp_variants(arr: np.ndarray) -> dict[str, bytes]:
    return {f"pil_{m}.bmp": pil_bytes(arr, "BMP", mode=m) for m in ("RGB", "P", "1", "L")}


def pil_tga_variants(arr: np.ndarray) -> dict[str, bytes]:
    out = {}
    for m in ("RGB", "RGBA", "L", "LA", "P"):
        for comp in (None, "tga_rle"):
            out[f"pil_{m}_{comp or 'raw'}.tga"] = pil_bytes(arr, "TGA", mode=m, compression=comp)
    return out


# ---------------------------------------------------------------- PNG (ISO/IEC 15948)

def _chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


def _pack_row(samples: np.ndarray, depth: int) -> bytes:
    """One scanline's samples (flattened) at `depth` bits, big-endian, padded to a byte."""
    s = samples.astype(np.uint32).ravel()
    if depth == 16:
        return s.astype(">u2").tobytes()
    if depth == 8:
        return s.astype(np.uint8).tobytes()
    per = 8 // depth
    pad = (-len(s)) % per
    s = np.concatenate([s, np.zeros(pad, np.uint32)]).reshape(-1, per)
    shifts = np.array([8 - depth * (i + 1) for i in range(per)], np.uint32)
    return (s << shifts).sum(axis=1).astype(np.uint8).tobytes()


def _filter(raw: bytes, prev: bytes, bpp: int, ftype: int) -> bytes:
    out = bytearray(len(raw))
    for i, x in enumerate(raw):
        a = raw[i - bpp] if i >= bpp else 0
        b = prev[i] if prev else 0
        c = prev[i - bpp] if (prev and i >= bpp) else 0
        if ftype == 0:
            p = 0
        elif ftype == 1:
            p = a
        elif ftype == 2:
            p = b
        elif ftype == 3:
            p = (a + b) >> 1
        else:
            pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
            p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (x - p) & 0xFF
    return bytes(out)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def png_bytes(samples: np.ndarray, color: int, depth: int, *, interlace: bool = False, filters=(0, 1, 2, 3, 4),
              palette: np.ndarray | None = None, trns: bytes | None = None, level: int = 6,
              strategy: int = zlib.Z_DEFAULT_STRATEGY, idat_parts: int = 1) -> bytes:
    """samples: [h, w, channels] integers of the colour type (indices for colour type 3)."""
    h, w = samples.shape[:2]
    ch = samples.shape[2] if samples.ndim == 3 else 1
    bpp = max(1, ch * depth // 8)
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    raw = bytearray()
    k = 0
    for x0, y0, dx, dy in passes:
        sub = samples[y0::dy, x0::dx]
        if sub.size == 0:
            continue
        prev = b""
        for row in sub:
            line = _pack_row(row, depth)
            ft = filters[k % len(filters)]
            k += 1
            raw += bytes([ft]) + _filter(line, prev, bpp, ft)
            prev = line
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 9, strategy)
    z = co.compress(bytes(raw)) + co.flush()
    ihdr = struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, 1 if interlace else 0)
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if palette is not None:
        out += _chunk(b"PLTE", palette.astype(np.uint8).tobytes())
    if trns is not None:
        out += _chunk(b"tRNS", trns)
    out += _chunk(b"tEXt", b"Comment\0test")   # an ancillary chunk to skip
    step = max(1, -(-len(z) // idat_parts))
    for i in range(0, len(z), step):
        out += _chunk(b"IDAT", z[i:i + step])
    return out + _chunk(b"IEND", b"")


def png_variants(arr: np.ndarray, seed: int = 0) -> dict[str, bytes]:
    rng = np.random.default_rng(seed)
    h, w, _ = arr.shape
    out = {}
    for il in (False, True):
        tag = "adam7" if il else "flat"
        out[f"rgb8_{tag}.png"] = png_bytes(arr, 2, 8, interlace=il)
        out[f"rgb16_{tag}.png"] = png_bytes(arr.astype(np.uint16) * 257 + rng.integers(0, 256, arr.shape), 2, 16,
                                            interlace=il)
        out[f"rgba8_{tag}.png"] = png_bytes(np.concatenate([arr, arr[:, :, :1]], -1), 6, 8, interlace=il)
        out[f"rgba16_{tag}.png"] = png_bytes(np.concatenate([arr, arr[:, :, :1]], -1).astype(np.uint16) * 257, 6, 16,
                                             interlace=il)
        out[f"ga8_{tag}.png"] = png_bytes(arr[:, :, :2], 4, 8, interlace=il)
        out[f"ga16_{tag}.png"] = png_bytes(arr[:, :, :2].astype(np.uint16) * 300, 4, 16, interlace=il)
        for d in (1, 2, 4, 8, 16):
            g = (arr[:, :, 1].astype(np.uint32) * ((1 << d) - 1) // 255)[:, :, None]
            out[f"grey{d}_{tag}.png"] = png_bytes(g, 0, d, interlace=il)
        for d in (1, 2, 4, 8):
            n = 1 << d
            pal = rng.integers(0, 256, size=(n, 3))
            idx = rng.integers(0, n, size=(h, w, 1))
            out[f"pal{d}_{tag}.png"] = png_bytes(idx, 3, d, interlace=il, palette=pal)
    pal = rng.integers(0, 256, size=(16, 3))
    out["pal4_trns.png"] = png_bytes(rng.integers(0, 16, size=(h, w, 1)), 3, 4, palette=pal, trns=bytes(range(0, 160, 10)))
    out["rgb8_trns.png"] = png_bytes(arr, 2, 8, trns=struct.pack(">HHH", 1, 2, 3))
    out["grey8_trns.png"] = png_bytes(arr[:, :, :1], 0, 8, trns=struct.pack(">H", 7))
    out["rgb8_stored.png"] = png_bytes(arr, 2, 8, level=0)
    out["rgb8_fixed.png"] = png_bytes(arr, 2, 8, strategy=zlib.Z_FIXED)
    out["rgb8_rle.png"] = png_bytes(arr, 2, 8, strategy=zlib.Z_RLE, level=9)
    out["rgb8_split_idat.png"] = png_bytes(arr, 2, 8, idat_parts=5)
    for f in range(5):
        out[f"rgb8_filter{f}.png"] = png_bytes(arr, 2, 8, filters=(f,))
    return out


# ---------------------------------------------------------------- BMP

def _bmp(info: bytes, extra: bytes, pixel_rows: list[bytes], hsz: int, gap: int = 0) -> bytes:
    data = b"".join(pixel_rows)
    off = 14 + len(info) + len(extra) + gap
    return struct.pack("<2sIHHI", b"BM", off + len(data), 0, 0, off) + info + extra + b"\0" * gap + data


def _rows(vals: np.ndarray, fmt: str, top_down: bool) -> list[bytes]:
    """vals [h, w] per-pixel integers packed with struct fmt ('<H' / '<I'), rows padded to 4 bytes."""
    rows = []
    order = range(vals.shape[0]) if top_down else range(vals.shape[0] - 1, -1, -1)
    for y in order:
        r = b"".join(struct.pack(fmt, int(v)) for v in vals[y])
        rows.append(r + b"\0" * ((-len(r)) % 4))
    return rows


def bmp_variants(arr: np.ndarray, seed: int = 0) -> dict[str, bytes]:
    rng = np.random.default_rng(seed)
    h, w, _ = arr.shape
    r, g, b = (arr[:, :, i].astype(np.uint32) for i in range(3))
    out = {}

    def info40(bpp, compress, top_down=False, colors=0):
        return struct.pack("<IiiHHIIiiII", 40, w, -h if top_down else h, 1, bpp, compress, 0, 2835, 2835, colors, 0)

    v555 = ((r >> 3) << 10) | ((g >> 3) << 5) | (b >> 3)
    out["rgb555.bmp"] = _bmp(info40(16, 0), b"", _rows(v555, "<H", False), 40)
    v565 = ((r >> 3) << 11) | ((g >> 2) << 5) | (b >> 3)
    out["rgb565_bitfields.bmp"] = _bmp(info40(16, 3, True), struct.pack("<III", 0xF800, 0x07E0, 0x001F),
                                       _rows(v565, "<H", True), 40)
    argb = (b << 24) | (g << 16) | (r << 8) | 0x5A   # unusual mask order
    out["bgrx_bitfields.bmp"] = _bmp(info40(32, 3), struct.pack("<III", 0xFF00, 0xFF0000, 0xFF000000),
                                     _rows(argb, "<I", False), 40)
    v444 = ((r >> 4) << 8) | ((g >> 4) << 4) | (b >> 4) | 0xF000
    out["rgb444_bitfields.bmp"] = _bmp(info40(16, 3), struct.pack("<III", 0xF00, 0xF0, 0xF), _rows(v444, "<H", False), 40)
    bgra = (np.uint32(0x80) << 24) | (r << 16) | (g << 8) | b
    for hsz in (108, 124):
        v = struct.pack("<IiiHHIIiiII", hsz, w, h, 1, 32, 3, 0, 2835, 2835, 0, 0)
        v += struct.pack("<IIII", 0xFF0000, 0xFF00, 0xFF, 0xFF000000) + b"BGRs" + b"\0" * 48
        if hsz == 124:
            v += b"\0" * 16
        out[f"v{4 if hsz == 108 else 5}_32.bmp"] = _bmp(v, b"", _rows(bgra, "<I", False), hsz)
        v24 = struct.pack("<IiiHHIIiiII", hsz, w, h, 1, 24, 0, 0, 2835, 2835, 0, 0) + b"\0" * (hsz - 40)
        rows24 = []
        for y in range(h - 1, -1, -1):
            row = arr[y, :, ::-1].tobytes()
            rows24.append(row + b"\0" * ((-len(row)) % 4))
        out[f"v{4 if hsz == 108 else 5}_24.bmp"] = _bmp(v24, b"", rows24, hsz)
    # 24-bit with a gap between header and pixels (stb's double skip of it)
    out["gap_24.bmp"] = _bmp(info40(24, 0), b"", [arr[y, :, ::-1].tobytes() + b"\0" * ((-3 * w) % 4)
                                                  for y in range(h - 1, -1, -1)], 40, gap=8)
    # OS/2 (12-byte header): 24-bit and 8-bit with a 3-byte palette
    os2 = struct.pack("<IHHHH", 12, w, h, 1, 24)
    out["os2_24.bmp"] = _bmp(os2, b"", [arr[y, :, ::-1].tobytes() + b"\0" * ((-3 * w) % 4)
                                        for y in range(h - 1, -1, -1)], 12)
    pal = rng.integers(0, 256, size=(256, 3), dtype=np.uint8)
    idx = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    os2_8 = struct.pack("<IHHHH", 12, w, h, 1, 8)
    out["os2_pal8.bmp"] = _bmp(os2_8, pal[:, ::-1].tobytes(), [idx[y].tobytes() + b"\0" * ((-w) % 4)
                                                               for y in range(h - 1, -1, -1)], 12)
    # 4-bit and 1-bit palettes (4-byte entries)
    pal16 = rng.integers(0, 256, size=(16, 4), dtype=np.uint8)
    idx4 = rng.integers(0, 16, size=(h, w), dtype=np.uint8)
    rows4 = []
    for y in range(h - 1, -1, -1):
        v = list(idx4[y]) + ([0] if w % 2 else [])
        row = bytes((v[i] << 4) | v[i + 1] for i in range(0, len(v), 2))
        rows4.append(row + b"\0" * ((-len(row)) % 4))
    out["pal4.bmp"] = _bmp(info40(4, 0, colors=16), pal16.tobytes(), rows4, 40)
    pal2 = rng.integers(0, 256, size=(2, 4), dtype=np.uint8)
    bits = rng.integers(0, 2, size=(h, w), dtype=np.uint8)
    rows1 = []
    for y in range(h):
        row = np.packbits(bits[y]).tobytes()
        rows1.append(row + b"\0" * ((-len(row)) % 4))
    out["pal1_topdown.bmp"] = _bmp(info40(1, 0, True, colors=2), pal2.tobytes(), rows1, 40)
    return out


# ---------------------------------------------------------------- TGA

def tga_variants(arr: np.ndarray, seed: int = 0) -> dict[str, bytes]:
    rng = np.random.default_rng(seed)
    h, w, _ = arr.shape
    r, g, b = (arr[:, :, i].astype(np.uint32) >> 3 for i in range(3))
    v = ((r << 10) | (g << 5) | b).astype("<u2")
    out = {}
    out["rgb16.tga"] = struct.pack("<BBBHHBHHHHBB", 0, 0, 2, 0, 0, 0, 0, 0, w, h, 16, 0) + v[::-1].tobytes()
    out["rgb15_topdown_id.tga"] = (struct.pack("<BBBHHBHHHHBB", 5, 0, 2, 0, 0, 0, 0, 0, w, h, 15, 0x20) + b"hello"
                                   + v.tobytes())
    pal = rng.integers(0, 1 << 15, size=40).astype("<u2")
    idx = rng.integers(0, 40, size=(h, w), dtype=np.uint8)
    out["cmap16.tga"] = (struct.pack("<BBBHHBHHHHBB", 0, 1, 1, 0, 40, 16, 0, 0, w, h, 8, 0) + pal.tobytes()
                         + idx[::-1].tobytes())
    pal24 = rng.integers(0, 256, size=(300, 3), dtype=np.uint8)
    idx16 = rng.integers(0, 300, size=(h, w)).astype("<u2")
    out["cmap24_idx16.tga"] = (struct.pack("<BBBHHBHHHHBB", 0, 1, 1, 0, 300, 24, 0, 0, w, h, 16, 0x20)
                               + pal24.tobytes() + idx16.tobytes())
    return out


# ---------------------------------------------------------------- Radiance HDR

def _rgbe(h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    m = rng.integers(128, 256, size=(h, w, 3), dtype=np.uint8)
    e = rng.integers(110, 140, size=(h, w, 1), dtype=np.uint8)
    e[0, 0, 0] = 0   # a zero exponent: black
    return np.concatenate([m, e], -1)


def _rle_channel(vals: bytes) -> bytes:
    out = bytearray()
    i = 0
    n = len(vals)
    while i < n:
        run = 1
        while i + run < n and run < 127 and vals[i + run] == vals[i]:
            run += 1
        if run >= 3:
            out += bytes([128 + run, vals[i]])
            i += run
            continue
        j = i
        while j < n and j - i < 128 and not (j + 2 < n and vals[j] == vals[j + 1] == vals[j + 2]):
            j += 1
        out += bytes([j - i]) + vals[i:j]
        i = j
    return bytes(out)


def hdr_bytes(rgbe: np.ndarray, rle: bool, header: bytes = b"#?RADIANCE\n# made for tests\nFORMAT=32-bit_rle_rgbe\n\n") -> bytes:
    h, w, _ = rgbe.shape
    out = header + b"-Y %d +X %d\n" % (h, w)
    if not rle:
        return out + rgbe.tobytes()
    for y in range(h):
        out += bytes([2, 2, w >> 8, w & 255])
        for c in range(4):
            out += _rle_channel(rgbe[y, :, c].tobytes())
    return out


def hdr_variants(seed: int = 0) -> dict[str, bytes]:
    big = _rgbe(9, 40, seed)
    big[3, 5:30, :] = big[3, 5, :]   # runs
    return {
        "flat_narrow.hdr": hdr_bytes(_rgbe(6, 5, seed), rle=False),
        "rle.hdr": hdr_bytes(big, rle=True),
        "flat_wide.hdr": hdr_bytes(_rgbe(4, 12, seed + 1), rle=False),   # width >= 8, not RLE: stb's goto
        "rgbe_magic.hdr": hdr_bytes(_rgbe(3, 9, seed + 2), rle=True, header=b"#?RGBE\nFORMAT=32-bit_rle_rgbe\n\n"),
    }


def hdr_expected(data_rgbe: np.ndarray) -> np.ndarray:
    """stbi__hdr_convert: mantissa * 2^(e - 136), zero exponent -> 0."""
    m = data_rgbe[:, :, :3].astype(np.float32)
    e = data_rgbe[:, :, 3:4].astype(np.int32)
    f = np.ldexp(np.float32(1.0), e - 136).astype(np.float32)
    return np.where(e == 0, np.float32(0), m * f).astype(np.float32)


# ---------------------------------------------------------------- GIF (first image; GIF89a / 87a)

def gif_lzw(indices: bytes, min_size: int, clear_every: int = 0) -> bytes:
    """LZW data sub-blocks of one raster: a clear code first, the code width growing with the table (12 bits at
    most, a clear when it is full, or every `clear_every` codes), the end code last."""
    clear, end = 1 << min_size, (1 << min_size) + 1
    out, acc, nbits = bytearray(), 0, 0
    size = min_size + 1

    def emit(code):
        nonlocal acc, nbits
        acc |= code << nbits
        nbits += size
        while nbits >= 8:
            out.append(acc & 0xFF)
            acc >>= 8
            nbits -= 8

    def reset():
        return {bytes([i]): i for i in range(clear)}, clear + 2

    table, nxt = reset()
    emit(clear)
    w, emitted = b"", 0
    for b in indices:
        wc = w + bytes([b])
        if wc in table:
            w = wc
            continue
        emit(table[w])
        emitted += 1
        if nxt < 4096 and not (clear_every and emitted % clear_every == 0):
            table[wc] = nxt
            nxt += 1
            if nxt - 1 == (1 << size) and size < 12:
                size += 1
        else:
            emit(clear)
            size = min_size + 1
            table, nxt = reset()
        w = bytes([b])
    if w:
        emit(table[w])
    emit(end)
    if nbits:
        out.append(acc & 0xFF)
    blocks = bytearray()
    for i in range(0, len(out), 255):
        chunk = out[i:i + 255]
        blocks += bytes([len(chunk)]) + chunk
    return bytes(blocks) + b"\0"


def _gif_table(pal: np.ndarray, bits: int) -> bytes:
    t = np.zeros((1 << bits, 3), np.uint8)
    t[:len(pal)] = pal[: 1 << bits]
    return t.tobytes()


def gif_bytes(idx: np.ndarray, pal: np.ndarray, *, local: bool = False, interlace: bool = False, version: bytes = b"89a",
              transparent: int | None = None, bgindex: int = 0, screen: tuple | None = None, offset=(0, 0),
              extras: bytes = b"", clear_every: int = 0, bits: int = 8) -> bytes:
    """idx uint8 [h, w] into `pal` (n x 3); the image at `offset` of a logical screen (default: the image)."""
    h, w = idx.shape
    sw, sh = screen or (w + offset[0], h + offset[1])
    g = b"GIF" + version + struct.pack("<HHBBB", sw, sh, 0 if local else 0x80 | (bits - 1), bgindex, 0)
    if not local:
        g += _gif_table(pal, bits)
    g += extras
    if transparent is not None:
        g += b"\x21\xF9\x04\x01\x00\x00" + bytes([transparent]) + b"\0"
    rows = idx
    if interlace:
        order = list(range(0, h, 8)) + list(range(4, h, 8)) + list(range(2, h, 4)) + list(range(1, h, 2))
        rows = idx[order]
    flags = (0x40 if interlace else 0) | ((0x80 | (bits - 1)) if local else 0)
    g += b"\x2C" + struct.pack("<HHHHB", offset[0], offset[1], w, h, flags)
    if local:
        g += _gif_table(pal, bits)
    g += bytes([max(2, bits)]) + gif_lzw(rows.astype(np.uint8).tobytes(), max(2, bits), clear_every)
    return g + b"\x3B"


def gif_variants(arr: np.ndarray, seed: int = 0) -> dict[str, bytes]:
    rng = np.random.default_rng(seed)
    h, w, _ = arr.shape
    out = {}
    pal = rng.integers(0, 256, size=(256, 3), dtype=np.uint8)
    idx = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    out["g_global.gif"] = gif_bytes(idx, pal)
    out["g_local_interlaced.gif"] = gif_bytes(idx, pal, local=True, interlace=True)
    out["g_87a_4bit.gif"] = gif_bytes(idx & 15, pal, version=b"87a", bits=4)
    out["g_2bit_runs.gif"] = gif_bytes(np.repeat(idx[:, :1] & 3, w, axis=1), pal, bits=2)
    out["g_transparent_bg.gif"] = gif_bytes(idx & 7, pal, transparent=3, bgindex=5, bits=3,
                                            screen=(w + 3, h + 2), offset=(2, 1))
    out["g_local_transparent.gif"] = gif_bytes(idx & 7, pal, local=True, transparent=0, bits=3)
    out["g_clears.gif"] = gif_bytes(idx, pal, clear_every=37)
    ext = b"\x21\xFE\x05hello\0" + b"\x21\xFF\x0BNETSCAPE2.0\x03\x01\x00\x00\0"
    out["g_extensions.gif"] = gif_bytes(idx & 63, pal, extras=ext, bits=6)
    if Image is not None:
        out["pil_P.gif"] = pil_bytes(arr, "GIF")
        out["pil_L_interlace.gif"] = pil_bytes(arr, "GIF", mode="L", interlace=True)
    return out


# ---------------------------------------------------------------- Photoshop PSD

def _packbits(row: bytes) -> bytes:
    out, i, n = bytearray(), 0, len(row)
    while i < n:
        j = i
        while j + 1 < n and row[j + 1] == row[i] and j - i < 127:
            j += 1
        if j > i:                                  # a run of j - i + 1
            out += bytes([257 - (j - i + 1), row[i]])
            i = j + 1
            continue
        j = i
        while j < n and j - i < 128 and not (j + 1 < n and row[j + 1] == row[j]):
            j += 1
        j = max(j, i + 1)
        out += bytes([j - i - 1]) + row[i:j]
        i = j
    return bytes(out)


def psd_bytes(planes: np.ndarray, *, depth: int = 8, rle: bool = False, mode: int = 3, extra: bytes = b"") -> bytes:
    """planes [c, h, w] (uint8, or uint16 for depth 16), channel by channel."""
    c, h, w = planes.shape
    b = b"8BPS" + struct.pack(">H6xHIIHH", 1, c, h, w, depth, mode)
    b += struct.pack(">I", len(extra)) + extra + struct.pack(">I", 0) + struct.pack(">I", 0)
    if not rle:
        dt = ">u2" if depth == 16 else "u1"
        return b + struct.pack(">H", 0) + planes.astype(dt).tobytes()
    rows = [_packbits(planes[k, y].astype(np.uint8).tobytes()) for k in range(c) for y in range(h)]
    return b + struct.pack(">H", 1) + b"".join(struct.pack(">H", len(r)) for r in rows) + b"".join(rows)


def psd_variants(arr: np.ndarray, seed: int = 0) -> dict[str, bytes]:
    rng = np.random.default_rng(seed)
    h, w, _ = arr.shape
    rgb = np.moveaxis(arr, 2, 0)
    alpha = rng.integers(0, 256, size=(1, h, w), dtype=np.uint8)
    alpha[0, :, ::3] = 255
    alpha[0, ::4, :] = 0
    runs = np.repeat(rgb[:, :, :1], w, axis=2)
    out = {}
    out["p_rgb.psd"] = psd_bytes(rgb)
    out["p_rgba.psd"] = psd_bytes(np.concatenate([rgb, alpha]))
    out["p_rgb_rle.psd"] = psd_bytes(rgb, rle=True)
    out["p_runs_rle.psd"] = psd_bytes(runs, rle=True)
    out["p_rgba_rle.psd"] = psd_bytes(np.concatenate([rgb, alpha]), rle=True, extra=b"\0" * 7)
    out["p_5ch.psd"] = psd_bytes(np.concatenate([rgb, alpha, alpha[:, ::-1]]))
    out["p_grey1ch.psd"] = psd_bytes(rgb[:1])
    out["p_2ch_rle.psd"] = psd_bytes(rgb[:2], rle=True)
    out["p_rgb16.psd"] = psd_bytes(rgb.astype(np.uint16) * 257 + rng.integers(0, 257, size=rgb.shape), depth=16)
    out["p_rgba16.psd"] = psd_bytes(np.concatenate([rgb, alpha]).astype(np.uint16) * 256 + 128, depth=16)
    out["p_cmyk.psd"] = psd_bytes(rgb, mode=4)   # not RGB: a failed load
    return out


# ---------------------------------------------------------------- Softimage PIC

def _pic_header(w: int, h: int) -> bytes:
    return (b"\x53\x80\xF6\x34" + struct.pack(">f", 3.71) + b"made for tests".ljust(80, b"\0") + b"PICT"
            + struct.pack(">HHfHH", w, h, 1.0, 3, 0))


def _pic_values(px: np.ndarray, mask: int) -> bytes:
    """the channels of `mask` (0x80 R, 0x40 G, 0x20 B, 0x10 A) of pixels px [n, 4], in that order"""
    cols = [k for k in range(4) if mask & (0x80 >> k)]
    return px[:, cols].astype(np.uint8).tobytes()


def _pic_row(px: np.ndarray, mask: int, kind: int) -> bytes:
    n = len(px)
    if kind == 0:
        return _pic_values(px, mask)
    out, i = bytearray(), 0
    while i < n:
        j = i
        while j + 1 < n and np.array_equal(px[j + 1], px[i]) and j - i < (254 if kind == 1 else 300):
            j += 1
        run = j - i + 1
        if kind == 1:                                  # pure RLE: count, value
            out += bytes([run]) + _pic_values(px[i:i + 1], mask)
        elif run > 1:                                  # mixed RLE: a repeat
            out += (bytes([run + 127]) if run <= 128 else b"\x80" + struct.pack(">H", run)) + _pic_values(px[i:i + 1], mask)
        else:                                          # mixed RLE: raw texels up to the next repeat
            j = i
            while j + 1 < n and j - i < 127 and not np.array_equal(px[j + 1], px[j]):
                j += 1
            run = j - i + 1
            out += bytes([run - 1]) + _pic_values(px[i:i + run], mask)
        i += run
    return bytes(out)


def pic_bytes(rgba: np.ndarray, packets: list[tuple[int, int]]) -> bytes:
    """rgba [h, w, 4]; packets: (channel mask, type 0 raw / 1 pure RLE / 2 mixed RLE), chained in order"""
    h, w, _ = rgba.shape
    b = _pic_header(w, h)
    for k, (mask, kind) in enumerate(packets):
        b += bytes([1 if k + 1 < len(packets) else 0, 8, kind, mask])
    for y in range(h):
        for mask, kind in packets:
            b += _pic_row(rgba[y], mask, kind)
    return b


def pic_variants(arr: np.ndarray, seed: int = 0) -> dict[str, bytes]:
    rng = np.random.default_rng(seed)
    h, w, _ = arr.shape
    a = rng.integers(0, 256, size=(h, w, 1), dtype=np.uint8)
    rgba = np.concatenate([arr, a], axis=2)
    runs = rgba.copy()
    runs[:, : w // 2] = runs[:, :1]
    out = {}
    out["raw.pic"] = pic_bytes(rgba, [(0xE0, 0)])
    out["raw_alpha.pic"] = pic_bytes(rgba, [(0xE0, 0), (0x10, 0)])
    out["pure.pic"] = pic_bytes(runs, [(0xE0, 1)])
    out["mixed.pic"] = pic_bytes(runs, [(0xE0, 2), (0x10, 2)])
    out["mixed_long.pic"] = pic_bytes(np.repeat(rgba[:, :1], w, axis=1), [(0xF0, 2)])
    out["split_channels.pic"] = pic_bytes(runs, [(0x80, 1), (0x40, 2), (0x20, 0)])
    out["green_only.pic"] = pic_bytes(rgba, [(0x40, 0)])
    return out


def corpus(seed: int = 0, h: int = 37, w: int = 53) -> dict[str, bytes]:
    """Every variant, for one picture size."""
    arr = picture(h, w, seed)
    files = {}
    if Image is not None:
        files.update(jpeg_variants(arr))
        files.update(pil_png_variants(arr))
        files.update(pil_bmp_variants(arr))
        files.update(pil_tga_variants(arr))
    files.update(png_variants(arr, seed))
    files.update(bmp_variants(arr, seed))
    files.update(tga_variants(arr, seed))
    files.update(hdr_variants(seed))
    files.update(gif_variants(arr, seed))
    files.update(psd_variants(arr, seed))
    files.update(pic_variants(arr, seed))
    return files
