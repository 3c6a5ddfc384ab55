"""OpenEXR scanline images (host side): the reader behind the image primitive's `Testbed::load_exr_image`
(src/testbed_image.cu:389-402 -> load_exr_gpu, src/common_device.cu:37-45 -> tinyexr LoadEXRFromMemory,
src/tinyexr_wrapper.cu:125-150), which the reference gets from the vendored tinyexr (dependencies/tinyexr).

Restated from the OpenEXR file layout (the spec tinyexr implements), numpy + zlib only:
  magic 20000630, version 2 (single-part scanline); header = attributes (name\\0 type\\0 int32 size value)
  ended by an empty name; then one uint64 offset per chunk; each chunk = int32 first scanline, int32
  byte count, data. Channels are stored in name order, each as a run of `width` values per scanline.
  Compression: NONE (0), ZIPS (2, one scanline per chunk), ZIP (3, 16 scanlines): zlib, then undo the
  byte predictor (b[i] += b[i-1] - 128) and the even/odd byte interleave.
Output follows LoadEXRFromMemory: RGBA float32 [height, width, 4], rows top to bottom; a missing A is 1,
a single-channel image fills R=G=B. Tiled, multi-part, deep and lossy (PIZ/PXR24/B44/DWA) files raise.
"""
import struct
import zlib

import numpy as np

MAGIC = 20000630
_PIXEL = {0: (np.uint32, 4), 1: (np.float16, 2), 2: (np.float32, 4)}  # UINT, HALF, FLOAT
_LINES_PER_CHUNK = {0: 1, 2: 1, 3: 16}


class ExrError(RuntimeError):
    pass


def _parse_header(buf):
    magic, version = struct.unpack_from("<ii", buf, 0)
    if magic != MAGIC:
        raise ExrError("not an OpenEXR file")
    if version & 0x200:
        raise ExrError("tiled EXR images are not supported")
    if version & 0x1000 or version & 0x800:
        raise ExrError("multi-part / deep EXR images are not supported")
    pos, attrs = 8, {}
    while True:
        end = buf.index(b"\0", pos)
        name = buf[pos:end].decode()
        pos = end + 1
        if not name:
            break
        end = buf.index(b"\0", pos)
        typ = buf[pos:end].decode()
        size = struct.unpack_from("<i", buf, end + 1)[0]
        attrs[name] = (typ, bytes(buf[end + 5:end + 5 + size]))
        pos = end + 5 + size
    return attrs, pos


def _channels(value):
    out, pos = [], 0
    while value[pos] != 0:
        end = value.index(b"\0", pos)
        name = value[pos:end].decode()
        ptype, = struct.unpack_from("<i", value, end + 1)
        out.append((name, ptype))
        pos = end + 1 + 16  # pixel type, pLinear + reserved, xSampling, ySampling
    return out


def _unzip(data, expected):
    raw = np.frombuffer(zlib.decompress(data), np.uint8)
    if raw.size != expected:
        raise ExrError(f"ZIP chunk inflated to {raw.size} bytes, expected {expected}")
    # predictor: t[i] = t[i-1] + raw[i] - 128 (mod 256)
    t = (np.cumsum(raw.astype(np.int64) - 128) + 128) % 256
    t[0] = raw[0]
    t = t.astype(np.uint8)
    # the first half holds the even bytes, the second half the odd bytes
    out = np.empty_like(t)
    half = (t.size + 1) // 2
    out[0::2] = t[:half]
    out[1::2] = t[half:]
    return out


def read_exr(path):
    """RGBA float32 [height, width, 4] as tinyexr's LoadEXRFromMemory returns it."""
    buf = open(path, "rb").read()
    attrs, pos = _parse_header(buf)
    for need in ("channels", "compression", "dataWindow"):
        if need not in attrs:
            raise ExrError(f"EXR header lacks '{need}'")
    chans = _channels(attrs["channels"][1])
    comp = attrs["compression"][1][0]
    if comp not in _LINES_PER_CHUNK:
        raise ExrError(f"EXR compression {comp} is not supported (NONE, ZIPS, ZIP only)")
    x0, y0, x1, y1 = struct.unpack("<iiii", attrs["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    lpc = _LINES_PER_CHUNK[comp]
    n_chunks = (h + lpc - 1) // lpc
    offsets = struct.unpack_from(f"<{n_chunks}Q", buf, pos)
    planes = {name: np.empty((h, w), _PIXEL[t][0]) for name, t in chans}
    row_bytes = sum(_PIXEL[t][1] for _, t in chans) * w
    for off in offsets:
        y, size = struct.unpack_from("<ii", buf, off)
        data = bytes(buf[off + 8:off + 8 + size])
        r0 = y - y0
        nl = min(lpc, h - r0)
        expected = nl * row_bytes
        block = np.frombuffer(data, np.uint8) if size == expected else _unzip(data, expected)
        p = 0
        for r in range(nl):
            for name, t in chans:
                dt, bpp = _PIXEL[t]
                planes[name][r0 + r] = np.frombuffer(block[p:p + w * bpp].tobytes(), dt)
                p += w * bpp
    out = np.zeros((h, w, 4), np.float32)
    names = {n.split(".")[-1].upper(): n for n in planes}
    if len(planes) == 1:
        v = next(iter(planes.values())).astype(np.float32)
        out[..., 0] = out[..., 1] = out[..., 2] = v
        out[..., 3] = 1.0
        return out
    for i, c in enumerate("RGBA"):
        if c in names:
            out[..., i] = planes[names[c]].astype(np.float32)
        elif c == "A":
            out[..., 3] = 1.0
    return out


def write_exr(path, rgba, compression=3, pixel_type=2):
    """Scanline EXR writer (NONE / ZIPS / ZIP; HALF or FLOAT channels A, B, G, R) for fixtures and tests."""
    rgba = np.asarray(rgba, np.float32)
    h, w = rgba.shape[:2]
    dt, bpp = _PIXEL[pixel_type]
    chans = [("A", 3), ("B", 2), ("G", 1), ("R", 0)]

    def attr(name, typ, value):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(value)) + value

    chl = b"".join(c.encode() + b"\0" + struct.pack("<iiii", pixel_type, 0, 1, 1) for c, _ in chans) + b"\0"
    box = struct.pack("<iiii", 0, 0, w - 1, h - 1)
    header = struct.pack("<ii", MAGIC, 2)
    header += attr("channels", "chlist", chl) + attr("compression", "compression", bytes([compression]))
    header += attr("dataWindow", "box2i", box) + attr("displayWindow", "box2i", box)
    header += attr("lineOrder", "lineOrder", b"\0") + attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    header += attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0)) + attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    header += b"\0"
    lpc = _LINES_PER_CHUNK[compression]
    chunks = []
    for y in range(0, h, lpc):
        nl = min(lpc, h - y)
        raw = b"".join(rgba[y + r, :, i].astype(dt).tobytes() for r in range(nl) for _, i in chans)
        if compression != 0:
            b = np.frombuffer(raw, np.uint8)
            inter = np.concatenate([b[0::2], b[1::2]]).astype(np.int64)
            pred = inter.copy()
            pred[1:] = (inter[1:] - inter[:-1] + 128 + 256) % 256
            z = zlib.compress(pred.astype(np.uint8).tobytes())
            raw = z if len(z) < len(raw) else raw
        chunks.append(struct.pack("<ii", y, len(raw)) + raw)
    table_at = len(header)
    data_at = table_at + 8 * len(chunks)
    offs, cur = [], data_at
    for c in chunks:
        offs.append(cur)
        cur += len(c)
    with open(path, "wb") as f:
        f.write(header + struct.pack(f"<{len(offs)}Q", *offs) + b"".join(chunks))
