"""Minimal PNG reader/writer for the command-line front end (cli.py).

The reference CLI reads and writes PNG through the `png` crate 0.17
(main.rs:28-75, 106-133): 8-bit RGB or RGBA in, RGB out.  This module covers
exactly that subset with the standard library (zlib): non-interlaced 8-bit
truecolour images, all five scanline filters on input, filter 0 on output.
Anything else is refused with ValueError, as the reference panics on it
("unsupported color type", main.rs:45).
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

SIGNATURE = b"\x89PNG\r\n\x1a\n"
_COLOR_CHANNELS = {2: 3, 6: 4}   # colour type -> bytes per pixel (8-bit depth)


def _chunks(data: bytes):
    pos = len(SIGNATURE)
    while pos + 8 <= len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        if zlib.crc32(kind + body) & 0xFFFFFFFF != crc:
            raise ValueError(f"PNG chunk {kind!r}: CRC mismatch")
        yield kind, body
        pos += 12 + n
        if kind == b"IEND":
            return


def _unfilter(raw: bytes, width: int, height: int, bpp: int) -> np.ndarray:
    """Scanline filters 0-4 reversed by nice_png_unfilter (libnice_hip.so)."""
    import ctypes
    from . import lib
    if len(raw) != height * (width * bpp + 1):
        raise ValueError("PNG image data has the wrong size")
    src = np.frombuffer(raw, np.uint8)
    out = np.empty(height * width * bpp, np.uint8)
    L = lib()
    L.nice_png_unfilter.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_void_p]
    if L.nice_png_unfilter(src.ctypes.data, width, height, bpp, out.ctypes.data) != 0:
        raise ValueError("PNG filter type unknown")
    return out


def read_png(path: str):
    """Returns (pixels: uint8 array of H*W*C bytes, width, height, channels)."""
    data = open(path, "rb").read()
    if not data.startswith(SIGNATURE):
        raise ValueError(f"{path}: not a PNG file")
    hdr, idat = None, []
    for kind, body in _chunks(data):
        if kind == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif kind == b"IDAT":
            idat.append(body)
    if hdr is None:
        raise ValueError(f"{path}: no IHDR chunk")
    width, height, depth, ctype, comp, filt, interlace = hdr
    if depth != 8 or ctype not in _COLOR_CHANNELS or comp or filt or interlace:
        raise ValueError("unsupported color type (8-bit non-interlaced RGB / RGBA only)")
    bpp = _COLOR_CHANNELS[ctype]
    px = _unfilter(zlib.decompress(b"".join(idat)), width, height, bpp)
    return px, width, height, bpp


def write_png(path: str, px, width: int, height: int, channels: int = 3, level: int = 6) -> None:
    """Writes 8-bit RGB (channels 3) or RGBA (4) pixels, filter 0."""
    if channels not in (3, 4):
        raise ValueError("channels must be 3 or 4")
    rows = np.asarray(px, np.uint8).reshape(height, width * channels)
    raw = np.concatenate([np.zeros((height, 1), np.uint8), rows], axis=1).tobytes()

    def chunk(kind: bytes, body: bytes) -> bytes:
        return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xFFFFFFFF)

    ctype = 2 if channels == 3 else 6
    with open(path, "wb") as fh:
        fh.write(SIGNATURE)
        fh.write(chunk(b"IHDR", struct.pack(">IIBBBBB", width, height, 8, ctype, 0, 0, 0)))
        fh.write(chunk(b"IDAT", zlib.compress(raw, level)))
        fh.write(chunk(b"IEND", b""))
