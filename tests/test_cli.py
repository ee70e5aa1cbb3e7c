"""Command-line front end (reference main.rs:17-139):
PNG I/O on the CPU, then PNG -> .nice -> PNG through the GPU codec, with the
.nice bytes equal to the oracle's code::encode of the PNG's pixels."""
import importlib
import os
import struct
import subprocess
import sys
import zlib

import numpy as np
import pytest

from conftest import ROOT, PKG_NAME

CLI = os.path.join(ROOT, PKG_NAME, "cli.py")


def _png_mod():
    return importlib.import_module(PKG_NAME + ".png")


def _write_filtered_png(path, px, w, h, c, filters):
    """PNG whose scanlines use the given filter types (cycled), to exercise the
    reader's unfiltering."""
    rows = px.reshape(h, w * c).astype(np.int32)
    out = bytearray()
    prev = np.zeros(w * c, np.int32)
    for y in range(h):
        ft = filters[y % len(filters)]
        cur = rows[y]
        a = np.concatenate([np.zeros(c, np.int32), cur[:-c]])
        b = prev
        cc = np.concatenate([np.zeros(c, np.int32), prev[:-c]])
        if ft == 0: pred = np.zeros_like(cur)
        elif ft == 1: pred = a
        elif ft == 2: pred = b
        elif ft == 3: pred = (a + b) >> 1
        else:
            p = a + b - cc
            pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - cc)
            pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, cc))
        out.append(ft)
        out.extend(((cur - pred) & 255).astype(np.uint8).tobytes())
        prev = cur

    def chunk(kind, body):
        return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xFFFFFFFF)
    with open(path, "wb") as fh:
        fh.write(b"\x89PNG\r\n\x1a\n")
        fh.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2 if c == 3 else 6, 0, 0, 0)))
        fh.write(chunk(b"IDAT", zlib.compress(bytes(out))))
        fh.write(chunk(b"IEND", b""))


@pytest.mark.parametrize("c", [3, 4])
def test_png_reader_all_filters(tmp_path, O, c):
    png = _png_mod()
    w, h = 37, 21
    px = O.gen_syn_v1(w, h, c, 3)
    p = str(tmp_path / "f.png")
    _write_filtered_png(p, px, w, h, c, [0, 1, 2, 3, 4])
    got, gw, gh, gc = png.read_png(p)
    assert (gw, gh, gc) == (w, h, c)
    assert np.array_equal(got, px)


def test_png_writer_roundtrip(tmp_path, O):
    png = _png_mod()
    px = O.gen_syn_v1(50, 30, 3, 1)
    p = str(tmp_path / "w.png")
    png.write_png(p, px, 50, 30, 3)
    got, w, h, c = png.read_png(p)
    assert (w, h, c) == (50, 30, 3) and np.array_equal(got, px)


def test_png_rejects_unsupported(tmp_path):
    png = _png_mod()
    p = str(tmp_path / "g.png")
    body = struct.pack(">IIBBBBB", 4, 4, 8, 0, 0, 0, 0)   # grayscale
    with open(p, "wb") as fh:
        fh.write(b"\x89PNG\r\n\x1a\n" + struct.pack(">I", len(body)) + b"IHDR" + body +
                 struct.pack(">I", zlib.crc32(b"IHDR" + body) & 0xFFFFFFFF))
    with pytest.raises(ValueError):
        png.read_png(p)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,c", [(320, 200, 3), (256, 144, 4), (24, 24, 3)])
def test_cli_png_nice_png(tmp_path, O, w, h, c):
    png = _png_mod()
    px = O.gen_syn_v1(w, h, c, 7)
    src = str(tmp_path / "in.png")
    _write_filtered_png(src, px, w, h, c, [4, 1, 2])
    r = subprocess.run([sys.executable, CLI, src, str(tmp_path / "out")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    stream = open(str(tmp_path / "out.nice"), "rb").read()
    assert stream == O.encode(px, w, h, c)          # main.rs:66: channels_out = channels
    r = subprocess.run([sys.executable, CLI, str(tmp_path / "out.nice"), str(tmp_path / "back")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got, gw, gh, gc = png.read_png(str(tmp_path / "back.png"))
    assert (gw, gh, gc) == (w, h, 3)                # main.rs:116: RGB output
    assert np.array_equal(got.reshape(-1, 3), px.reshape(-1, c)[:, :3])
