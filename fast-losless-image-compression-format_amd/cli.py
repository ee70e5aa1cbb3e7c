"""Command-line front end, mirroring the reference binary (main.rs:17-139):

    python fast-losless-image-compression-format_amd/cli.py IN.png OUT[.nice]
    python fast-losless-image-compression-format_amd/cli.py IN.nice OUT[.png]

A .png input (8-bit RGB or RGBA, main.rs:42-46) is encoded with channels_out =
its channel count (main.rs:66) and written to OUT, ".nice" appended when
missing (main.rs:59-61).  A .nice input is decoded and written as an RGB PNG
(main.rs:106-127), ".png" appended when missing.  The codec runs on the GPU
through libnice_hip.so.  Streams the reference decoder cannot read (4-channel
headers, spilled table headers of small/flat images) are decoded with the
tolerant options; --strict refuses them as the reference would.  Timings are
printed like the reference's (milliseconds).
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys
import time

import numpy as np


def _pkg():
    # the package directory name has hyphens: load it by path
    here = os.path.dirname(os.path.abspath(__file__))
    name = "fast-losless-image-compression-format_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(here, "__init__.py"),
                                                  submodule_search_locations=[here])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--strict", action="store_true", help="decode only what the reference decoder can")
    args = ap.parse_args(argv)
    nice = _pkg()
    png = importlib.import_module(nice.__name__ + ".png")
    dst = args.dst
    print(f"a_file_from: {args.src}")
    print(f"a_file_to: {dst}")
    if args.src.endswith(".png"):
        t0 = time.perf_counter()
        px, w, h, ch = png.read_png(args.src)
        print(f"png: {(time.perf_counter() - t0) * 1e3:.0f}")
        if not dst.endswith(".nice"):
            dst += ".nice"
        print(f"bytes length: {px.size}")
        out = bytearray()
        t1 = time.perf_counter()
        nice.encode(px, nice.Image.new(w, h, ch), ch, out)
        print(f"{(time.perf_counter() - t1) * 1e3:.0f}")
        with open(dst, "wb") as fh:
            fh.write(out)
        print(f"read png file: {args.src}")
        return 0
    if args.src.endswith(".nice"):
        data = open(args.src, "rb").read()
        t0 = time.perf_counter()
        flags = nice.DEC_STRICT_REFERENCE if args.strict else (nice.DEC_TOLERANT_HEADER | nice.DEC_ALPHA_FILL_FF)
        px, img = nice.decode_bytes(data, flags)
        print(f"nice elapsed in: {(time.perf_counter() - t0) * 1e3:.0f}")
        if not dst.endswith(".png"):
            dst += ".png"
        rgb = np.frombuffer(px, np.uint8).reshape(-1, img.channels)[:, :3]
        t1 = time.perf_counter()
        png.write_png(dst, rgb, img.width, img.height, 3)
        print(f"png{(time.perf_counter() - t1) * 1e3:.0f}")
        return 0
    print("input must be a .png or a .nice file", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
