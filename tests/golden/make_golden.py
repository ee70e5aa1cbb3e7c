#!/usr/bin/env python3
"""Regenerate the golden fixtures in this directory.

Each case is a small deterministic raster (raw bytes, `<name>.in`) and the NICE2
stream the oracle restatement of code::encode (code.rs:59-457) produces for it
(`<name>.nice`); `manifest.json` lists shape, channels and SHA-256 of both.
The oracle itself is pinned by the reference's own known-answer tests
(bitwriter.rs:86-97, bitreader.rs:106-146, hfe.rs:300-348) and by SURVEY.md
Appendix C probe sizes (tests/test_oracle_kat.py).  No reference stream exists
to pin these files against (the Rust reference cannot be built here), so they
freeze the oracle's output: a change in any of them is a parity regression of
either side.

    python tests/golden/make_golden.py          # rewrite fixtures
    python tests/golden/make_golden.py --check  # verify, exit 1 on mismatch
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402


def cases():
    rng = np.random.default_rng(20261015)
    out = [
        ("syn64x64x4_s1", O.gen_syn_v1(64, 64, 4, 1), 64, 64, 4),
        ("syn96x40x3_s7", O.gen_syn_v1(96, 40, 3, 7), 96, 40, 3),
        ("syn160x120x3_s1", O.gen_syn_v1(160, 120, 3, 1), 160, 120, 3),
        ("syn256x128x4_s3", O.gen_syn_v1(256, 128, 4, 3), 256, 128, 4),
        ("syn128x128x3_s1", O.gen_syn_v1(128, 128, 3, 1), 128, 128, 3),
        ("grad48x32x4", O.gen_gradient(48, 32, 4), 48, 32, 4),
        ("noise20x17x3", rng.integers(0, 256, 20 * 17 * 3, dtype=np.uint8), 20, 17, 3),
        ("flat33x9x4", np.tile(np.array([9, 8, 7, 255], np.uint8), 33 * 9), 33, 9, 4),
        ("px1x1x3", np.array([1, 2, 3], np.uint8), 1, 1, 3),
        ("col2x9x3", O.gen_syn_v1(2, 9, 3, 2), 2, 9, 3),
        ("empty0x0x4", np.zeros(0, np.uint8), 0, 0, 4),
    ]
    pal = np.array([[10, 20, 30], [10, 21, 31], [200, 100, 50], [12, 22, 29]], np.uint8)
    idx = rng.integers(0, 4, (30, 40))
    idx[:, 10:25] = 2
    out.append(("palette40x30x3", pal[idx].reshape(-1), 40, 30, 3))
    st = np.zeros((20, 70, 3), np.uint8)
    st[:, :, 0] = (np.arange(20)[:, None] // 3) * 20
    st[::5, ::3, 1] = 200
    out.append(("stripes70x20x3", st.reshape(-1), 70, 20, 3))
    return out


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def main(check):
    manifest = {"generator": "tests/golden/make_golden.py", "cases": []}
    bad = 0
    for name, px, w, h, c in cases():
        px = np.ascontiguousarray(px, np.uint8)
        s, st = O.encode(px, w, h, c, with_stats=True)
        try:
            O.decode(s, O.DEC_STRIDE)
            decodable = True
        except O.OracleDecodeError:
            decodable = False   # e.g. a 5-bit max code length field that spilled (> 31)
        try:
            O.decode(s, O.DEC_REFERENCE)
            ref_decodable = True    # the literal reference decoder terminates on it
        except O.OracleDecodeError:
            ref_decodable = False
        entry = {"name": name, "width": w, "height": h, "channels": c,
                 "max_code_len": list(st.max_aob), "decodable": decodable,
                 "ref_decodable": ref_decodable,
                 "in_sha256": sha(px.tobytes()), "nice_sha256": sha(s), "nice_len": len(s)}
        manifest["cases"].append(entry)
        pin, pst = os.path.join(HERE, name + ".in"), os.path.join(HERE, name + ".nice")
        if check:
            ok = (open(pin, "rb").read() == px.tobytes()) and (open(pst, "rb").read() == s)
            print(("ok  " if ok else "BAD ") + name)
            bad += not ok
        else:
            open(pin, "wb").write(px.tobytes())
            open(pst, "wb").write(s)
    if not check:
        with open(os.path.join(HERE, "manifest.json"), "w") as fh:
            json.dump(manifest, fh, indent=1)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main("--check" in sys.argv))
