"""Diagnostic: strip-split decode of a few images against the originals;
prints the first mismatching pixels (row, column, strip).  GPU only."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib
nice = importlib.import_module("fast-losless-image-compression-format_amd")
from oracle import oracle as O

def stripes(w, h):
    st = np.zeros((h, w, 3), np.uint8)
    st[:, :, 0] = (np.arange(h)[:, None] // 7) * 20
    st[::5, ::3, 1] = 200
    return st.reshape(-1)

for k in (2, 3):
    os.environ["NICE_DEC_SPLIT"] = str(k)
    for name, px, w, h in [("stripes900x60", stripes(900, 60), 900, 60), ("stripes900x12", stripes(900, 12), 900, 12),
                           ("flat", np.full(900 * 10 * 3, 7, np.uint8), 900, 10)]:
        s = O.encode(px, w, h, 3)
        try:
            got, _ = nice.decode_bytes(s, flags=nice.DEC_TOLERANT_HEADER)
        except nice.NiceError as e:
            print(k, name, "error", e); continue
        g = np.frombuffer(got, np.uint8).reshape(h, w, 3)
        e = px.reshape(h, w, 3)
        bad = np.argwhere((g != e).any(axis=2))
        nseg = (w + 15) // 16; sps = (nseg + k - 1) // k
        print(k, name, "mismatches", len(bad))
        for (yy, xx) in bad[:12]:
            print("   row", yy, "col", xx, "strip", (xx // 16) // sps, "got", g[yy, xx], "want", e[yy, xx])
