"""Diagnostic: encode frames of given shapes on the GPU and compare with the
oracle byte for byte (NICE_LIB_PATH selects a library build).
Usage: enc_check.py W H C [W H C ...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import importlib
import numpy as np
nice = importlib.import_module("fast-losless-image-compression-format_amd")
from oracle import oracle as O
import test_width_sweep as tw
a = [int(x) for x in sys.argv[1:]]
for i in range(0, len(a), 3):
    W, H, C = a[i:i + 3]
    for gen in ("sweep", "syn"):
        px = tw._frame(O, W, C, W * 7 + C) if gen == "sweep" and H == 12 else O.gen_syn_v1(W, H, C, 1)
        want = O.encode(px, W, H, C)
        got = bytes(nice.encode_bytes(px, W, H, C))
        d = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), None)
        print(f"{W}x{H}x{C} {gen}: {'OK' if got == want else f'DIFF len {len(got)}/{len(want)} first {d}'}", flush=True)
