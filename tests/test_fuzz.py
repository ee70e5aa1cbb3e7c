"""Corrupted streams: bit flips in the data of valid streams must be decoded by
the HIP path exactly as the oracle decodes them -- the same pixels where the
oracle decodes, an error where it fails -- in the default (intent) mode and in
STRICT_REFERENCE mode (the literal reference, RGB streams).  Exercises the
decoder's error paths: sync, first-pass events and their placement, head
emission, reconstruction."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [("syn97x50x3", 97, 50, 3, 2), ("syn300x200x3", 300, 200, 3, 5), ("syn160x120x4", 160, 120, 4, 4),
         ("grad120x80x3", 120, 80, 3, 0)]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_bitflip_parity(nice, O, case):
    name, w, h, c, seed = case
    px = O.gen_gradient(w, h, c) if seed == 0 else O.gen_syn_v1(w, h, c, seed)
    s = O.encode(px, w, h, c)
    rng = np.random.default_rng(seed + 100)
    for t in range(24):
        b = bytearray(s)
        for _ in range(int(rng.integers(1, 4))):
            pos = int(rng.integers(13 + 40, len(b)))   # past the header and most of the tables
            b[pos] ^= 1 << int(rng.integers(0, 8))
        b = bytes(b)
        modes = [(nice.DEC_ALPHA_FILL_FF, O.DEC_STRIDE)]
        if c == 3:
            modes.append((nice.DEC_STRICT_REFERENCE, O.DEC_REFERENCE))
        for gflags, oflags in modes:
            try:
                ref, _ = O.decode(b, oflags)
            except O.OracleDecodeError:
                ref = None
            try:
                got, _ = nice.decode_bytes(b, flags=gflags)
            except nice.NiceError:
                got = None
            assert (ref is None) == (got is None), (name, t, oflags)
            if ref is not None:
                g = np.frombuffer(got, np.uint8)[: ref.size].reshape(-1, c)[:, :3]
                assert np.array_equal(g, ref.reshape(-1, c)[:, :3]), (name, t, oflags)
