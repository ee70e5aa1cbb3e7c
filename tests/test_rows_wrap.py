"""References that wrap past the row end into the row being decoded.

Luma reference 3 (offset W-3, code.rs:141-142) of the pixel at column W-3 is
pixel 0 of the *same* row (one row up, three to the right, wrapped).  The row
kernel resolves such references after lane 0 has its first three pixels
(W_CUR).  With W % 16 in {1, 2} the last 16-pixel segment holds only one or
two pixels, so column W-3 lies in the second-to-last segment: these frames
place a pixel at column W-3 that only luma reference 3 predicts (a fresh
random colour at columns 0 / 1 of every row, copied with a small offset), and
decode must equal the input for every segment size."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(O, W, H, seed):
    rng = np.random.default_rng(seed)
    px = O.gen_syn_v1(W, H, 3, 7 + seed).reshape(H, W, 3).copy()
    for y in range(H):
        c = rng.integers(0, 256, 3)
        px[y, 0] = c
        px[y, 1] = (c + [1, 2, 3]) % 256
        px[y, W - 3] = (c + [5, 7, 3]) % 256
        px[y, W - 2] = (px[y, 1].astype(int) + [9, 4, 2]) % 256
    return px.reshape(-1)


@pytest.mark.parametrize("seg", ["16", "8"])
@pytest.mark.parametrize("W", [1601, 1602, 1600, 1615])
def test_wrap_to_current_row(nice, O, W, seg, opts):
    opts.setenv("NICE_DEC_SEG", seg)
    opts.setenv("NICE_DEC_SPLIT", "0")
    H = 48
    px = _frame(O, W, H, 0)
    s = O.encode(px, W, H, 3)
    ref, _ = O.decode(s)
    assert np.array_equal(ref[:W * H * 3], px)   # the oracle round trip (fixture sanity)
    got, _ = nice.decode_bytes(s, flags=nice.DEC_TOLERANT_HEADER)
    g = np.frombuffer(got, np.uint8)
    assert np.array_equal(g[:W * H * 3], px), (W, seg)
