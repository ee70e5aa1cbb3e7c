"""Host model of the row reconstructor's LDS ring addressing (dec_rows_body,
csrc/nice_decode.hip): the table-form pre-pass reads a reference of record
class c at word 4 + slot(y - rows_c) * RS + 17 * lane + d + (d >> 4),
d = p - px_c, with no wrap logic, because every emitted row also writes two
halos -- lane 0 its first three pixels past the end of the row above, the last
lane its last three pixels before the start of the next slot.  This replays
the kernel's stores for whole frames and checks that every reference the
reference codec can make (code.rs:141-145 offsets: rows 1..3 back, -3..3
pixels) reads the pixel the raster says, except the ones into the current row
(W_CUR, patched by the last lane).  CPU only: it pins the index arithmetic.
"""
import numpy as np
import pytest

# record classes 4..13 -> (rows back, pixels back), as cls_rows / cls_px
UP_CLASSES = {4: (1, 0), 5: (1, -1), 6: (2, 0), 7: (1, -3), 8: (3, -1), 9: (3, 0),
              10: (3, 1), 11: (1, 3), 12: (3, 3), 13: (3, -3)}
RB = 4


def g(x):
    return x + (x >> 4)   # Python >> on ints is arithmetic, as the kernel's int shift


def ring_stride(w):
    return w + (w >> 4) + 24


def replay(w, rows_to_emit, img):
    """Ring words after emitting rows 0..rows_to_emit-1 (value = pixel id + 1)."""
    rs = ring_stride(w)
    ring = np.zeros(4 * rs + RB, dtype=np.int64)
    nseg = (w + 15) // 16
    for y in range(rows_to_emit):
        base = RB + (y & 3) * rs
        for lane in range(nseg):
            x0 = 16 * lane
            nvalid = min(16, w - x0)
            for p in range(16):   # padding pixels (p >= nvalid) land in the spare words
                val = img[y, x0 + p] if p < nvalid else img[y, x0 + nvalid - 1]
                ring[base + x0 + (x0 >> 4) + p] = val
        if y > 0:   # lane 0: row y-1's right halo
            hb = RB + ((y - 1) & 3) * rs
            for k in range(3):
                ring[hb + g(w + k)] = img[y, k]
        nb = RB + ((y + 1) & 3) * rs   # last lane: row y+1's left halo
        for x in range(w - 3, w):
            ring[nb + (x - w) - 1] = img[y, x]
    return ring


@pytest.mark.parametrize("w", [64, 100, 1000, 3840])
def test_table_form_reads_match_raster(w):
    h = 9
    img = (np.arange(h * w, dtype=np.int64) + 1).reshape(h, w)
    rs = ring_stride(w)
    nseg = (w + 15) // 16
    for y in range(4, h):
        ring = replay(w, y, img)   # the ring as row y's pre-pass sees it
        checked = 0
        for c, (rows, px) in UP_CLASSES.items():
            dxp3 = px + 3
            off = ((y - rows) & 3) * rs + 3 - dxp3          # rtab[.][c].y
            for lane in range(nseg):
                lb = 17 * lane
                for p in range(min(16, w - 16 * lane)):
                    x = 16 * lane + p
                    ad = lb + off
                    if p < 3 or p > 12:
                        ad += (p + 3 - dxp3) >> 4             # padding word crossed
                    got = ring[RB + ad + p]
                    i = y * w + x - (rows * w + px)          # the raster reference
                    tx = x - px
                    if rows == 1 and tx >= w:                # into row y itself: W_CUR
                        assert lane == nseg - 1
                        continue
                    assert got == img.flat[i], (w, y, c, lane, p)
                    checked += 1
        assert checked > 0


def test_ring_fits_two_blocks_per_cu_at_4k():
    # dec_rows at 3840 columns: 256 lanes, tails + ring must leave two blocks per CU
    w, thr = 3840, 256
    lds = (thr * 7 + 8 + 4 * ring_stride(w)) * 4 + 384    # + static (class table, rtab)
    assert 2 * lds <= 160 * 1024
