"""Device Huffman code lengths (enc_tables' wave-parallel BinaryHeap replay,
nice_huffman.hpp) against the oracle's literal replay of hfe.rs:58-87 + std
BinaryHeap on random count vectors -- tie-heavy, sparse and wide counts, every
stream size of the format (code.rs:91-116) plus tiny heaps.  Count totals
reach 3 * 2^30, the largest a frame can produce (the boundary caps frames at
2^30 pixels, at most 3 symbols per pixel per stream): the device heap keys
hold 32-bit counts and 32-bit merge sums, so totals in 2^31 .. 3 * 2^30 (where
a signed or narrowing slip would show) are covered explicitly."""
import ctypes

import numpy as np
import pytest

SIZES = [256, 13, 64, 32, 11, 343, 64, 32, 32, 11, 3, 2, 1]


TOTAL_MAX = 3 << 30   # SC_RGB at the 2^30-pixel frame cap


def _big_total(c, rng):
    """Scales c so its total lands in [2^31, 3 * 2^30] (at most TOTAL_MAX)."""
    c = c.astype(np.float64)
    s = c.sum()
    if s == 0:
        c[0], s = 1.0, 1.0
    target = rng.integers(1 << 31, TOTAL_MAX + 1)
    c = np.floor(c * (target / s))
    return np.minimum(c, TOTAL_MAX).astype(np.uint64)


def _vectors(n, k, rng):
    out = []
    for m in range(k):
        mode = m % 9
        if mode == 0:
            c = rng.integers(0, 4, n)
        elif mode == 1:
            c = rng.integers(0, 50, n)
        elif mode == 2:
            c = np.where(rng.integers(0, 3, n) == 0, 0, rng.integers(0, 100000, n))
        elif mode == 3:
            c = np.where(rng.integers(0, 2, n) == 0, 5, 7)
        elif mode == 4:   # wide counts; a stream total below 2^31
            c = rng.integers(0, (1 << 31) // n, n)
        elif mode == 5:   # Fibonacci-like: deep trees
            f = [1, 1]
            while len(f) < n:
                f.append(min(f[-1] + f[-2], (1 << 31) // n))
            c = np.array(f[:n])[rng.permutation(n)]
        elif mode == 6:   # wide counts, total in 2^31 .. 3 * 2^30
            c = _big_total(rng.integers(0, 1 << 20, n), rng)
        elif mode == 7:   # Fibonacci-like, total in 2^31 .. 3 * 2^30
            f = [1, 1]
            while len(f) < n:
                f.append(f[-1] + f[-2])
            c = _big_total(np.array(f[:n], dtype=np.float64)[rng.permutation(n)], rng)
        else:   # one dominant symbol: merges near the full total, ties among the rest
            c = rng.integers(0, 3, n).astype(np.uint64)
            c[rng.integers(0, n)] = TOTAL_MAX - int(c.sum())
        assert int(c.sum()) <= TOTAL_MAX
        out.append(c.astype(np.uint32))
    return np.stack(out)


def test_vectors_cover_large_totals():
    """The generator itself (no GPU): the large-total modes reach 2^31+."""
    rng = np.random.default_rng(0)
    for n in (2, 11, 343):
        tot = _vectors(n, 18, rng).astype(np.uint64).sum(axis=1)
        assert tot.max() <= TOTAL_MAX
        assert (tot >= (1 << 31)).sum() >= 4


@pytest.mark.gpu
@pytest.mark.parametrize("n", sorted(set(SIZES)))
def test_device_code_lengths_match_oracle(nice, O, n):
    rng = np.random.default_rng(n)
    k = 600
    counts = _vectors(n, k, rng)
    aob = np.zeros((k, n), dtype=np.uint8)
    L = nice.lib()
    L.nice_test_code_lengths.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    rc = L.nice_test_code_lengths(counts.ctypes.data, k, n, aob.ctypes.data)
    assert rc == 0
    for v in range(k):
        ref = O.code_lengths(counts[v].astype(np.uint64))
        assert np.array_equal(aob[v], ref), (n, v, counts[v][:16])
