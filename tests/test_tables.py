"""Device Huffman code lengths (enc_tables' wave-parallel BinaryHeap replay,
nice_huffman.hpp) against the oracle's literal replay of hfe.rs:58-87 + std
BinaryHeap on random count vectors -- tie-heavy, sparse and wide counts, every
stream size of the format (code.rs:91-116) plus tiny heaps.  Count totals
stay below 2^31, as a frame's do (the boundary caps frames at 2^30 pixels, at
most 3 symbols per pixel per stream), matching the device's 32-bit sums."""
import ctypes

import numpy as np
import pytest

SIZES = [256, 13, 64, 32, 11, 343, 64, 32, 32, 11, 3, 2, 1]


def _vectors(n, k, rng):
    out = []
    for m in range(k):
        mode = m % 6
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
        else:   # Fibonacci-like: deep trees
            f = [1, 1]
            while len(f) < n:
                f.append(min(f[-1] + f[-2], (1 << 31) // n))
            c = np.array(f[:n])[rng.permutation(n)]
        out.append(c.astype(np.uint32))
    return np.stack(out)


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
