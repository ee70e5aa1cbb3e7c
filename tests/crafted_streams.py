"""Hand-built NICE2 streams (test input; no encoder involved).

The encoder never emits some things the reference decoder accepts: tables of
26-31 bits that are read only a few times, runs with trailing zero digits.
These streams are written directly from the format:
file header, ten table headers (5-bit max, 7-bit lengths, hfe.rs:97-103),
then prefix and payload symbols in the decoder's grammar (code.rs:576-671),
MSB first, canonical codes from the oracle's restatement of hfe.rs:255-296.

Every symbol sequence keeps the pixel grammar valid for the reference (no
reference before the image start, no LUMA2 on row 0, runs inside the image),
so whether the reference decoder finishes depends only on its bit reader:
`read_24bits_noclear` with a table of 26-31 bits wraps its u8 offset at some
alignments (bitreader.rs:85-98).  The oracle decides which streams do.
"""
import numpy as np

# stream sizes (code.rs:91-116) and the payload streams of each prefix
SIZES = [256, 13, 64, 32, 11, 343, 64, 32, 32, 11]
BR_OFF = lambda W: [1, W, W - 1, 2, 2 * W]
LUMA_OFF = lambda W: [1, W, W - 1, W - 3, 3, 3 * W - 1, 3 * W, 3 * W + 1, W + 3, 3 * W + 3, 3 * W - 3]
DEEP_STREAMS = [0, 2, 3, 5, 6, 7, 8]   # alphabets that can hold a 25-31 bit table


class _Bits:
    def __init__(self):
        self.bits = []

    def put(self, v, n):
        for k in range(n - 1, -1, -1):
            self.bits.append((v >> k) & 1)

    def tobytes(self):
        b = self.bits + [0] * (-len(self.bits) % 8)
        return np.packbits(np.array(b, np.uint8)).tobytes()


def _lengths(O, rng, n, deep_lo=None, deep_hi=None):
    """Code lengths from O.code_lengths of random counts; a deep table (max in
    [deep_lo, deep_hi]) from Fibonacci-skewed counts."""
    for _ in range(2000):
        if deep_lo is None:
            counts = rng.integers(1, 60, n).astype(np.uint64)
        else:
            # a Fibonacci chain of K small counts (depth K - 1) under a
            # balanced tree of the other symbols, all of them heavier
            K = int(rng.integers(max(2, deep_lo - 12), min(deep_hi, n) + 1))
            fib = [1, 1]
            while len(fib) < K + 2:
                fib.append(fib[-1] + fib[-2])
            counts = rng.integers(fib[K + 1], 2 * fib[K + 1], n).astype(np.uint64)
            idx = rng.permutation(n)[:K]
            counts[idx] = np.array(fib[:K], np.uint64)
        aob = O.code_lengths(counts)
        mx = int(aob.max())
        if deep_lo is None and mx <= 24:
            return aob
        if deep_lo is not None and deep_lo <= mx <= deep_hi:
            return aob
    raise RuntimeError("no table in range")


def make_stream(O, seed, W=None, H=None, deep=None, deep_lo=25, deep_hi=31, zero_digits=True):
    """One random stream.  Returns (bytes, info dict)."""
    rng = np.random.default_rng(seed)
    W = int(W if W is not None else rng.integers(4, 40))
    H = int(H if H is not None else rng.integers(1, 8))
    N = W * H
    if deep is None:
        deep = int(rng.choice(DEEP_STREAMS))
    lens = [_lengths(O, rng, n, deep_lo, deep_hi) if st == deep else _lengths(O, rng, n)
            for st, n in enumerate(SIZES)]
    codes = [O.canonical(l) for l in lens]
    b = _Bits()
    for st in range(10):
        b.put(int(lens[st].max()), 5)
        for v in lens[st]:
            b.put(int(v), 7)
    assert len(b.bits) == 6056

    def sym(st, v):
        b.put(int(codes[st][v]), int(lens[st][v]))

    # mode weights: how often the deep stream is read decides how likely a
    # wrapping read is, so both outcomes occur
    w = rng.random(5) ** 2
    i = 0
    while i < N:
        if i == 0:
            mode = 1   # RGB (predicts from pixel 0 itself, code.rs:640)
        else:
            mode = int(rng.choice(5, p=w / w.sum()))
            if mode == 4 and i < W:
                mode = 3
        if mode == 0:
            k = int(rng.choice([k for k, o in enumerate(BR_OFF(W)) if 0 < o <= i]))
            sym(1, 0); sym(9, k)
        elif mode == 1:
            sym(1, 1); sym(0, rng.integers(256)); sym(0, rng.integers(256)); sym(0, rng.integers(256))
        elif mode == 2:
            k = int(rng.choice([k for k, o in enumerate(LUMA_OFF(W)) if 0 < o <= i]))
            sym(1, 2); sym(4, k); sym(2, rng.integers(64)); sym(3, rng.integers(32)); sym(3, rng.integers(32))
        elif mode == 3:
            sym(1, 3); sym(5, rng.integers(343))
        else:
            sym(1, 4); sym(6, rng.integers(64)); sym(7, rng.integers(32)); sym(8, rng.integers(32))
        i += 1
        if i < N and rng.random() < 0.25:
            r = int(rng.integers(1, min(N - i, 80) + 1))
            m = r - 1
            while True:               # code.rs:393-405: digits m % 8, m /= 8
                sym(1, 5 + m % 8)
                if m < 8:
                    break
                m //= 8
            if zero_digits and rng.random() < 0.3:
                for _ in range(int(rng.integers(1, 3))):
                    sym(1, 5)         # a zero digit adds nothing (code.rs:668)
            i += r
    sym(1, int(rng.integers(5)))      # the extra prefix the reference reads (code.rs:660)
    hdr = b"nice" + W.to_bytes(4, "big") + H.to_bytes(4, "big") + bytes([3])
    tail = bytes(rng.integers(0, 256, int(rng.integers(0, 6)), dtype=np.uint8)) + bytes(5)
    info = {"W": W, "H": H, "deep": deep, "max": int(lens[deep].max())}
    return hdr + b.tobytes() + tail, info


def make_slow_sync(O, seed, W, H, every=20):
    """A stream whose Huffman parse re-synchronises only after thousands of
    bits (the Jacobi fixpoint of the slice-parallel parse then needs tens of
    iterations).  Every pixel is RGB with zero residuals except one pixel in
    about `every` (SMALL_DIFF, a random index): the prefix table gives RGB the
    1-bit code 0 and the RGB table is uniform (eight bits, code(0) = 0), so a
    zero pixel is 25 zero bits and a parse that starts at the wrong bit keeps
    reading 25-bit zero events at that offset; only the SMALL_DIFF pixels can
    move it, and each lands it on the true boundary with probability about
    1/25.  Returns the stream (header channels 3)."""
    rng = np.random.default_rng(seed)
    N = W * H
    lens = []
    for st, n in enumerate(SIZES):
        if st == 0:
            counts = np.full(n, 1000, np.uint64)              # uniform: every RGB code 8 bits
        elif st == 1:
            counts = rng.integers(1, 60, n).astype(np.uint64)
            counts[1] = 1 << 20                               # RGB prefix: 1 bit
        else:
            counts = rng.integers(1, 60, n).astype(np.uint64)
        lens.append(O.code_lengths(counts))
    codes = [O.canonical(l) for l in lens]
    assert int(lens[1][1]) == 1 and int(codes[1][1]) == 0
    assert (lens[0] == 8).all() and int(codes[0][0]) == 0
    head = _Bits()
    for st in range(10):
        head.put(int(lens[st].max()), 5)
        for v in lens[st]:
            head.put(int(v), 7)
    # events: 25 zero bits, or SMALL_DIFF (prefix 3, index) at the breakers
    brk = np.zeros(N, bool)
    brk[1:] = rng.random(N - 1) < 1.0 / every
    idx = rng.integers(0, 343, N)
    ev_len = np.where(brk, int(lens[1][3]) + lens[5][idx].astype(np.int64), 25)
    start = np.concatenate([[0], np.cumsum(ev_len)])
    extra = 0   # the extra prefix the reference reads after the last pixel (code.rs:660): RGB, '0'
    bits = np.zeros(int(start[-1]) + 1 + extra, np.uint8)
    pc, pl = int(codes[1][3]), int(lens[1][3])
    for i in np.nonzero(brk)[0]:
        v = (pc << int(lens[5][idx[i]])) | int(codes[5][idx[i]])
        n = pl + int(lens[5][idx[i]])
        b0 = int(start[i])
        bits[b0:b0 + n] = [(v >> (n - 1 - k)) & 1 for k in range(n)]
    allbits = np.concatenate([np.array(head.bits, np.uint8), bits])
    allbits = np.concatenate([allbits, np.zeros(-len(allbits) % 8, np.uint8)])
    hdr = b"nice" + W.to_bytes(4, "big") + H.to_bytes(4, "big") + bytes([3])
    s = hdr + np.packbits(allbits).tobytes() + bytes(5)
    return s
