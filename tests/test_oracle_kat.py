"""The CPU oracle against the reference's own known-answer tests.

bitwriter.rs:86-97, bitreader.rs:106-146 and hfe.rs:300-348 are ported here
literally; SURVEY.md Appendix C values (an independent restatement made during
the survey) cross-check whole streams.
"""
import numpy as np
import pytest


def test_bitwriter_kat(O):
    # bitwriter.rs:89-97: write_8bits(2,3) x3, write_8bits(2,0) -> 0b1111_1100
    assert O.kat_writer()[0] == 0b1111_1100


def test_bitreader_kat(O):
    # bitreader.rs:106-118
    assert O.kat_reader(bytes([252] * 6), [0, 0, 0, 0], [2, 2, 2, 2]) == [3, 3, 3, 0]


def test_bitreader24_kat(O):
    # bitreader.rs:133-146: read_24bits / read_24bits_noclear with 9 bits
    got = O.kat_reader(bytes([252] * 6), [1, 2, 1, 1], [9, 9, 9, 9])
    assert got == [0b111111001, 0b111110011, 0b111110011, 0b111100111]


def test_hfe_roundtrip_kat(O):
    # hfe.rs:300-348: 256 symbols with counts i*10 round-trip through the entropy coder
    rc, n, mx = O.kat_hfe()
    assert rc == 0
    assert (n, mx) == (316310, 15)


@pytest.mark.parametrize("n,expect", [(256, 71), (343, 88), (64, 23), (32, 13), (13, 6), (11, 5)])
def test_all_zero_tree_depth(O, n, expect):
    # BinaryHeap tie-breaking on all-zero counts
    assert int(O.code_lengths([0] * n).max()) == expect


def test_code_lengths_kraft(O):
    rng = np.random.default_rng(5)
    for n in (11, 13, 32, 64, 256, 343):
        counts = rng.integers(0, 1000, size=n)
        counts[rng.random(n) < 0.3] = 0
        aob = O.code_lengths(counts).astype(np.int64)
        assert abs(sum(2.0 ** -a for a in aob) - 1.0) < 1e-12
        codes = O.canonical(aob)
        # prefix-free (usize arithmetic makes codes of >= 64 bits meaningless,
        # hfe.rs:285; such lengths only occur for zero-count symbols)
        words = sorted(format(int(c), "0%db" % a) for c, a in zip(codes, aob) if a < 64)
        for a, b in zip(words, words[1:]):
            assert not b.startswith(a)


@pytest.mark.parametrize("w,h,c,size,maxaob", [
    (256, 256, 3, 95641, None),
    (512, 512, 4, 375493, None),
    (1920, 1080, 4, 2816649, [9, 10, 9, 5, 5, 12, 11, 7, 7, 8]),
])
def test_syn_v1_sizes(O, w, h, c, size, maxaob):
    px = O.gen_syn_v1(w, h, c, 1)
    s, st = O.encode(px, w, h, c, with_stats=True)
    assert len(s) == size
    if maxaob is not None:
        assert list(st.max_aob) == maxaob


def test_gradient_512(O):
    g = O.gen_gradient(512, 512, 4)
    s, st = O.encode(g, 512, 512, 4, with_stats=True)
    assert len(s) == 97318
    assert list(st.max_aob) == [73, 10, 25, 15, 7, 109, 23, 13, 13, 7]
    with pytest.raises(RuntimeError):      # the reference decoder fails on it
        s3 = bytearray(s); s3[12] = 3
        O.decode(bytes(s3))


def test_rgba_stream_equals_rgb_stream(O):
    px4 = O.gen_syn_v1(96, 64, 4, 7)
    px3 = px4.reshape(-1, 4)[:, :3].copy()
    s4 = O.encode(px4, 96, 64, 4)
    s3 = O.encode(px3, 96, 64, 3)
    assert s4[:12] == s3[:12] and s4[12] == 4 and s3[12] == 3 and s4[13:] == s3[13:]


def test_reference_decoder_fails_rgba(O):
    px4 = O.gen_syn_v1(64, 64, 4, 2)
    with pytest.raises(RuntimeError):
        O.decode(O.encode(px4, 64, 64, 4))


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_oracle_roundtrip_rgb(O, seed):
    px = O.gen_syn_v1(160, 120, 3, seed)
    s = O.encode(px, 160, 120, 3)
    d, (w, h, ch) = O.decode(s, O.DEC_STRIDE)
    assert (w, h, ch) == (160, 120, 3) and np.array_equal(d, px)
    try:
        d2, _ = O.decode(s)                 # literal reference semantics
        assert np.array_equal(d2, px)
    except O.OracleDecodeError as e:
        # seed 4: a 27-bit max code length makes the reference refill loop wrap
        # its u8 bit offset (bitreader.rs:88-97) and spin forever
        assert e.rc == O.E_HANG and seed == 4


def test_reference_hang_domain(O):
    px = O.gen_syn_v1(160, 120, 3, 4)
    s, st = O.encode(px, 160, 120, 3, with_stats=True)
    assert max(st.max_aob) > 24
    with pytest.raises(O.OracleDecodeError) as ei:
        O.decode(s)
    assert ei.value.rc == O.E_HANG
