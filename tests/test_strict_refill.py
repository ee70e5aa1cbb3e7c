"""Strict mode against the reference's bit reader (bitreader.rs:78-100).

`read_24bits_noclear(max)` refills byte by byte while its u8 bit offset is
above 32 - max; for tables of 26-31 bits the loop can step the offset below
zero, wrap, and never end.  Whether it does depends on each read's bit
alignment and on how many bytes earlier reads already pulled in, so it is a
property of the whole symbol sequence.  The GPU strict mode
(`dec_strict_refill`) must fail on exactly the streams where the oracle's
literal reader hangs, and decode the others to the reference's pixels.

The streams are hand-built (tests/crafted_streams.py): random tables with one
25-31 bit stream, random grammar-valid pixel events, runs with trailing zero
digits (which the reference's run loop reads and the encoder never writes).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import crafted_streams as C

SEEDS = range(160)


def _outcomes(O, s):
    try:
        ref = O.decode(s)[0]
    except O.OracleDecodeError as e:
        ref = e
    try:
        intent = O.decode(s, O.DEC_STRIDE)[0]
    except O.OracleDecodeError as e:
        intent = e
    return ref, intent


def test_crafted_streams_cover_both_outcomes(O):
    """The corpus holds 26-31 bit tables the reference reads to the end and
    ones on which it hangs; 25-bit tables never hang; the intent decoder reads
    every stream."""
    kinds = {"ok26": 0, "hang": 0, "ok25": 0}
    for seed in SEEDS:
        s, info = C.make_stream(O, seed)
        ref, intent = _outcomes(O, s)
        assert not isinstance(intent, Exception), (seed, intent)
        if isinstance(ref, Exception):
            assert ref.rc == -5 and info["max"] >= 26, (seed, info, ref)
            kinds["hang"] += 1
        else:
            assert np.array_equal(ref, intent)
            kinds["ok26" if info["max"] >= 26 else "ok25"] += 1
    assert min(kinds.values()) >= 10, kinds


def test_oracle_lazy_lut_equals_literal(O, tmp_path):
    """The oracle keeps tables over 20 bits as code intervals instead of the
    reference's 2^max array (hfe.rs:191-202): a build with every table lazy
    decodes the same corpus (and SYN-v1 streams) to the same result."""
    so = tmp_path / "liboracle_lazy.so"
    src = os.path.join(os.path.dirname(O.__file__), "nice_oracle.c")
    subprocess.run(["gcc", "-O2", "-fPIC", "-std=c11", "-shared", "-DLUT_LAZY_BITS=3", "-o", str(so), src],
                   check=True)
    streams = [C.make_stream(O, seed, deep_lo=12, deep_hi=20)[0] for seed in range(40)]
    streams += [O.encode(O.gen_syn_v1(w, h, 3, sd), w, h, 3) for w, h, sd in [(333, 211, 3), (256, 64, 8)]]

    def run():
        out = []
        for s in streams:
            for mode in (O.DEC_REFERENCE, O.DEC_STRIDE):
                try:
                    out.append(O.decode(s, mode)[0].tobytes())
                except O.OracleDecodeError as e:
                    out.append(e.rc)
        return out

    a = run()
    orig = O.lib
    lazy = ctypes.CDLL(str(so))
    try:
        O.lib = lambda: lazy
        b = run()
    finally:
        O.lib = orig
    assert a == b


@pytest.mark.gpu
def test_strict_matches_reference_reader(nice, O):
    """GPU strict mode == the literal reference decode on every crafted stream
    (fail where it hangs, its pixels where it finishes); the default mode ==
    the intent decode."""
    for seed in SEEDS:
        s, info = C.make_stream(O, seed)
        ref, intent = _outcomes(O, s)
        try:
            got = np.frombuffer(nice.decode_bytes(s, flags=nice.DEC_STRICT_REFERENCE)[0], np.uint8)
        except nice.NiceError as e:
            got = e
        if isinstance(ref, Exception):
            assert isinstance(got, Exception), (seed, info)
        else:
            assert not isinstance(got, Exception), (seed, info, got)
            assert np.array_equal(got, ref), (seed, info)
        dflt = np.frombuffer(nice.decode_bytes(s)[0], np.uint8)
        assert np.array_equal(dflt, intent), (seed, info)
