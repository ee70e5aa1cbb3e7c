"""Committed golden fixtures (tests/golden/, made by make_golden.py): the oracle
must still produce them (CPU), and the HIP codec must produce / invert them
through the C ABI (GPU)."""
import json
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(HERE, "manifest.json")))["cases"]
IDS = [c["name"] for c in MANIFEST]


def _load(case):
    px = np.fromfile(os.path.join(HERE, case["name"] + ".in"), dtype=np.uint8)
    s = open(os.path.join(HERE, case["name"] + ".nice"), "rb").read()
    return px, s


def _rgb(px, c):
    return px.reshape(-1, c)[:, :3].reshape(-1) if px.size else px


@pytest.mark.parametrize("case", MANIFEST, ids=IDS)
def test_oracle_reproduces_golden(O, case):
    px, s = _load(case)
    w, h, c = case["width"], case["height"], case["channels"]
    assert len(s) == case["nice_len"]
    assert O.encode(px, w, h, c) == s
    if not case["decodable"]:
        assert max(case["max_code_len"]) > 31          # header spill: nobody can decode it
        with pytest.raises(O.OracleDecodeError):
            O.decode(s, O.DEC_STRIDE)
        return
    got, (gw, gh, gc) = O.decode(s, O.DEC_STRIDE)
    assert (gw, gh, gc) == (w, h, c)
    assert np.array_equal(_rgb(got, c), _rgb(px, c))
    if case["ref_decodable"]:
        ref, _ = O.decode(s, O.DEC_REFERENCE)
        assert np.array_equal(ref, got)


@pytest.mark.gpu
@pytest.mark.parametrize("case", MANIFEST, ids=IDS)
def test_hip_golden(nice, case):
    px, s = _load(case)
    w, h, c = case["width"], case["height"], case["channels"]
    assert nice.encode_bytes(px, w, h, c) == s
    if not case["decodable"]:
        with pytest.raises(nice.NiceError):
            nice.decode_bytes(s)
        return
    got, img = nice.decode_bytes(s)
    assert (img.width, img.height, img.channels) == (w, h, c)
    got = np.frombuffer(got, np.uint8)
    assert np.array_equal(_rgb(got, c), _rgb(px, c))
    if case["ref_decodable"]:
        strict, _ = nice.decode_bytes(s, nice.DEC_STRICT_REFERENCE)
        assert strict == bytes(got)
    elif case["channels"] == 3:
        with pytest.raises(nice.NiceError):
            nice.decode_bytes(s, nice.DEC_STRICT_REFERENCE)
