"""enc_classify_slide (round 6): RGBA frames with W <= 4095 and 16-byte aligned
pixel memory go through the per-lane sliding-window classify -- a lane owns 4
consecutive pixels and reads aligned row windows whose offsets depend on
W mod 4 (one kernel per residue), its coded flags go out in ballot order and
enc_rundigits transposes them.  Every stream must equal the oracle's and the
pair kernel's (NICE_ENC_NO_SLIDE): every W mod 4, the narrowest widths
(references wrapping across rows), the ring's widest rows, frames whose pixel
count is not a multiple of 4 (a lane's last pixels past the frame), batches
whose blocks cross frames, and deep-code (> 25-bit) frames."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PAIR, SLIDE = 5, 7


def _last(nice, ctx):
    L = nice.lib()
    L.nice_test_last_classify.argtypes = [ctypes.c_void_p]
    L.nice_test_last_classify.restype = ctypes.c_int
    return L.nice_test_last_classify(ctx.ptr)


def _encode(nice, frames, w, h, ctx):
    """frames: list of RGBA arrays; rows of a 16-byte aligned stride."""
    import torch
    n = len(frames)
    stride = (w * h * 4 + 15) // 16 * 16
    t = torch.zeros((n, stride), dtype=torch.uint8)
    for i, f in enumerate(frames):
        t[i, :w * h * 4] = torch.from_numpy(f)
    t = t.cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    nice.encode_batch(t, w, h, 4, out, lens, ctx=ctx)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    return [bytes(o[i, :int(lens[i])]) for i in range(n)]


def _check(nice, O, frames, w, h, opts):
    want = [O.encode(f, w, h, 4) for f in frames]
    ctx = nice.Context(0)
    got = _encode(nice, frames, w, h, ctx)
    assert _last(nice, ctx) == SLIDE
    for i in range(len(frames)):
        assert got[i] == want[i], (w, h, i, len(got[i]), len(want[i]))
    opts.setenv("NICE_ENC_NO_SLIDE", 1)
    got = _encode(nice, frames, w, h, ctx)
    assert _last(nice, ctx) == PAIR
    assert got == want
    opts.delenv("NICE_ENC_NO_SLIDE")


@pytest.mark.parametrize("w", [3, 4, 5, 6, 7, 8, 13, 61, 64, 65, 66, 67, 511, 1023, 1024, 1025, 1026, 2047,
                               3839, 3840, 4093, 4094, 4095])
def test_slide_widths(nice, O, w, opts):
    h = 37 if w < 1000 else 9
    frames = [O.gen_syn_v1(w, h, 4, w + 1), O.gen_rgb_field(w, h, 4, w + 2, (1, 3))]
    _check(nice, O, frames, w, h, opts)


def test_slide_batch_crossing_frames(nice, O, opts):
    """40 frames of 333 x 77 (25 641 pixels: 26 tiles, the last partial; N % 4
    = 1): the blocks' tile ranges cross frames and every frame ends mid-lane."""
    w, h = 333, 77
    frames = [O.gen_syn_v1(w, h, 4, 100 + i) for i in range(40)]
    _check(nice, O, frames, w, h, opts)


def test_slide_deep_codes(nice, O, opts):
    """Frames whose Huffman codes pass 25 bits (the long-code pack path)."""
    w, h = 512, 64
    frames = [O.gen_deep_codes(w, h, 4, seed=s) for s in (1, 2)]
    _check(nice, O, frames, w, h, opts)


def test_slide_4k(nice, O, opts):
    w, h = 3840, 2160
    _check(nice, O, [O.gen_syn_v1(w, h, 4, 1)], w, h, opts)
