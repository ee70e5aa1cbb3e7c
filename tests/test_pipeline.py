"""Streamed host pipeline (BASELINE config 5): host
frames -> H2D -> encode -> D2H streams, and back, overlapped over HIP streams.
Parity: every stream equals the oracle's code::encode output byte for byte, and
every decoded frame equals the input, for pinned and pageable host buffers,
ragged last chunks and depth 1..3."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(O, n, w, h, c, seed0=1):
    return [O.gen_syn_v1(w, h, c, seed0 + i) for i in range(n)]


@pytest.mark.parametrize("batch,depth", [(3, 2), (4, 1), (2, 3), (16, 3)])
def test_pipe_encode_decode_pageable(nice, O, batch, depth):
    w, h, c, n = 160, 96, 4, 7
    frames = _frames(O, n, w, h, c)
    p = nice.Pipeline(w, h, c, batch=batch, depth=depth)
    outs = [np.zeros(p.stream_stride, np.uint8) for _ in range(n)]
    lens = p.encode(frames, outs)
    for i in range(n):
        assert outs[i][:lens[i]].tobytes() == O.encode(frames[i], w, h, c), i
    dec = [np.zeros(w * h * c, np.uint8) for _ in range(n)]
    st = p.decode(outs, lens, dec)
    assert st == [0] * n
    for i in range(n):
        assert np.array_equal(dec[i].reshape(-1, c)[:, :3], frames[i].reshape(-1, c)[:, :3]), i
        assert (dec[i].reshape(-1, c)[:, 3] == 255).all()
    p.close()


def test_pipe_pinned_rgb(nice, O):
    import torch
    w, h, c, n = 333, 77, 3, 9
    frames = _frames(O, n, w, h, c, seed0=20)
    p = nice.Pipeline(w, h, c, batch=4, depth=3)
    src = [torch.from_numpy(f).pin_memory() for f in frames]
    outs = [torch.zeros(p.stream_stride, dtype=torch.uint8).pin_memory() for _ in range(n)]
    lens = p.encode(src, outs)
    for i in range(n):
        assert outs[i][:lens[i]].numpy().tobytes() == O.encode(frames[i], w, h, c), i
    dec = [torch.zeros(w * h * c, dtype=torch.uint8).pin_memory() for _ in range(n)]
    assert p.decode(outs, lens, dec) == [0] * n
    for i in range(n):
        assert np.array_equal(dec[i].numpy(), frames[i]), i


def test_pipe_bad_stream_status(nice, O):
    w, h, c = 160, 120, 3
    f = O.gen_syn_v1(w, h, c, 3)
    p = nice.Pipeline(w, h, c, batch=2, depth=2)
    good = np.frombuffer(O.encode(f, w, h, c), np.uint8).copy()
    bad = good.copy()
    bad[4:8] = [0, 0, 0, 9]            # wrong width for this pipe
    outs = [np.zeros(w * h * c, np.uint8) for _ in range(2)]
    with pytest.raises(nice.NiceError):
        p.decode([good, bad], [good.size, bad.size], outs)
    assert np.array_equal(outs[0], f)


def test_pipe_decode_unsettled_chunks_redone(nice, O, opts):
    """One queued sync iteration per chunk: the parse of long slices has not
    settled after it, so the device settle (dec_sync_settle: a sequential parse
    of the frames still changing) and the iteration behind it must give the
    fixpoint -- exact pixels, no host check."""
    opts.setenv("NICE_DEC_SYNC_QUEUED", "1")
    w, h, c, n = 640, 480, 4, 9
    frames = _frames(O, n, w, h, c, seed0=40)
    p = nice.Pipeline(w, h, c, batch=2, depth=2)
    outs = [np.zeros(p.stream_stride, np.uint8) for _ in range(n)]
    lens = p.encode(frames, outs)
    dec = [np.zeros(w * h * c, np.uint8) for _ in range(n)]
    assert p.decode(outs, lens, dec) == [0] * n
    for i in range(n):
        assert np.array_equal(dec[i].reshape(-1, c)[:, :3], frames[i].reshape(-1, c)[:, :3]), i
    p.close()


def test_pipe_decode_unsettled_with_bad_stream(nice, O, opts):
    """The settle path with an error in a settled chunk: every good frame
    exact, the bad frame's status an error (its pixels are undefined, nice.h)."""
    opts.setenv("NICE_DEC_SYNC_QUEUED", "1")
    w, h, c, n = 640, 480, 4, 5
    frames = _frames(O, n, w, h, c, seed0=60)
    p = nice.Pipeline(w, h, c, batch=2, depth=2)
    outs = [np.zeros(p.stream_stride, np.uint8) for _ in range(n)]
    lens = list(p.encode(frames, outs))
    outs[3] = outs[3].copy()
    outs[3][lens[3] // 2:lens[3]] ^= 0x5A          # corrupt the second half of frame 3's data
    dec = [np.zeros(w * h * c, np.uint8) for _ in range(n)]
    st = p.decode(outs, lens, dec, raise_on_error=False)
    assert st[3] != 0
    for i in (0, 1, 2, 4):
        assert st[i] == 0, (i, st)
        assert np.array_equal(dec[i].reshape(-1, c)[:, :3], frames[i].reshape(-1, c)[:, :3]), i
    p.close()


@pytest.mark.parametrize("c", [3, 4])
def test_pipe_checksums(nice, O, c):
    """nice_pipe_set_checksums: the device checksum of every stream and every
    decoded frame equals checksum64 of the bytes the pipe hands back (RGB frames
    of odd size: unaligned device frames), while the host buffers are reused."""
    w, h, n = 333, 77, 9
    frames = _frames(O, n, w, h, c, seed0=70)
    p = nice.Pipeline(w, h, c, batch=2, depth=2)
    outs = [np.zeros(p.stream_stride, np.uint8) for _ in range(n)]
    p.checksums(True)
    lens = p.encode(frames, outs)
    sums = p.last_sums
    for i in range(n):
        assert sums[i] == nice.checksum64(O.encode(frames[i], w, h, c)), i
    dec = [np.zeros(w * h * c, np.uint8) for _ in range(n)]
    assert p.decode(outs, lens, dec) == [0] * n
    for i in range(n):
        assert p.last_sums[i] == nice.checksum64(dec[i]), i
    p.close()
