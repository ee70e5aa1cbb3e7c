"""Strip-split row reconstruction (dec_rows_split): one wide frame decoded by
several workgroups on separate CUs, each owning a strip of row segments and
exchanging its first / last three pixels per row (the raster wrap of
code.rs:412-413 and the +-3-pixel references of code.rs:141-145 cross strip
edges).  Pixels must equal the oracle's decode for every strip count, partial
last segments (W % 16 = 1, 2), long runs and reference chains crossing strips,
RGB and RGBA; a corrupted stream must fail with a status, not hang.
NICE_DEC_SPLIT=k forces k strips on frames narrow enough for one workgroup."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cases(O):
    rng = np.random.default_rng(77)
    cases = [
        ("syn1000x40x3", O.gen_syn_v1(1000, 40, 3, 3), 1000, 40, 3),
        ("syn1601x30x4", O.gen_syn_v1(1601, 30, 4, 4), 1601, 30, 4),   # W % 16 == 1
        ("syn1058x25x3", O.gen_syn_v1(1058, 25, 3, 5), 1058, 25, 3),   # W % 16 == 2
        ("grad800x64x3", O.gen_gradient(800, 64, 3), 800, 64, 3),
    ]
    st = np.zeros((60, 900, 3), np.uint8)          # runs across strips and rows
    st[:, :, 0] = (np.arange(60)[:, None] // 7) * 20
    st[::5, ::3, 1] = 200
    cases.append(("stripes900x60x3", st.reshape(-1), 900, 60, 3))
    pal = np.array([[10, 20, 30], [10, 21, 31], [200, 100, 50], [12, 22, 29]], np.uint8)
    idx = rng.integers(0, 4, (50, 777))
    idx[:, 300:500] = 2
    cases.append(("palette777x50x3", pal[idx].reshape(-1), 777, 50, 3))
    return cases


def _check(nice, O, px, w, h, c):
    s = O.encode(px, w, h, c)
    got, img = nice.decode_bytes(s, flags=nice.DEC_ALPHA_FILL_FF | nice.DEC_TOLERANT_HEADER)
    g = np.frombuffer(got, np.uint8).reshape(-1, c)
    return np.array_equal(g[:, :3], px.reshape(-1, c)[:, :3])


@pytest.mark.parametrize("k", [2, 3, 5])
def test_split_forced_strips(nice, O, k, opts):
    opts.setenv("NICE_DEC_SPLIT", str(k))
    for name, px, w, h, c in _cases(O):
        assert _check(nice, O, px, w, h, c), (name, k)


def test_split_default_wide(nice, O, opts):
    """W > 4096 splits by default (ceil(W / 16 / 256) strips); =0 disables."""
    px = O.gen_syn_v1(8200, 9, 4, 8)
    assert _check(nice, O, px, 8200, 9, 4)
    opts.setenv("NICE_DEC_SPLIT", "0")
    assert _check(nice, O, px, 8200, 9, 4)


def test_split_batch_rgb_out(nice, O, opts):
    """A batch (several frames, each split) through the device API, RGBA
    streams decoded to 3-channel output."""
    import torch
    opts.setenv("NICE_DEC_SPLIT", "3")
    w, h, c, n = 1200, 20, 4, 5
    frames = [O.gen_syn_v1(w, h, c, 30 + i) for i in range(n)]
    streams = [O.encode(f, w, h, c) for f in frames]
    stride = (max(len(s) for s in streams) + 255) // 256 * 256
    sb = torch.zeros((n, stride), dtype=torch.uint8)
    for i, s in enumerate(streams):
        sb[i, :len(s)] = torch.frombuffer(bytearray(s), dtype=torch.uint8)
    sb = sb.cuda()
    lens = torch.tensor([len(s) for s in streams], dtype=torch.int64, device="cuda")
    dec = torch.zeros((n, w * h * 3), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    nice.decode_batch(sb, lens, w, h, 3, dec, status, flags=nice.DEC_TOLERANT_HEADER)
    torch.cuda.synchronize()
    assert status.cpu().tolist() == [0] * n
    for i in range(n):
        assert np.array_equal(dec[i].cpu().numpy(), frames[i].reshape(-1, 4)[:, :3].reshape(-1)), i


def test_split_corrupt_stream_fails_fast(nice, O, opts):
    """A stream whose records reference outside the image or mis-parse: the
    split decode reports an error (or decodes) without waiting on a strip that
    stopped -- it returns well inside the per-row poll timeout."""
    opts.setenv("NICE_DEC_SPLIT", "4")
    w, h, c = 1500, 30, 3
    px = O.gen_syn_v1(w, h, c, 12)
    s = bytearray(O.encode(px, w, h, c))
    rng = np.random.default_rng(5)
    for trial in range(6):
        t = bytearray(s)
        for pos in rng.integers(800, len(t), 8):
            t[pos] ^= 0xFF
        t0 = time.time()
        try:
            nice.decode_bytes(bytes(t), flags=nice.DEC_ALPHA_FILL_FF | nice.DEC_TOLERANT_HEADER)
        except nice.NiceError:
            pass
        assert time.time() - t0 < 3.0, trial
    assert _check(nice, O, px, w, h, c)   # the context still decodes afterwards


@pytest.mark.parametrize("seg", ["8", "16"])
def test_row_segment_sizes(nice, O, seg, opts):
    """dec_rows8 (8-pixel segments, on request since round 4) and dec_rows (16)
    forced on the same frames: identical pixels."""
    opts.setenv("NICE_DEC_SEG", seg)
    opts.setenv("NICE_DEC_SPLIT", "0")
    for name, px, w, h, c in _cases(O) + [("syn64x9x3", O.gen_syn_v1(64, 9, 3, 2), 64, 9, 3),
                                          ("syn2047x12x4", O.gen_syn_v1(2047, 12, 4, 3), 2047, 12, 4)]:
        assert _check(nice, O, px, w, h, c), (name, seg)


def _split_stats(nice, ctx):
    import ctypes
    L = nice.lib()
    L.nice_test_split_redos.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32)]
    nf, nr = ctypes.c_uint32(), ctypes.c_uint32()
    assert L.nice_test_split_redos(ctx.ptr, ctypes.byref(nf), ctypes.byref(nr)) == 0
    return nf.value, nr.value


def _decode_dev(nice, O, px, w, h, c, ctx, stream=None, stream_bytes=None):
    import torch
    s = stream_bytes if stream_bytes is not None else O.encode(px, w, h, c)
    sb = torch.zeros((1, (len(s) + 255) // 256 * 256), dtype=torch.uint8)
    sb[0, :len(s)] = torch.frombuffer(bytearray(s), dtype=torch.uint8)
    sb = sb.cuda()
    lens = torch.tensor([len(s)], dtype=torch.int64, device="cuda")
    dec = torch.zeros((1, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    if stream is not None:   # the inputs are ready before `stream` runs (no device-wide sync)
        stream.wait_stream(torch.cuda.current_stream())
    nice.decode_batch(sb, lens, w, h, 4, dec, status, flags=nice.DEC_ALPHA_FILL_FF | nice.DEC_TOLERANT_HEADER,
                      stream=stream, ctx=ctx)
    return dec, status


def test_split_wider_than_16384(nice, O):
    """W > 16384 (one workgroup cannot hold a row's segments) decodes through
    the strip split too (was: the 64-lane dec_reconstruct)."""
    import torch
    w, h, c = 20000, 48, 4
    px = O.gen_syn_v1(w, h, c, 21)
    ctx = nice.Context(0)
    dec, status = _decode_dev(nice, O, px, w, h, c, ctx)
    torch.cuda.synchronize()
    assert int(status[0]) == 0
    assert np.array_equal(dec[0].view(-1, 4)[:, :3].cpu().numpy(), px.reshape(-1, 4)[:, :3])
    nf, nr = _split_stats(nice, ctx)
    assert nf == 1 and nr == 0


def test_split_not_coresident_falls_back(nice, O):
    """A 16384-wide decode queued while another stream's kernel holds every CU
    but one for 1.5 s: exact pixels, status 0, no NICE_E_HIP.  Workgroups go
    to the XCDs round-robin, so strips on XCDs with no free CU (and blocks of
    the parse kernels) start only when the occupying blocks end; whether the
    split then ran co-resident or a strip timed out and its frame was redone
    depends on that order -- both must give the same pixels."""
    import ctypes
    import torch
    w, h, c = 16384, 64, 4
    px = O.gen_syn_v1(w, h, c, 22)
    s = O.encode(px, w, h, c)
    ctx = nice.Context(0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    L = nice.lib()
    L.nice_test_occupy.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 5
    busy = torch.cuda.Stream()
    work = torch.cuda.Stream()
    sb = torch.zeros((1, (len(s) + 255) // 256 * 256), dtype=torch.uint8)
    sb[0, :len(s)] = torch.frombuffer(bytearray(s), dtype=torch.uint8)
    sb = sb.cuda()
    lens = torch.tensor([len(s)], dtype=torch.int64, device="cuda")
    dec = torch.zeros((1, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    flags = nice.DEC_ALPHA_FILL_FF | nice.DEC_TOLERANT_HEADER
    # first decode: sizes the context's scratch (no allocation -- which could
    # synchronise the device -- in the timed one)
    nice.decode_batch(sb, lens, w, h, 4, dec, status, flags=flags, stream=work, ctx=ctx)
    torch.cuda.synchronize()
    assert int(status[0]) == 0 and _split_stats(nice, ctx) == (1, 0)
    dec.zero_()
    torch.cuda.synchronize()
    # one block per CU (96 KB of LDS each: no 82 KB strip block fits beside it);
    # one CU frees after 20 ms, the rest after 1.5 s
    assert L.nice_test_occupy(ctypes.c_void_p(busy.cuda_stream), cus, 1, 20000, 1500000, 96 * 1024) == 0
    t0 = time.time()
    nice.decode_batch(sb, lens, w, h, 4, dec, status, flags=flags, stream=work, ctx=ctx)
    work.synchronize()
    dt = time.time() - t0
    torch.cuda.synchronize()
    assert int(status[0]) == 0
    assert np.array_equal(dec[0].view(-1, 4)[:, :3].cpu().numpy(), px.reshape(-1, 4)[:, :3])
    nf, nr = _split_stats(nice, ctx)
    print(f"decode beside the occupying kernel: {dt:.2f} s, frames redone: {nr}")
    assert nf == 1 and nr in (0, 1)


@pytest.mark.parametrize("shape", [(16384, 64, 4), (20000, 24, 3)], ids=["16384x64x4", "20000x24x3"])
def test_split_absent_strip_redone(nice, O, shape, opts):
    """A strip that never becomes resident (test hook split_absent: the last
    strip of each frame returns at entry): its neighbour's halo wait times out
    (0.2 s), the frame's strips stop, and the fallback launch (dec_rows_wide;
    dec_reconstruct above 16384 columns) reconstructs the frame exactly."""
    import torch
    from conftest import set_hooks
    w, h, c = shape
    px = O.gen_syn_v1(w, h, c, 23)
    ctx = nice.Context(0)
    set_hooks(nice, ctx, split_absent=1)
    t0 = time.time()
    dec, status = _decode_dev(nice, O, px, w, h, c, ctx)
    torch.cuda.synchronize()
    dt = time.time() - t0
    assert int(status[0]) == 0
    assert np.array_equal(dec[0].view(-1, 4)[:, :3].cpu().numpy(), px.reshape(-1, c)[:, :3])
    assert _split_stats(nice, ctx) == (1, 1)
    assert dt < 5.0, dt
