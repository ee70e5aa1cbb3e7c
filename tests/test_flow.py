"""The dataflow row kernel (dec_rows_flow, small batches) against the oracle.

Rows overlap in groups of waves that synchronise through LDS stamps: wave w of
row y waits for waves w-1..w+1 of row y-1 (references reach +-3 pixels, rows
1..3 back, code.rs:141-145), wave 0 for all of row y-1 (its entry is the
previous row's last pixel, code.rs:412-413), the last wave also for row y-1's
wave 0 (halos) and for row y's first pixels (W_CUR).  Widths that put one,
two, three and four waves on a row, partial last segments and waves
(W % 16 in {1, 2}: column W-3 in the second-to-last segment, which can sit in
the previous wave), every row-group count the kernel takes, and a batch of
frames: the pixels must equal the input, as with the barrier kernel (dec_rows,
NICE_DEC_FLOW=0).  Round 6: rows of 4097..8192 pixels (5..8 waves, one row
group, 4-row ring) take this kernel too instead of the strip split."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(O, W, H, C, seed):
    """SYN-v1 with, on every row, a pixel at column W-3 that only luma
    reference 3 (offset W-3: pixel 0 of the same row) predicts."""
    rng = np.random.default_rng(seed)
    px = O.gen_syn_v1(W, H, C, seed).reshape(H, W, C).copy()
    for y in range(H):
        c = rng.integers(0, 256, 3)
        px[y, 0, :3] = c
        px[y, 1, :3] = (c + [1, 2, 3]) % 256
        px[y, W - 3, :3] = (c + [5, 7, 3]) % 256
    return px.reshape(-1)


def _decode(nice, s, C):
    got, _ = nice.decode_bytes(s, flags=nice.DEC_TOLERANT_HEADER | nice.DEC_ALPHA_FILL_FF)
    return np.frombuffer(got, np.uint8).reshape(-1, C)[:, :3].reshape(-1)


@pytest.mark.parametrize("W", [64, 66, 1025, 1026, 1040, 1921, 2050, 3073, 3840, 4096,
                               4097, 5000, 6145, 7680, 8192])   # round 6: up to 8 waves per row
def test_flow_widths(nice, O, W, opts):
    H = 40
    for C in (3, 4):
        px = _frame(O, W, H, C, W + C)
        s = O.encode(px, W, H, C)
        rgb = px.reshape(-1, C)[:, :3].reshape(-1)
        try:
            ref, _ = O.decode(s[:12] + bytes([3]) + s[13:], O.DEC_TOLERANT)
        except O.OracleDecodeError:
            continue   # tables outside the decodable domain (see test_width_sweep)
        assert np.array_equal(ref, rgb)
        for k in ("0", "1", "2", "3", "4"):
            opts.setenv("NICE_DEC_FLOW", k)
            assert np.array_equal(_decode(nice, s, C), rgb), (W, C, k)


def test_flow_batch(nice, O, opts):
    """Several frames in one call (one block per frame), RGBA in, RGB and RGBA out."""
    import torch
    W, H, n = 1920, 64, 6
    frames = [_frame(O, W, H, 4, 100 + i) for i in range(n)]
    streams = [O.encode(f, W, H, 4) for f in frames]
    stride = (max(len(s) for s in streams) + 255) // 256 * 256
    dev = torch.device("cuda", 0)
    st = torch.zeros((n, stride), dtype=torch.uint8)
    for i, s in enumerate(streams):
        st[i, :len(s)] = torch.from_numpy(np.frombuffer(s, np.uint8))
    st = st.to(dev)
    ln = torch.tensor([len(s) for s in streams], dtype=torch.int64, device=dev)
    for k in ("2", "0"):
        opts.setenv("NICE_DEC_FLOW", k)
        for oc in (3, 4):
            out = torch.zeros((n, W * H * oc), dtype=torch.uint8, device=dev)
            status = torch.zeros(n, dtype=torch.int32, device=dev)
            nice.decode_batch(st, ln, W, H, oc, out, status)
            torch.cuda.synchronize()
            assert int(status.abs().sum()) == 0
            o = out.cpu().numpy()
            for i in range(n):
                got = o[i].reshape(-1, oc)[:, :3].reshape(-1)
                want = frames[i].reshape(-1, 4)[:, :3].reshape(-1)
                assert np.array_equal(got, want), (k, oc, i)


def test_flow_tall_ragged(nice, O, opts):
    """1283 x 719 (81 segments: a second wave of 17 lanes, W % 16 = 3; the shape
    tests/test_abi.py's C++ round trip uses) through both row-group counts.  A
    rejected round-5 variant of the kernel's waits (head stamps, never shipped)
    decoded this shape wrong (gpurun_out/r05za) while the narrower widths above
    passed; the shipped kernel must keep it exact."""
    W, H = 1283, 719
    for C in (3, 4):
        px = _frame(O, W, H, C, 7 + C)
        s = O.encode(px, W, H, C)
        rgb = px.reshape(-1, C)[:, :3].reshape(-1)
        for k in ("1", "2"):
            opts.setenv("NICE_DEC_FLOW", k)
            assert np.array_equal(_decode(nice, s, C), rgb), (C, k)


@pytest.mark.parametrize("k", ["1", "2"])
def test_flow_timeout_falls_back(nice, O, opts, k):
    """a wait that times out (0.2 s: the workgroup was preempted or
    time-sliced) sends the frame to the barrier kernel instead of failing it.
    NICE_TEST_FLOW_ABSENT makes the block's last wave return at entry, so the
    waves waiting on it time out; the frame must still decode exactly, status 0,
    and be counted as redone."""
    import ctypes
    import torch
    W, H = 1920, 48
    px = _frame(O, W, H, 4, 3)
    s = O.encode(px, W, H, 4)
    dev = torch.device("cuda", 0)
    st = torch.from_numpy(np.frombuffer(s + bytes(-len(s) % 256), np.uint8).copy()).view(1, -1).to(dev)
    ln = torch.tensor([len(s)], dtype=torch.int64, device=dev)
    out = torch.zeros((1, W * H * 4), dtype=torch.uint8, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    ctx = nice.Context(0)
    opts.setenv("NICE_DEC_FLOW", k)
    opts.setenv("NICE_TEST_FLOW_ABSENT", 1)
    nice.decode_batch(st, ln, W, H, 4, out, status, ctx=ctx)
    torch.cuda.synchronize()
    assert int(status[0]) == 0
    got = out[0].view(-1, 4)[:, :3].cpu().numpy().reshape(-1)
    assert np.array_equal(got, px.reshape(-1, 4)[:, :3].reshape(-1))
    L = nice.lib()
    L.nice_test_split_redos.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32)]
    nf, nr = ctypes.c_uint32(), ctypes.c_uint32()
    assert L.nice_test_split_redos(ctx.ptr, ctypes.byref(nf), ctypes.byref(nr)) == 0
    assert (nf.value, nr.value) == (1, 1)
