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
NICE_DEC_FLOW=0)."""
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


@pytest.mark.parametrize("W", [64, 66, 1025, 1026, 1040, 1921, 2050, 3073, 3840, 4096])
def test_flow_widths(nice, O, W, monkeypatch):
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
            monkeypatch.setenv("NICE_DEC_FLOW", k)
            assert np.array_equal(_decode(nice, s, C), rgb), (W, C, k)


def test_flow_batch(nice, O, monkeypatch):
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
        monkeypatch.setenv("NICE_DEC_FLOW", k)
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
