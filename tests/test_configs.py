"""BASELINE.json configs 4 and 5 at their full workloads on one GPU.

Config 4: one 16384x16384 RGBA image encoded through the band C ABI in 8
bands (the split the 8-rank run uses; here one process, exchanges on the
host), byte-exact against the oracle's code::encode (code.rs:59-457), then
decoded back on the GPU.
Config 5: 48 x 3840x2160 RGBA frames streamed from pinned host memory through
the pipeline (H2D / kernels / D2H overlapped), every stream byte-exact against
the oracle, every frame decoded back exactly.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_config4_16k_band_encode_8_bands(nice, O):
    import torch
    from conftest import band_encode
    w, h, c = 16384, 16384, 4
    px = O.gen_syn_v1(w, h, c, 4)
    t = torch.from_numpy(px).cuda()
    got = band_encode(nice, t, w, h, c, 8)
    want = O.encode(px, w, h, c)
    assert got.numel() == len(want)
    g = got.cpu().numpy()
    wv = np.frombuffer(want, np.uint8)
    bad = np.flatnonzero(g != wv)
    assert bad.size == 0, f"first differing byte {bad[0]} of {len(want)}"
    del wv, g
    # decode on the GPU (one frame, the row kernel with its ring in global memory)
    dec = torch.empty(w * h * c, dtype=torch.uint8, device="cuda")
    lens = torch.tensor([got.numel()], dtype=torch.int64, device="cuda")
    sbuf = torch.zeros(1, (got.numel() + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
    sbuf[0, :got.numel()] = got
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    nice.decode_batch(sbuf, lens, w, h, c, dec.view(1, -1), status)
    torch.cuda.synchronize()
    assert int(status[0]) == 0
    assert torch.equal(dec.view(-1, 4)[:, :3], t.view(-1, 4)[:, :3])
    assert bool((dec.view(-1, 4)[:, 3] == 255).all())


def test_config5_streamed_48x4k(nice, O):
    import torch
    w, h, c, n = 3840, 2160, 4, 48
    frames = [O.gen_syn_v1(w, h, c, s) for s in range(1, n + 1)]
    p = nice.Pipeline(w, h, c, batch=16, depth=3)
    src = [torch.from_numpy(f).pin_memory() for f in frames]
    outs = [torch.zeros(p.stream_stride, dtype=torch.uint8).pin_memory() for _ in range(n)]
    lens = p.encode(src, outs)
    for i in range(n):
        assert outs[i][:lens[i]].numpy().tobytes() == O.encode(frames[i], w, h, c), i
    dec = [torch.zeros(w * h * c, dtype=torch.uint8).pin_memory() for _ in range(n)]
    assert p.decode(outs, lens, dec) == [0] * n
    for i in range(n):
        d = dec[i].numpy().reshape(-1, 4)
        assert np.array_equal(d[:, :3], frames[i].reshape(-1, 4)[:, :3]), i
        assert (d[:, 3] == 255).all(), i
    p.close()
