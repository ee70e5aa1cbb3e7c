"""Classify kernel routing: every frame shape the reference encodes the same
way (code.rs:141-145, 159-414) goes through an LDS-staged kernel where the
rows fit -- the 16K-pixel ring (W <= 4777), the strip kernel (RGBA, W % 1024
== 0), the 32K-pixel ring (W <= 10239: 8K UHD's 7680, RGB rows), per-tile
row windows for every wider shape (RGB, or RGBA rows that are not whole
tiles) -- including the band API (config 4).  Streams must equal the oracle's and
the test hook must name the fast kernel."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WINDOW, TINY, RING, RING2, STRIP, PAIR, TWIN, SLIDE = range(8)


def _same(got, want, what):
    if got != want:   # no pytest repr of multi-MB byte strings
        d = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), min(len(got), len(want)))
        pytest.fail(f"{what}: lengths {len(got)} / {len(want)}, first differing byte {d}")


def _last(nice, ctx):
    L = nice.lib()
    L.nice_test_last_classify.argtypes = [ctypes.c_void_p]
    L.nice_test_last_classify.restype = ctypes.c_int
    return L.nice_test_last_classify(ctx.ptr)


def _encode_dev(nice, px, w, h, c, ctx):
    import torch
    t = torch.from_numpy(px.reshape(1, -1)).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((1, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(1, dtype=torch.int64, device="cuda")
    nice.encode_batch(t, w, h, c, out, lens, ctx=ctx)
    torch.cuda.synchronize()
    return bytes(out[0, :int(lens[0])].cpu().numpy())


@pytest.mark.parametrize("shape,kind", [((7680, 64, 4), RING2), ((6000, 32, 3), RING2), ((10239, 9, 4), RING2),
                                        ((10239, 11, 3), RING2), ((4777, 20, 4), RING), ((4778, 20, 3), RING2),
                                        ((4095, 20, 4), SLIDE), ((4095, 20, 3), RING), ((1000, 30, 4), SLIDE),
                                        ((8192, 12, 4), STRIP), ((10240, 5, 3), TWIN), ((11000, 5, 4), TWIN),
                                        ((10241, 9, 3), TWIN), ((12000, 7, 4), TWIN), ((20000, 5, 3), TWIN)],
                         ids=lambda v: "x".join(map(str, v)) if isinstance(v, tuple) else str(v))
def test_route_and_bitexact(nice, O, shape, kind):
    w, h, c = shape
    px = O.gen_syn_v1(w, h, c, 3)
    ctx = nice.Context(0)
    got = _encode_dev(nice, px, w, h, c, ctx)
    assert _last(nice, ctx) == kind
    _same(got, O.encode(px, w, h, c), shape)


def test_8k_uhd_batch(nice, O):
    """Two 7680 x 256 RGBA frames (8K UHD rows) in one batch: ring2, byte-exact."""
    import torch
    w, h, c, n = 7680, 256, 4, 2
    frames = np.stack([O.gen_syn_v1(w, h, c, s) for s in (4, 5)])
    ctx = nice.Context(0)
    t = torch.from_numpy(frames).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    nice.encode_batch(t, w, h, c, out, lens, ctx=ctx)
    torch.cuda.synchronize()
    assert _last(nice, ctx) == RING2
    for i in range(n):
        _same(bytes(out[i, :int(lens[i])].cpu().numpy()), O.encode(frames[i], w, h, c), i)


@pytest.mark.parametrize("shape,kind", [((1920, 1080, 4, 4), PAIR), ((1000, 700, 3, 3), RING),
                                        ((7680, 300, 4, 3), RING2), ((8192, 200, 4, 2), STRIP),
                                        ((11000, 60, 4, 3), TWIN), ((10300, 50, 3, 2), TWIN)],
                         ids=lambda v: "x".join(map(str, v)) if isinstance(v, tuple) else str(v))
def test_band_routes(nice, O, shape, kind):
    """The band API's classify takes the same kernels (a band's first block
    prefills from the 3 rows + 3 pixels before it)."""
    import importlib
    import torch
    from conftest import PKG_NAME
    S = importlib.import_module(PKG_NAME + ".sharded")
    w, h, c, R = shape
    px = O.gen_syn_v1(w, h, c, 9)
    backends = []
    got = S.encode_bands(torch.from_numpy(px).cuda(), w, h, c, R, backends=backends).cpu().numpy().tobytes()
    assert [_last(nice, be.ctx) for be in backends] == [kind] * R
    _same(got, O.encode(px, w, h, c), shape)
