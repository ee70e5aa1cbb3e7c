"""enc_pack's over-cap path (hfe.rs:110-113, bitwriter.rs:55-73).

A packer group (4 tiles, 4096 pixels) collects its codes in an LDS buffer of
32 bits per pixel.  A group that goes over it -- only possible after its first
tiles have already been OR-ed into the buffer -- is counted and OR-ed into the
output directly instead, and the next group on the block must clear the whole
buffer.  The test hook pack_cap_bpp=b lowers the buffer to b bits per pixel so ordinary
frames reach that path (mid-group, after tiles were written); a frame with one
row of noise in a smooth image reaches it at the real cap.  Every stream must
equal the oracle's byte for byte.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def cap_hook(nice):
    """Sets the default context's packer cap (bits per pixel); reset after."""
    from conftest import set_hooks
    ctx = nice._ctx(0)
    yield lambda b: set_hooks(nice, ctx, pack_cap_bpp=b)
    set_hooks(nice, ctx)


@pytest.mark.parametrize("cap", [4, 8, 12])
def test_pack_cap_single_frames(nice, O, cap, cap_hook):
    cap_hook(cap)
    for w, h, c, seed in [(1920, 1080, 4, 3), (4096, 64, 4, 5), (1000, 333, 3, 2)]:
        px = O.gen_syn_v1(w, h, c, seed)
        want = O.encode(px, w, h, c)
        got = nice.encode_bytes(px, w, h, c)
        assert got == want, (w, h, c, cap)


def test_pack_cap_batch(nice, O, cap_hook):
    """A batch: blocks move between frames and reuse their LDS buffer across
    over-cap and ordinary groups."""
    import torch
    cap_hook(11)   # SYN-v1 averages ~10.7 bits/px: both kinds of group
    w, h, c, n = 1280, 720, 4, 6
    frames = np.stack([O.gen_syn_v1(w, h, c, s) for s in range(1, n + 1)])
    px = torch.from_numpy(frames).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    nice.encode_batch(px, w, h, c, out, lens)
    torch.cuda.synchronize()
    L = lens.cpu().numpy()
    host = out.cpu().numpy()
    for i in range(n):
        want = O.encode(frames[i], w, h, c)
        assert bytes(host[i, :L[i]]) == want, i


def test_pack_cap_bands(nice, O):
    import importlib
    import torch
    from conftest import PKG_NAME, set_hooks
    S = importlib.import_module(PKG_NAME + ".sharded")
    w, h, c, R = 2048, 512, 4, 3
    px = O.gen_syn_v1(w, h, c, 4)
    want = O.encode(px, w, h, c)
    backends = []
    for _ in range(R):
        be = S.HipBands(0)
        be.ctx = nice._Ctx(0)
        set_hooks(nice, be.ctx, pack_cap_bpp=8)
        backends.append(be)
    got = S.encode_bands(torch.from_numpy(px).cuda(), w, h, c, R, backends=backends).cpu().numpy().tobytes()
    assert got == want


def test_pack_noise_row_real_cap(nice, O):
    """Rows of uniform noise in a 4096-wide frame of RGB-mode pixels with
    geometric residuals (oracle gen_rgb_field): each noise row is one packer
    group whose residuals take the rare 15-17 bit codes of stream 0, about 50
    bits per pixel, so the group goes over the real cap after its first tiles;
    the groups after it reuse the buffer."""
    w, h, c = 4096, 1024, 4
    px = O.gen_rgb_field(w, h, c, 1, [300, 301, 400])
    want, st = O.encode(px, w, h, c, with_stats=True)
    assert st.max_emitted_aob <= 25   # not a long-code frame: the one-pass packer runs
    aob = np.array(st.aob[0:256])
    rare = aob[np.array(st.hist[0:256]) > 0].max()
    assert 3 * rare > 40, rare        # a noise pixel: prefix + three rare residuals
    got = nice.encode_bytes(px, w, h, c)
    assert got == want


def test_pack_rare_path_mixed(nice, O):
    """Waves whose pixels mix >32-bit codes (noise in a frame of RGB-mode
    pixels with geometric residuals) with runs longer than 64 pixels (extra
    run digits, code.rs:391-406): the packer's entry-by-entry path, next to
    ordinary waves; the stream must equal the oracle's."""
    w, h, c = 2048, 256, 4
    px = O.gen_rgb_field(w, h, c, 3, [40, 41, 200]).reshape(h, w, c)
    for y in (40, 41, 200):          # noise rows cut by runs of 65..300 pixels
        x = 17
        while x < w - 400:
            n = 65 + (x * 7) % 236
            px[y, x:x + n, :3] = px[y, x, :3]
            x += n + 50
    px[120, 100:1900, :3] = (5, 6, 7)   # one long run in the smooth field
    px = px.reshape(-1)
    want, st = O.encode(px, w, h, c, with_stats=True)
    assert st.max_emitted_aob <= 25
    got = nice.encode_bytes(px, w, h, c)
    if got != want:
        d = next(i for i in range(min(len(got), len(want))) if got[i] != want[i])
        pytest.fail(f"first differing byte {d} of {len(want)} (got {len(got)})")
