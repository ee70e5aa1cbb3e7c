"""GPU parity: the HIP encoder must produce the oracle's stream byte for byte and
the HIP decoder must reproduce the oracle's pixels, through the C ABI.

Encode parity is bit-exact against the literal restatement of code::encode.
Decode parity: against the oracle's reference-mode decode where the reference
terminates (channels == 3, every max code length <= 24), and against the
original pixels (and the oracle's intent-mode decode) everywhere else.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames():
    """(name, pixels, w, h, c) cases covering the reference test surface."""
    from conftest import oracle_mod
    O = oracle_mod()
    rng = np.random.default_rng(1234)
    cases = [
        ("syn512x4", O.gen_syn_v1(512, 512, 4, 1), 512, 512, 4),
        ("syn256x3", O.gen_syn_v1(256, 256, 3, 1), 256, 256, 3),
        ("syn160x120x3s4", O.gen_syn_v1(160, 120, 3, 4), 160, 120, 3),
        ("syn1920x1080x4", O.gen_syn_v1(1920, 1080, 4, 3), 1920, 1080, 4),
        ("grad512x4", O.gen_gradient(512, 512, 4), 512, 512, 4),
        ("grad64x48x3", O.gen_gradient(64, 48, 3), 64, 48, 3),
        ("odd37x23x4", O.gen_syn_v1(37, 23, 4, 9), 37, 23, 4),
        ("wide1000x7x3", O.gen_syn_v1(1000, 7, 3, 5), 1000, 7, 3),
        # W > 5000: window classify (no LDS ring); W > 8192: row decode with its ring in global memory
        ("wide6000x12x4", O.gen_syn_v1(6000, 12, 4, 6), 6000, 12, 4),
        ("wide9000x6x3", O.gen_syn_v1(9000, 6, 3, 7), 9000, 6, 3),
        ("noise300x200x3", rng.integers(0, 256, 300 * 200 * 3, dtype=np.uint8), 300, 200, 3),
        ("noise128x128x4", rng.integers(0, 256, 128 * 128 * 4, dtype=np.uint8), 128, 128, 4),
        ("flat640x480x4", np.tile(np.array([9, 8, 7, 255], np.uint8), 640 * 480), 640, 480, 4),
        ("w1", O.gen_syn_v1(1, 50, 3, 2), 1, 50, 3),
        ("w2", O.gen_syn_v1(2, 30, 3, 2), 2, 30, 3),
        ("w3", O.gen_syn_v1(3, 20, 4, 2), 3, 20, 4),
        ("5x5", O.gen_syn_v1(5, 5, 3, 2), 5, 5, 3),
        ("1x1", np.array([1, 2, 3], np.uint8), 1, 1, 3),
    ]
    # stripes: long runs crossing encoder tiles (1024 px) and decoder segments
    st = np.zeros((300, 700, 3), np.uint8)
    st[:, :, 0] = (np.arange(300)[:, None] // 7) * 20
    st[::5, ::3, 1] = 200
    cases.append(("stripes700x300x3", st.reshape(-1), 700, 300, 3))
    # few colours: back references and luma references dominate
    pal = np.array([[10, 20, 30], [10, 21, 31], [200, 100, 50], [12, 22, 29]], np.uint8)
    idx = rng.integers(0, 4, (90, 333))
    idx[:, 100:200] = 2
    cases.append(("palette333x90x3", pal[idx].reshape(-1), 333, 90, 3))
    return cases


CASES = _frames()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_encode_bitexact(nice, O, case):
    name, px, w, h, c = case
    want = O.encode(px, w, h, c)
    got = nice.encode_bytes(px, w, h, c)
    assert len(got) == len(want), (len(got), len(want))
    if got != want:
        d = next(i for i in range(len(want)) if got[i] != want[i])
        pytest.fail(f"{name}: first differing byte {d} of {len(want)}")


def test_encode_empty(nice, O):
    for w, h in [(0, 0), (7, 0), (0, 5)]:
        px = np.zeros(0, np.uint8)
        assert nice.encode_bytes(px, w, h, 4) == O.encode(px, w, h, 4)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_decode_matches(nice, O, case):
    name, px, w, h, c = case
    s = O.encode(px, w, h, c)
    rgb = px.reshape(-1, c)[:, :3].reshape(-1)
    try:
        got, img = nice.decode_bytes(s)
    except nice.NiceError as e:
        # only streams outside the decodable domain may be refused
        with pytest.raises(O.OracleDecodeError):
            O.decode(s, O.DEC_STRIDE)
        return
    assert (img.width, img.height, img.channels) == (w, h, c)
    g = np.frombuffer(got, np.uint8).reshape(-1, c)
    assert np.array_equal(g[:, :3].reshape(-1), rgb), name
    if c == 4:
        assert (g[:, 3] == 255).all()
    if c == 3:
        ref, _ = O.decode(s, O.DEC_STRIDE)
        assert np.array_equal(np.frombuffer(got, np.uint8), ref)
    else:
        # RGBA: the stream is the RGB stream with header byte 12 = 4;
        # the oracle decodes the byte-12-patched stream, alpha is filled
        ref, dims = O.decode(s[:12] + bytes([3]) + s[13:], O.DEC_STRIDE)
        assert dims == (w, h, 3)
        assert np.array_equal(g[:, :3].reshape(-1), ref)


@pytest.mark.parametrize("parse", ["fast", "general"])
def test_decode_parse_paths(nice, O, parse, opts):
    """dec_sync decodes a frame whose codes all fit the first-level tables and
    whose pixel events fit 64 bits from one window per event (DecTables::fast),
    others symbol by symbol with refills and the long-code search; forcing the
    general path (NICE_DEC_SLOW_PARSE) must give the same pixels."""
    if parse == "general":
        opts.setenv("NICE_DEC_SLOW_PARSE", "1")
    for name, px, w, h, c in CASES:
        if name not in ("syn512x4", "syn1920x1080x4", "syn256x3", "odd37x23x4", "noise300x200x3",
                        "stripes700x300x3", "palette333x90x3", "wide9000x6x3"):
            continue
        # tolerant header: small frames spill the 5-bit max field (hfe.rs:97-99)
        got, _ = nice.decode_bytes(O.encode(px, w, h, c), flags=nice.DEC_ALPHA_FILL_FF | nice.DEC_TOLERANT_HEADER)
        g = np.frombuffer(got, np.uint8).reshape(-1, c)
        assert np.array_equal(g[:, :3], px.reshape(-1, c)[:, :3]), (name, parse)


@pytest.mark.parametrize("case", [c for c in CASES if c[4] == 3], ids=[c[0] for c in CASES if c[4] == 3])
def test_decode_strict_reference(nice, O, case):
    """STRICT_REFERENCE: fail exactly where the literal reference fails (or may not
    terminate); otherwise identical pixels."""
    name, px, w, h, c = case
    s = O.encode(px, w, h, c)
    try:
        ref, _ = O.decode(s)
        ref_ok = True
    except O.OracleDecodeError:
        ref_ok = False
    try:
        got, _ = nice.decode_bytes(s, flags=nice.DEC_STRICT_REFERENCE)
        ok = True
    except nice.NiceError:
        ok = False
    assert ok == ref_ok, (name, ok, ref_ok)
    if ok:
        assert np.array_equal(np.frombuffer(got, np.uint8), ref)


def test_batch_device_roundtrip(nice, O):
    import torch
    w, h, c, n = 640, 360, 4, 6
    frames = np.stack([O.gen_syn_v1(w, h, c, s) for s in range(1, n + 1)])
    px = torch.from_numpy(frames).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    nice.encode_batch(px, w, h, c, out, lens)
    torch.cuda.synchronize()
    L = lens.cpu().numpy()
    for i in range(n):
        want = O.encode(frames[i], w, h, c)
        assert L[i] == len(want)
        assert bytes(out[i, :L[i]].cpu().numpy()) == want
    dec = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    nice.decode_batch(out, lens, w, h, 4, dec, status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    got = dec.cpu().numpy().reshape(n, -1, 4)
    assert np.array_equal(got[:, :, :3], frames.reshape(n, -1, 4)[:, :, :3])


def test_decode_record_tags_across_calls(nice, O):
    """Run pixels are record slots without the call's tag (no per-call prefill):
    on one context and one shape, frames full of coded pixels alternate with
    frames of long runs over 20 calls (the 4-bit tags wrap every 15) -- stale
    records of an earlier call must never show through a run."""
    import torch
    w, h, c = 640, 360, 4
    busy = O.gen_syn_v1(w, h, c, 11)
    runs = busy.reshape(h, w, c).copy()
    runs[:, 37:600] = runs[:, 36:37]          # each row: one long run
    runs = runs.reshape(-1)
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    ctx = nice.Context(0)
    for i in range(20):
        fr = [busy, runs] if i % 2 == 0 else [runs, busy]
        px = torch.from_numpy(np.stack(fr)).cuda()
        out = torch.zeros((2, bound), dtype=torch.uint8, device="cuda")
        lens = torch.zeros(2, dtype=torch.int64, device="cuda")
        nice.encode_batch(px, w, h, c, out, lens, ctx=ctx)
        dec = torch.zeros((2, w * h * 4), dtype=torch.uint8, device="cuda")
        status = torch.zeros(2, dtype=torch.int32, device="cuda")
        nice.decode_batch(out, lens, w, h, 4, dec, status, ctx=ctx)
        torch.cuda.synchronize()
        assert (status.cpu().numpy() == 0).all(), i
        got = dec.cpu().numpy().reshape(2, -1, 4)
        assert np.array_equal(got[:, :, :3], np.stack(fr).reshape(2, -1, 4)[:, :, :3]), i


def test_config2_single_4k(nice, O):
    """BASELINE config 2: one 3840x2160 RGBA frame through the host entry points
    (nice_encode / nice_decode): byte-exact stream, exact round trip."""
    w, h, c = 3840, 2160, 4
    px = O.gen_syn_v1(w, h, c, 2)
    want = O.encode(px, w, h, c)
    got = nice.encode_bytes(px.tobytes(), w, h, c)
    assert bytes(got) == want
    dec, img = nice.decode_bytes(want)
    assert (img.width, img.height, img.channels) == (w, h, c)
    g = np.frombuffer(dec, np.uint8).reshape(-1, 4)
    assert np.array_equal(g[:, :3], px.reshape(-1, 4)[:, :3])


def test_config3_batch_64x1080p(nice, O):
    """BASELINE config 3: a batch of 64 x 1920x1080 RGBA frames through the
    device batch API -- every stream byte-exact to the oracle, every frame
    decoded back."""
    import torch
    w, h, c, n = 1920, 1080, 4, 64
    frames = np.stack([O.gen_syn_v1(w, h, c, s) for s in range(1, n + 1)])
    px = torch.from_numpy(frames).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    nice.encode_batch(px, w, h, c, out, lens)
    dec = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    nice.decode_batch(out, lens, w, h, 4, dec, status)
    torch.cuda.synchronize()
    L = lens.cpu().numpy()
    host = out.cpu().numpy()
    for i in range(n):
        want = O.encode(frames[i], w, h, c)
        assert L[i] == len(want), i
        assert bytes(host[i, :L[i]]) == want, i
    assert (status.cpu().numpy() == 0).all()
    got = dec.view(n, -1, 4)[:, :, :3]
    assert torch.equal(got, px.view(n, -1, 4)[:, :, :3])


@pytest.mark.parametrize("bits", [1024, 2048, 4096, 8192, 16384])
def test_decode_long_slices(nice, O, bits, opts):
    """Every parse slice size: emission runs from checkpoint sub-slices (the
    default picks long slices only for large batches); checkpoints every 512
    bits up to 4096-bit slices (1024-bit slices hold one), every 1024 from 8192
    (round 6)."""
    opts.setenv("NICE_DEC_SLICE_BITS", str(bits))
    for name, px, w, h, c in CASES:
        if name not in ("syn512x4", "syn1920x1080x4", "stripes700x300x3", "noise300x200x3"):
            continue
        s = O.encode(px, w, h, c)
        try:
            O.decode(s, O.DEC_STRIDE)
        except O.OracleDecodeError:
            with pytest.raises(nice.NiceError):
                nice.decode_bytes(s)
            continue
        got, _ = nice.decode_bytes(s)
        g = np.frombuffer(got, np.uint8).reshape(-1, c)
        assert np.array_equal(g[:, :3].reshape(-1), px.reshape(-1, c)[:, :3].reshape(-1)), name


@pytest.mark.parametrize("mode", [("NICE_DEC_NO_EVENTS", "1"), ("NICE_DEC_EV_CAP", "16"),
                                  ("NICE_DEC_EV_CAP", "64")])
@pytest.mark.parametrize("bits", [1024, 4096])
def test_decode_event_paths(nice, O, mode, bits, opts):
    """Record emission without the first pass's events (every slice parsed again)
    and with a capacity so small that most slices overflow (mixed paths)."""
    opts.setenv(*mode)
    opts.setenv("NICE_DEC_SLICE_BITS", str(bits))
    for name, px, w, h, c in CASES:
        if name not in ("syn512x4", "syn1920x1080x4", "stripes700x300x3", "noise300x200x3", "odd37x23x4"):
            continue
        s = O.encode(px, w, h, c)
        try:
            O.decode(s, O.DEC_STRIDE)
        except O.OracleDecodeError:
            with pytest.raises(nice.NiceError):
                nice.decode_bytes(s)
            continue
        got, _ = nice.decode_bytes(s)
        g = np.frombuffer(got, np.uint8).reshape(-1, c)
        assert np.array_equal(g[:, :3].reshape(-1), px.reshape(-1, c)[:, :3].reshape(-1)), (name, mode, bits)


def test_decode_single_wave_rows(nice, O, opts):
    """The single-wave row kernel (used for W < 64 or W > 16384) on wide images."""
    opts.setenv("NICE_DEC_SINGLE_WAVE", "1")
    for name, px, w, h, c in CASES:
        if name not in ("syn512x4", "odd37x23x4", "palette333x90x3"):
            continue
        s = O.encode(px, w, h, c)
        try:
            O.decode(s, O.DEC_STRIDE)
        except O.OracleDecodeError:
            with pytest.raises(nice.NiceError):
                nice.decode_bytes(s)
            continue
        got, _ = nice.decode_bytes(s)
        g = np.frombuffer(got, np.uint8).reshape(-1, c)
        assert np.array_equal(g[:, :3].reshape(-1), px.reshape(-1, c)[:, :3].reshape(-1)), name


# SYN-v1 RGB frames inside the literal reference decoder's domain (the oracle's
# reference-mode decode terminates; (256, 64, 8) and (200, 64, 4) have 25-bit
# tables, which never wrap the reference's refill loop), and frames with 26-31
# bit tables on which the reference's refill loop wraps and never ends
# (bitreader.rs:85-98): strict mode must fail on exactly those.
STRICT_DOMAIN = [(512, 512, 1), (512, 512, 2), (333, 211, 3), (640, 480, 4), (1920, 1080, 5),
                 (1000, 997, 6), (300, 300, 7), (256, 64, 8), (1024, 768, 9), (200, 150, 10),
                 (200, 64, 4), (256, 64, 1), (160, 60, 2), (100, 100, 4), (240, 48, 9), (140, 70, 10)]


@pytest.mark.parametrize("case", STRICT_DOMAIN, ids=[f"{w}x{h}s{s}" for w, h, s in STRICT_DOMAIN])
def test_decode_strict_reference_domain(nice, O, case):
    """Strict mode decodes exactly the streams the literal reference decodes
    (identical pixels) and refuses the others."""
    w, h, seed = case
    px = O.gen_syn_v1(w, h, 3, seed)
    s = O.encode(px, w, h, 3)
    try:
        ref, _ = O.decode(s)
    except O.OracleDecodeError:
        with pytest.raises(nice.NiceError):
            nice.decode_bytes(s, flags=nice.DEC_STRICT_REFERENCE)
        # the intent decoder reads them correctly
        got, _ = nice.decode_bytes(s)
        assert np.array_equal(np.frombuffer(got, np.uint8), px)
        return
    got, _ = nice.decode_bytes(s, flags=nice.DEC_STRICT_REFERENCE)
    assert np.array_equal(np.frombuffer(got, np.uint8), ref)
    assert np.array_equal(ref, px)
