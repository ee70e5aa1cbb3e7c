"""Codes longer than 25 bits (bitwriter.rs:55-73).

The reference writer keeps a u32 cache and a u8 bit offset: a code whose
length plus the pending bits exceeds 32 makes `32 - bit_offset` wrap, the
shift is masked and the code is *added* into the cache, mangling the pending
bits.  Such streams are still well defined (the encoder output is what
parity means, SURVEY.md §0 finding 7).  The generator (oracle
`gen_deep_codes`) gives small-diff symbol counts that grow like Fibonacci
numbers, so the Huffman merge (hfe.rs:72-84) chains them and the rarest
emitted symbols get 26-31 bit codes; the oracle's counters pin that the
frames really emit long and wrapped codes.  The GPU streams (single frame,
RGB and RGBA, batched with ordinary frames, band API) must be byte-exact.
"""
import numpy as np
import pytest

# (w, h, channels, K): K Fibonacci-weighted symbols
DEEP = [(2048, 2048, 4, 30), (2048, 1280, 3, 29), (2560, 2400, 4, 31)]


def _deep(O, w, h, c, k, seed=1):
    return O.gen_deep_codes(w, h, c, seed, k)


@pytest.mark.parametrize("case", DEEP, ids=[f"{w}x{h}x{c}k{k}" for w, h, c, k in DEEP])
def test_oracle_emits_long_and_wrapped_codes(O, case):
    w, h, c, k = case
    s, st = O.encode(_deep(O, w, h, c, k), w, h, c, with_stats=True)
    assert st.max_emitted_aob >= 29
    assert st.n_long_emits > 10
    assert st.n_wrapped_emits >= 3
    # stream 5's max (zero-count chain under the Fibonacci chain) spills the
    # 5-bit header field and takes 8-bit length fields (hfe.rs:98-103)
    assert st.max_aob[5] > 128


@pytest.mark.gpu
@pytest.mark.parametrize("case", DEEP, ids=[f"{w}x{h}x{c}k{k}" for w, h, c, k in DEEP])
def test_long_codes_single_frame(nice, O, case):
    w, h, c, k = case
    px = _deep(O, w, h, c, k)
    want = O.encode(px, w, h, c)
    got = nice.encode_bytes(px, w, h, c)
    assert len(got) == len(want)
    if got != want:
        d = next(i for i in range(len(want)) if got[i] != want[i])
        pytest.fail(f"first differing byte {d} of {len(want)}")


@pytest.mark.gpu
def test_long_codes_batch_mixed(nice, O):
    """A batch where some frames have long codes and others do not: each frame
    takes its own packer, all byte-exact."""
    import torch
    w, h, c = 2048, 2048, 4
    frames = np.stack([_deep(O, w, h, c, 30, 1), O.gen_syn_v1(w, h, c, 5), _deep(O, w, h, c, 30, 7),
                       O.gen_syn_v1(w, h, c, 6)])
    n = len(frames)
    px = torch.from_numpy(frames).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    nice.encode_batch(px, w, h, c, out, lens)
    torch.cuda.synchronize()
    L = lens.cpu().numpy()
    host = out.cpu().numpy()
    for i in range(n):
        want, st = O.encode(frames[i], w, h, c, with_stats=True)
        assert L[i] == len(want), i
        assert bytes(host[i, :L[i]]) == want, i
        assert (st.n_wrapped_emits > 0) == (i % 2 == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [3, 8])
def test_long_codes_band_api(nice, O, R):
    """One long-code image through the band C ABI (config 4 path): no refusal,
    byte-exact after assembly."""
    import torch
    from conftest import band_encode
    w, h, c = 2560, 2400, 4
    px = _deep(O, w, h, c, 31)
    want = O.encode(px, w, h, c)
    got = band_encode(nice, torch.from_numpy(px).cuda(), w, h, c, R).cpu().numpy().tobytes()
    assert got == want


@pytest.mark.gpu
def test_long_code_stream_decode_refused_cleanly(nice, O):
    """The spilled table header of these streams is outside every decoder's
    domain (the oracle refuses too): a status code, never a crash."""
    w, h, c, k = DEEP[0]
    s = O.encode(_deep(O, w, h, c, k), w, h, c)
    with pytest.raises(O.OracleDecodeError):
        O.decode(s, O.DEC_STRIDE)
    with pytest.raises(nice.NiceError):
        nice.decode_bytes(s)


@pytest.mark.gpu
def test_long_code_at_band_start(nice, O):
    """Bands that start with a long payload code whose wrapped write covers the
    previous band's last bits (the first code, a 1-bit prefix, leaves the
    payload in band_bit0's byte): the write is deferred to the band's trailer
    and applied after the merge; the stream is byte-exact."""
    import torch
    import importlib
    from conftest import PKG_NAME
    S = importlib.import_module(PKG_NAME + ".sharded")
    w, h, c = 2560, 2400, 4
    T = w * h // 1024
    starts = list(range(100, T, 500))   # the rarest symbols sit at these tiles' first pixels
    px = O.gen_deep_codes_at(w, h, c, 1, 31, [t * 1024 for t in starts])
    want = O.encode(px, w, h, c)
    bounds = [0] + starts + [T]
    ranges = list(zip(bounds[:-1], bounds[1:]))
    st = {}
    got = S.encode_bands(torch.from_numpy(px).cuda(), w, h, c, len(ranges), ranges=ranges, stats=st)
    assert st["deferred"], "no band started with a deferred wrapped write: move the split"
    assert got.cpu().numpy().tobytes() == want

