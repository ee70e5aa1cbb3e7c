"""Single-image encode sharded over ranks.

GPU: the band C ABI in one process (device-resident steps, and the
host-returning ones) must give the oracle's stream byte for byte; and the
RCCL orchestration with world size 1.
CPU: the exchange logic of encode_sharded over gloo with 3 ranks and a mock
band backend must assemble exactly what a single process assembles, and a
step failing on one rank must make every rank raise.
"""
import importlib
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from conftest import PKG_NAME, ROOT


def _sharded():
    return importlib.import_module(PKG_NAME + ".sharded")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1000, 700, 4, 2), (2048, 300, 3, 3), (640, 480, 4, 4), (8192, 8192, 4, 8)])
def test_band_api_matches_oracle(nice, O, shape):
    """The device-resident steps (runs_dev / tables_dev / pack_bits), bands on
    their own streams, one host read."""
    import torch
    S = _sharded()
    w, h, c, R = shape
    px = O.gen_syn_v1(w, h, c, 7)
    if shape[0] == 640:   # flat image: runs cross every band
        px = np.tile(np.array([9, 8, 7, 255], np.uint8), w * h)
    want = O.encode(px, w, h, c)
    got = S.encode_bands(torch.from_numpy(px).cuda(), w, h, c, R).cpu().numpy().tobytes()
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1000, 700, 4, 2), (640, 480, 4, 4)])
def test_band_api_host_steps(nice, O, shape):
    """The host-returning steps (nice_band_runs / nice_band_tables /
    nice_band_pack), driven band by band."""
    import ctypes
    import torch
    S = _sharded()
    w, h, c, R = shape
    px = O.gen_syn_v1(w, h, c, 7)
    if shape[0] == 640:
        px = np.tile(np.array([9, 8, 7, 255], np.uint8), w * h)
    want = O.encode(px, w, h, c)
    t = torch.from_numpy(px).cuda()
    L = nice.lib()
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.nice_band_runs.argtypes = [vp, vp, u32, vp]
    L.nice_band_tables.argtypes = [vp, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.nice_band_pack.argtypes = [vp, vp, u64, vp, u64]
    bes = [S.HipBands(0) for _ in range(R)]
    for be in bes:
        be.ctx = nice._Ctx(0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ranges = [S.band_tiles(w, h, r, R) for r in range(R)]
    firsts = []
    for be, (lo, hi) in zip(bes, ranges):
        p0, p1 = S.band_pixels(w, h, lo, hi)
        firsts.append(int(be.classify(t[p0 * c: p1 * c], p0, w, h, c, c, lo, hi)[0]))
    hist = torch.zeros(858, dtype=torch.int32, device="cuda")
    for r, be in enumerate(bes):
        later = [f for f in firsts[r + 1:] if f != S.NONE]
        hr = torch.empty(858, dtype=torch.int32, device="cuda")
        assert L.nice_band_runs(be.ctx.ptr, st, later[0] if later else w * h, hr.data_ptr()) == 0
        hist += hr
    bits, seeds = [], []
    for be in bes:
        b, sd = u64(), u64()
        assert L.nice_band_tables(be.ctx.ptr, st, hist.data_ptr(), ctypes.byref(b), ctypes.byref(sd)) == 0
        bits.append(b.value)
        seeds.append(sd.value)
    assert len(set(seeds)) == 1
    bit0s = [seeds[0] + sum(bits[:r]) for r in range(R)]
    parts = []
    for r, be in enumerate(bes):
        n = be.words(bit0s[r], bits[r])
        buf = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
        assert L.nice_band_pack(be.ctx.ptr, st, bit0s[r], buf.data_ptr(), n) == 0
        parts.append(buf[:n])
    got = bes[0].assemble(torch.cat(parts), bit0s, bits, w, h).cpu().numpy().tobytes()
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("delta", [+1, -1, "zero"])
def test_band_pack_wrong_bits_reported(nice, O, delta):
    """nice_band_pack_bits with a band_bits other than the band's own (after
    nice_band_tables_dev): nothing is written past the caller's words, and
    nice_band_assemble returns NICE_E_ARG instead of a corrupt stream.  The
    d_info tensor is freed and overwritten before the pack (the context keeps
    its own copy)."""
    import torch
    S = _sharded()
    w, h, c, R = 1000, 700, 4, 3
    px = torch.from_numpy(O.gen_syn_v1(w, h, c, 7)).cuda()
    bes = [S.HipBands(0) for _ in range(R)]
    for be in bes:
        be.ctx = nice._Ctx(0)
    ranges = [S.band_tiles(w, h, r, R) for r in range(R)]
    edges = []
    for be, (lo, hi) in zip(bes, ranges):
        p0, p1 = S.band_pixels(w, h, lo, hi)
        edges.append(be.classify(px[p0 * c: p1 * c], p0, w, h, c, c, lo, hi))
    nxt = S.band_next_of(torch.stack(edges)[:, 0], w * h).to(torch.int32)
    hist = torch.stack([be.runs(nxt[r]) for r, be in enumerate(bes)]).sum(0, dtype=torch.int32)
    infos = [be.tables(hist) for be in bes]
    info = torch.stack(infos).cpu()
    for be in bes:   # the caller's d_info buffers go away (the caching allocator reuses them)
        be._info.fill_(-1)
        be._info = None
    del infos
    torch.cuda.synchronize()
    bits = [int(x) for x in info[:, 0]]
    seed = int(info[0, 1])
    bit0s = [seed + sum(bits[:r]) for r in range(R)]
    wrong = list(bits)
    wrong[1] = 0 if delta == "zero" else bits[1] + delta
    wbit0s = [seed + sum(wrong[:r]) for r in range(R)]   # consistent offsets: only the device sees it
    parts = []
    for r, be in enumerate(bes):
        n = be.words(wbit0s[r], wrong[r])
        buf = torch.full((n + 64,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        be.pack(wbit0s[r], wrong[r], buf[:n])
        torch.cuda.synchronize()
        assert (buf[n:] == 0x5A5A5A5A).all(), r   # the guard words untouched
        parts.append(buf[:n])
    with pytest.raises(nice.NiceError):
        bes[0].assemble(torch.cat(parts), wbit0s, wrong, w, h)
    # the right counts still assemble the oracle's stream
    parts = []
    for r, be in enumerate(bes):
        parts.append(be.pack(bit0s[r], bits[r]))
    got = bes[0].assemble(torch.cat(parts), bit0s, bits, w, h).cpu().numpy().tobytes()
    assert got == O.encode(px.cpu().numpy(), w, h, c)


@pytest.mark.gpu
def test_encode_sharded_world1_rccl(nice, O, tmp_path):
    """encode_sharded over a real process group (nccl = RCCL), one rank."""
    script = tmp_path / "one.py"
    script.write_text(textwrap.dedent(f"""
        import importlib, sys, numpy as np, torch, torch.distributed as dist
        sys.path.insert(0, {ROOT!r})
        from oracle import oracle as O
        S = importlib.import_module({PKG_NAME!r} + ".sharded")
        dist.init_process_group("nccl")
        torch.cuda.set_device(0)
        w, h = 1500, 900
        px = O.gen_syn_v1(w, h, 4, 3)
        out = S.encode_sharded(S.HipBands(0), dist, torch.from_numpy(px).cuda(), 0, w, h, 4)
        ok = out.cpu().numpy().tobytes() == O.encode(px, w, h, 4)
        dist.destroy_process_group()
        print("OK" if ok else "MISMATCH")
    """))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29561", RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().endswith("OK")


MOCK_WORKER = textwrap.dedent("""
    import importlib, json, sys
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    S = importlib.import_module({pkg!r} + ".sharded")
    NiceError = importlib.import_module({pkg!r}).NiceError

    W, H = 300, 40
    N = W * H
    FAIL = {fail!r}   # (rank, step) that raises, or None

    class Mock:
        # deterministic stand-in for the band steps: band r has 'first coded'
        # 100*r+5 (none for r == 1), histogram r+1 per bin, 1000*(r+1)+r bits,
        # words = bit pattern of (rank, index); assembly concatenates the words
        def __init__(self, r): self.r = r
        def _fail(self, step):
            if FAIL and FAIL[0] == self.r and FAIL[1] == step:
                raise NiceError(-7, step)
        def classify(self, px, px0, w, h, c, co, lo, hi):
            self._fail("classify")
            f = S.NONE if self.r == 1 else 100 * self.r + 5
            return torch.tensor([f, f], dtype=torch.int64)
        def runs(self, band_next):
            self._fail("runs")
            self.band_next = int(band_next)
            return torch.full((858,), self.r + 1, dtype=torch.int32)
        def tables(self, hist):
            self._fail("tables")
            self.hist_total = int(hist.sum())
            return torch.tensor([1000 * (self.r + 1) + self.r, 6160], dtype=torch.int64)
        def words(self, bit0, bits):
            return ((bit0 + bits + 31) >> 5) - (bit0 >> 5) + 2 if bits else 2
        def pack(self, bit0, bits):
            self._fail("pack")
            n = self.words(bit0, bits)
            return torch.arange(n, dtype=torch.int32) + (self.r << 20)
        def assemble(self, cat, bit0s, bitss, w, h):
            return cat

    dist.init_process_group("gloo")
    r, R = dist.get_rank(), dist.get_world_size()
    m = Mock(r)
    try:
        out = S.encode_sharded(m, dist, torch.zeros(4), 0, W, H, 4, device="cpu")
        res = {{"rank": r, "band_next": m.band_next, "hist_total": m.hist_total,
               "out": None if out is None else out.tolist()}}
    except NiceError as e:
        res = {{"rank": r, "error": str(e)}}
    got = [None] * R
    dist.all_gather_object(got, res)
    if r == 0:
        print(json.dumps(got))
    dist.destroy_process_group()
""")


def _run_mock(tmp_path, fail, port):
    import json
    script = tmp_path / "w.py"
    script.write_text(MOCK_WORKER.format(root=ROOT, pkg=PKG_NAME, fail=fail))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    return sorted(json.loads([l for l in out.stdout.splitlines() if l.startswith("[")][-1]),
                  key=lambda d: d["rank"])


def test_sharded_exchange_gloo(tmp_path):
    res = _run_mock(tmp_path, None, 29547)
    # band 0's runs end at band 2's first coded pixel (band 1 has none); the last band's at N
    assert [d["band_next"] for d in res] == [205, 205, 300 * 40]
    assert all(d["hist_total"] == 858 * (1 + 2 + 3) for d in res)
    # root receives every band's words in rank order
    bits = [1000 * (r + 1) + r for r in range(3)]
    bit0 = [6160 + sum(bits[:r]) for r in range(3)]
    want = []
    for r in range(3):
        n = ((bit0[r] + bits[r] + 31) >> 5) - (bit0[r] >> 5) + 2
        want += [i + (r << 20) for i in range(n)]
    assert res[0]["out"] == want
    assert res[1]["out"] is None and res[2]["out"] is None


@pytest.mark.parametrize("fail", [(1, "classify"), (2, "runs"), (0, "tables"), (1, "pack"), (0, "pack")])
def test_sharded_error_every_rank_raises(tmp_path, fail):
    """A step failing on one rank: every rank raises (none waits in a
    collective), naming the step."""
    port = 29600 + 7 * ["classify", "runs", "tables", "pack"].index(fail[1]) + fail[0]
    res = _run_mock(tmp_path, list(fail), port)
    assert all("error" in d for d in res), res
    assert all(("nice_band_" + fail[1]) in d["error"] for d in res), res


# ---- eight-rank rehearsal with real band bit counts (CPU, gloo) -------------
ORACLE_WORKER = textwrap.dedent("""
    import importlib, json, sys
    sys.path.insert(0, {root!r})
    import numpy as np, torch, torch.distributed as dist
    from oracle import oracle as O
    S = importlib.import_module({pkg!r} + ".sharded")

    W, H, C = 2048, 2048, 4
    N = W * H
    MAX = np.uint64(2**64 - 1)

    def image(R):
        # Fibonacci-skewed small diffs (codes up to 29 bits), the rarest
        # symbols forced onto the first pixels of bands 1 and 2; rows
        # 700..1039 one flat colour: a run from band 2 across all of band 3
        # (no coded pixel: 0 bits) into band 4
        starts = [S.band_tiles(W, H, r, R)[0] * 1024 for r in range(R)]
        return O.gen_deep_codes_flat(W, H, C, 1, 29, [starts[1], starts[2]], (700, 1040))

    class OracleBands:
        # the band steps restated from the oracle's whole-image stream: a band's
        # bits are [bit of its first coded pixel, bit of the next band's), its
        # words that slice at its stream word positions (nice_band_words)
        def __init__(self, px, R):
            self.px, self.R = px, R
            self.stream, self.bit = O.encode_bitpos(px, W, H, C)
            _, st = O.encode(px, W, H, C, with_stats=True)
            self.hist = np.array(st.hist, dtype=np.int64)
            self.coded = np.nonzero(self.bit[:N] != MAX)[0]
        def _first_from(self, p):
            k = np.searchsorted(self.coded, p)
            return int(self.coded[k]) if k < len(self.coded) else None
        def classify(self, px, px0, w, h, c, co, lo, hi):
            self.lo, self.hi = lo * 1024, min(hi * 1024, N)
            k0, k1 = np.searchsorted(self.coded, [self.lo, self.hi])
            f = int(self.coded[k0]) if k1 > k0 else S.NONE
            l = int(self.coded[k1 - 1]) if k1 > k0 else S.NONE
            return torch.tensor([f, l], dtype=torch.int64)
        def runs(self, band_next):
            self.band_next = int(band_next)
            r = dist.get_rank()
            part = self.hist // self.R + (self.hist % self.R if r == 0 else 0)
            return torch.from_numpy(part.astype(np.int32))
        def tables(self, hist):
            self.hist_ok = bool(np.array_equal(hist.numpy().astype(np.int64), self.hist))
            f = self._first_from(self.lo)
            start = int(self.bit[f]) if f is not None and f < self.hi else None
            nxt = self._first_from(self.hi)
            end = int(self.bit[nxt]) if nxt is not None else int(self.bit[N])
            bits = end - start if start is not None else 0
            return torch.tensor([bits, int(self.bit[0])], dtype=torch.int64)
        def words(self, bit0, bits):
            return ((bit0 + bits + 31) >> 5) - (bit0 >> 5) + 2 if bits else 2
        def pack(self, bit0, bits):
            n = self.words(bit0, bits)
            if not n:
                return torch.zeros(0, dtype=torch.int32)
            allb = np.unpackbits(np.frombuffer(self.stream, np.uint8))
            w0 = (bit0 >> 5) * 32
            buf = np.zeros((n - 2) * 32, np.uint8)
            buf[bit0 - w0: bit0 - w0 + bits] = allb[bit0: bit0 + bits]
            wd = np.packbits(buf).view(">u4").astype(np.int64)
            return torch.from_numpy(np.concatenate([wd, [0, 0]]).astype(np.uint32).view(np.int32))
        def assemble(self, cat, bit0s, bitss, w, h):
            seed, end = bit0s[0], bit0s[0] + sum(bitss)
            out = np.zeros(((end + 31) >> 5) * 32 + 64, np.uint8)
            out[:seed] = np.unpackbits(np.frombuffer(self.stream, np.uint8))[:seed]   # the root's header
            words = cat.numpy().view(np.uint32)
            off = 0
            for b0, b in zip(bit0s, bitss):
                n = self.words(b0, b)
                if n:
                    seg = np.unpackbits(words[off: off + n - 2].astype(">u4").view(np.uint8))
                    out[(b0 >> 5) * 32: (b0 >> 5) * 32 + seg.size] |= seg
                off += n
            by = np.packbits(out[:end + (-end) % 8]).tobytes()
            B = end >> 3
            P = by[B] if end & 7 else 0
            return by[:B] + bytes([P, P, 0, 0, 0])

    dist.init_process_group("gloo")
    r, R = dist.get_rank(), dist.get_world_size()
    px = image(R)
    be = OracleBands(px, R)
    out = S.encode_sharded(be, dist, torch.zeros(4), 0, W, H, C, device="cpu")
    res = {{"rank": r, "band_next": be.band_next, "hist_ok": be.hist_ok, "lo": be.lo}}
    if r == 0:
        res["equal"] = out == be.stream
        res["len"] = len(be.stream)
    got = [None] * R
    dist.all_gather_object(got, res)
    if r == 0:
        # per-band bits and first-pixel cost, from the same oracle data
        info = []
        for q in range(R):
            lo, hi = S.band_tiles(W, H, q, R)
            lo, hi = lo * 1024, min(hi * 1024, N)
            f = be._first_from(lo)
            nb = None if f is None or f >= hi else be._first_from(f + 1)
            cost = int(be.bit[nb] - be.bit[f]) if nb is not None else None
            info.append({{"first": f if f is not None and f < hi else None, "first_cost": cost}})
        print(json.dumps({{"ranks": got, "bands": info}}))
    dist.destroy_process_group()
""")


def test_sharded_exchange_gloo_8_ranks(tmp_path, O):
    """encode_sharded's exchange at world size 8 (the config-4 split) over
    gloo, with band steps restated from the oracle's whole-image stream (real
    bit counts, so bands start at arbitrary bit offsets): a 2048^2 frame with
    ~30-bit codes, the rarest forced onto band starts, and a flat region whose
    run starts in band 2, covers all of band 3 (0 bits) and ends in band 4.
    The root's assembled stream must equal the oracle's whole-image encode.
    (The same split runs on the GPU's band API in test_configs /
    test_long_codes; this covers the rank exchange at the driver's 8 ranks.)"""
    import json
    script = tmp_path / "w8.py"
    script.write_text(ORACLE_WORKER.format(root=ROOT, pkg=PKG_NAME))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                          "--master-addr", "127.0.0.1", "--master-port", "29671", str(script)],
                         capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    ranks = sorted(res["ranks"], key=lambda d: d["rank"])
    bands = res["bands"]
    print(bands)
    assert ranks[0]["equal"], "assembled stream differs from the oracle's"
    assert all(d["hist_ok"] for d in ranks)
    # band 3 lies inside the run: no coded pixel, so band 2's runs end in band 4
    assert bands[3]["first"] is None
    assert ranks[2]["band_next"] == ranks[3]["band_next"] == bands[4]["first"]
    assert bands[4]["first"] >= 1040 * 2048
    # bands 1 and 2 start with the rarest symbols: a pixel of >= 28 bits, a
    # 1-2 bit small-diff prefix and a small-diff code of over 25 bits (the
    # reference writer's wrapped write, bitwriter.rs:55-73)
    assert all(bands[q]["first"] == ranks[q]["lo"] and bands[q]["first_cost"] >= 28 for q in (1, 2))
