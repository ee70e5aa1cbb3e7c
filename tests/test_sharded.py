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
            return ((bit0 + bits + 31) >> 5) - (bit0 >> 5) + 2 if bits else 0
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
