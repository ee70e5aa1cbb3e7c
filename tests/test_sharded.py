"""Single-image encode sharded over ranks.

GPU: the band C ABI run band by band in one process, with the exchanges done
on the host, must give the oracle's stream byte for byte; and the RCCL
orchestration with world size 1.
CPU: the exchange logic of encode_sharded over gloo with 2 ranks and a mock
band backend must assemble exactly what a single process assembles.
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
    import torch
    S = _sharded()
    w, h, c, R = shape
    px = O.gen_syn_v1(w, h, c, 7)
    if shape[0] == 640:   # flat image: runs cross every band
        px = np.tile(np.array([9, 8, 7, 255], np.uint8), w * h)
    want = O.encode(px, w, h, c)
    t = torch.from_numpy(px).cuda()
    N = w * h
    # one context per band: a context holds one band's state between the steps
    ctxs = [S.HipBands(0) for _ in range(R)]
    for be in ctxs:
        be.ctx = nice._Ctx(0)
    ranges = [S.band_tiles(w, h, r, R) for r in range(R)]
    firsts = []
    for be, (lo, hi) in zip(ctxs, ranges):
        p0, p1 = S.band_pixels(w, h, lo, hi)
        firsts.append(int(be.classify(t[p0 * c: p1 * c], p0, w, h, c, c, lo, hi)[0]))
    hist = None
    for r, be in enumerate(ctxs):
        later = [f for f in firsts[r + 1:] if f != S.NONE]
        hr = be.runs(later[0] if later else N)
        hist = hr.clone() if hist is None else hist + hr
    bits, seeds = [], []
    for be in ctxs:
        b, s = be.tables(hist)
        bits.append(b)
        seeds.append(s)
    assert len(set(seeds)) == 1
    bit0s = [seeds[0] + sum(bits[:r]) for r in range(R)]
    words = torch.cat([be.pack(bit0s[r], bits[r]) for r, be in enumerate(ctxs)])
    got = ctxs[0].assemble(words, bit0s, bits, w, h).cpu().numpy().tobytes()
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

    W, H = 300, 40
    N = W * H

    class Mock:
        # deterministic stand-in for the band steps: band r has 'first coded'
        # 100*r+5 (none for r == 1), histogram r+1 per bin, 1000*(r+1)+r bits,
        # words = bit pattern of (rank, index); assembly concatenates the words
        def __init__(self, r): self.r = r
        def classify(self, px, px0, w, h, c, co, lo, hi):
            f = S.NONE if self.r == 1 else 100 * self.r + 5
            return torch.tensor([f, f], dtype=torch.int64)
        def runs(self, band_next):
            self.band_next = band_next
            return torch.full((858,), self.r + 1, dtype=torch.int64)
        def tables(self, hist):
            self.hist_total = int(hist.sum())
            return 1000 * (self.r + 1) + self.r, 6160
        def words(self, bit0, bits):
            return ((bit0 + bits + 31) >> 5) - (bit0 >> 5) if bits else 0
        def pack(self, bit0, bits):
            n = self.words(bit0, bits)
            return torch.arange(n, dtype=torch.int32) + (self.r << 20)
        def assemble(self, cat, bit0s, bitss, w, h):
            return cat

    dist.init_process_group("gloo")
    r, R = dist.get_rank(), dist.get_world_size()
    m = Mock(r)
    out = S.encode_sharded(m, dist, torch.zeros(4), 0, W, H, 4, device="cpu")
    res = {{"rank": r, "band_next": m.band_next, "hist_total": m.hist_total,
           "out": None if out is None else out.tolist()}}
    got = [None] * R
    dist.all_gather_object(got, res)
    if r == 0:
        print(json.dumps(got))
    dist.destroy_process_group()
""")


def test_sharded_exchange_gloo(tmp_path):
    import json
    script = tmp_path / "w.py"
    script.write_text(MOCK_WORKER.format(root=ROOT, pkg=PKG_NAME))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                          "--master-addr", "127.0.0.1", "--master-port", "29547", str(script)],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    res = sorted(json.loads([l for l in out.stdout.splitlines() if l.startswith("[")][-1]),
                 key=lambda d: d["rank"])
    # band 0's runs end at band 2's first coded pixel (band 1 has none); the last band's at N
    assert [d["band_next"] for d in res] == [205, 205, 300 * 40]
    assert all(d["hist_total"] == 858 * (1 + 2 + 3) for d in res)
    # root receives every band's words in rank order
    bits = [1000 * (r + 1) + r for r in range(3)]
    bit0 = [6160 + sum(bits[:r]) for r in range(3)]
    want = []
    for r in range(3):
        n = ((bit0[r] + bits[r] + 31) >> 5) - (bit0[r] >> 5)
        want += [i + (r << 20) for i in range(n)]
    assert res[0]["out"] == want
    assert res[1]["out"] is None and res[2]["out"] is None
