"""One image encoded by several GPUs (BASELINE config 4).

Rows of tiles are split into bands, one per rank.  Every rank holds its band
plus the 3 rows (+3 pixels) its references reach, classifies it on its own GPU
and takes part in the exchange steps the format needs -- all over
``torch.distributed`` (backend "nccl" = RCCL over xGMI on MI355X; "gloo" in
the CPU tests):

1. all-gather of each band's first/last coded pixel: a run that starts in one
   band may end in a later one, and its length fixes the run digits
   (code.rs:371-407);
2. all-reduce of the 858-bin symbol histogram, so every rank builds the same
   Huffman tables (hfe.rs:51-117);
3. all-gather of the band bit counts: each band's bit offset in the stream;
4. gather-v of the band words to the root (grouped point-to-point sends and
   receives, ``batch_isend_irecv`` = one ncclGroupStart/End on RCCL, so the
   peers' transfers run concurrently over their own xGMI links), which ORs the
   shared boundary words and writes header and tail.

A band step that fails on one rank (a NiceError from the C ABI) is reported
through the next exchange (an error word rides along in each gathered or
reduced tensor), so every rank raises instead of waiting in a collective.

The root's bytes equal ``encode_bytes`` of the whole image.  The band steps
go through a *backend* object (``HipBands`` drives libnice_hip.so); the
exchange logic is backend-independent so it can be tested with gloo on CPU.
"""
from __future__ import annotations

import ctypes

NONE = 0xFFFFFFFF


def tile_pixels() -> int:
    from . import lib
    L = lib()
    L.nice_tile_pixels.restype = ctypes.c_uint32
    return int(L.nice_tile_pixels())


def band_tiles(width: int, height: int, rank: int, world: int, tile: int = 1024):
    """Tile range [lo, hi) of `rank` (contiguous, as even as possible)."""
    n_tiles = (width * height + tile - 1) // tile
    return n_tiles * rank // world, n_tiles * (rank + 1) // world


def band_pixels(width: int, height: int, lo: int, hi: int, tile: int = 1024):
    """Pixel range [px0, px1) a rank must hold for tiles [lo, hi): the band and
    the 3 rows + 3 pixels before it (code.rs:141-145 references)."""
    n = width * height
    b0 = lo * tile
    return max(0, b0 - 3 * width - 3), min(n, hi * tile)


class HipBands:
    """Band steps on the GPU through the C ABI (include/nice.h)."""

    def __init__(self, device: int = 0):
        from . import _ctx, lib
        self.L = lib()
        self.ctx = _ctx(device)
        self.device = device
        L = self.L
        vp, u8, u32, u64 = ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64
        L.nice_band_classify.argtypes = [vp, vp, vp, u64, u64, u32, u32, u8, u8, u32, u32, vp]
        L.nice_band_runs.argtypes = [vp, vp, u32, vp]
        L.nice_band_tables.argtypes = [vp, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.nice_band_words.argtypes = [u64, u64]
        L.nice_band_words.restype = u64
        L.nice_band_pack.argtypes = [vp, vp, u64, vp, u64]
        L.nice_band_assemble.argtypes = [vp, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64), u32, vp, u64,
                                         ctypes.POINTER(u64)]

    def _st(self):
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, rc, what):
        from . import NiceError
        if rc != 0:
            raise NiceError(rc, what)

    def classify(self, px, px0, width, height, channels, channels_out, lo, hi):
        import torch
        edges = torch.empty(2, dtype=torch.int32, device=px.device)
        self._check(self.L.nice_band_classify(self.ctx.ptr, self._st(), ctypes.c_void_p(px.data_ptr()), px0,
                                              px.numel() // channels, width, height, channels, channels_out,
                                              lo, hi, ctypes.c_void_p(edges.data_ptr())), "nice_band_classify")
        return edges.to(torch.int64) & NONE

    def runs(self, band_next):
        import torch
        hist = torch.empty(858, dtype=torch.int32, device=f"cuda:{self.device}")
        self._check(self.L.nice_band_runs(self.ctx.ptr, self._st(), band_next, ctypes.c_void_p(hist.data_ptr())),
                    "nice_band_runs")
        return hist

    def tables(self, hist_total):
        import torch
        bits, seed = ctypes.c_uint64(), ctypes.c_uint64()
        # the C ABI reads the histogram on this rank's GPU (gloo reduces on the host)
        h = hist_total.to(device=f"cuda:{self.device}", dtype=torch.int32).contiguous()
        self._check(self.L.nice_band_tables(self.ctx.ptr, self._st(), ctypes.c_void_p(h.data_ptr()),
                                            ctypes.byref(bits), ctypes.byref(seed)), "nice_band_tables")
        return int(bits.value), int(seed.value)

    def words(self, bit0, bits):
        return int(self.L.nice_band_words(bit0, bits))

    def pack(self, bit0, bits):
        import torch
        n = self.words(bit0, bits)
        out = torch.zeros(max(n, 1), dtype=torch.int32, device=f"cuda:{self.device}")
        self._check(self.L.nice_band_pack(self.ctx.ptr, self._st(), bit0, ctypes.c_void_p(out.data_ptr()), n),
                    "nice_band_pack")
        return out[:n]

    def assemble(self, words_cat, bit0s, bitss, width, height):
        import torch
        from . import encode_bound
        R = len(bit0s)
        cap = encode_bound(width, height)
        out = torch.empty((cap + 3) // 4 * 4, dtype=torch.uint8, device=f"cuda:{self.device}")
        b0 = (ctypes.c_uint64 * R)(*bit0s)
        bb = (ctypes.c_uint64 * R)(*bitss)
        n = ctypes.c_uint64()
        w = words_cat.contiguous()
        self._check(self.L.nice_band_assemble(self.ctx.ptr, self._st(), ctypes.c_void_p(w.data_ptr()), b0, bb, R,
                                              ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(n)),
                    "nice_band_assemble")
        return out[: n.value]


def _step(fn, *args):
    """Runs a band step; returns (result, 0) or (None, status code)."""
    from . import NiceError
    try:
        return fn(*args), 0
    except NiceError as e:
        return None, int(e.code) if int(e.code) else -1


def _raise_if(err: int, what: str):
    if err:
        from . import NiceError
        raise NiceError(err, what + " (on some rank)")


def encode_sharded(backend, dist, px, px0: int, width: int, height: int, channels: int,
                   channels_out: int | None = None, root: int = 0, device=None):
    """Encode one image across the ranks of the default process group.

    ``px``: this rank's pixels [px0, px0 + len) (a uint8 tensor on the rank's
    device, covering ``band_pixels`` of its ``band_tiles``).  Returns the
    stream (uint8 tensor) on ``root``, None elsewhere.  ``device`` is where
    collective tensors live (the rank's GPU for RCCL, "cpu" for gloo)."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = device if device is not None else px.device
    co = channels if channels_out is None else channels_out
    n = width * height
    lo, hi = band_tiles(width, height, rank, world)
    # 1. edges -> the first coded pixel after this band (+ error word)
    edges, err = _step(backend.classify, px, px0, width, height, channels, co, lo, hi)
    if edges is None:
        edges = torch.full((2,), NONE, dtype=torch.int64)
    mine = torch.cat([edges.to(device=dev, dtype=torch.int64),
                      torch.tensor([err], dtype=torch.int64, device=dev)])
    all_edges = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(all_edges, mine)
    ge = torch.stack(all_edges).cpu()
    _raise_if(int(ge[:, 2].min()), "nice_band_classify")
    later = [int(e[0]) for e in ge[rank + 1:] if int(e[0]) != NONE]
    band_next = later[0] if later else n
    # 2. histogram -> identical tables everywhere (error count in the last slot)
    hist, err = _step(backend.runs, band_next)
    h = torch.zeros(859, dtype=torch.int64, device=dev)
    if hist is not None:
        h[:858] = hist.to(device=dev, dtype=torch.int64)
    h[858] = 1 if err else 0
    dist.all_reduce(h)
    _raise_if(-1 if int(h[858]) else 0, "nice_band_runs")
    res, err = _step(backend.tables, h[:858])
    bits, seed = res if res is not None else (0, 0)
    # 3. bit counts -> offsets
    b = torch.tensor([bits, err], dtype=torch.int64, device=dev)
    all_bits = [torch.empty_like(b) for _ in range(world)]
    dist.all_gather(all_bits, b)
    gb = torch.stack(all_bits).cpu()
    _raise_if(int(gb[:, 1].min()), "nice_band_tables")
    bitss = [int(x) for x in gb[:, 0]]
    bit0s = [seed + sum(bitss[:r]) for r in range(world)]
    words = backend.pack(bit0s[rank], bitss[rank])
    # 4. gather-v of the band words to the root: grouped P2P, all peers at once
    counts = [backend.words(bit0s[r], bitss[r]) for r in range(world)]
    if rank != root:
        if counts[rank]:
            for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, words.to(dev).contiguous(), root)]):
                q.wait()
        return None
    parts, ops = [], []
    for r in range(world):
        if r == rank:
            parts.append(words.to(dev))
        elif counts[r]:
            buf = torch.empty(counts[r], dtype=words.dtype, device=dev)
            ops.append(dist.P2POp(dist.irecv, buf, r))
            parts.append(buf)
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    cat = torch.cat(parts) if parts else words.new_zeros(0)
    return backend.assemble(cat.to(words.device), bit0s, bitss, width, height)


def encode_bands(px, width: int, height: int, channels: int, n_bands: int, device: int = 0,
                 backends: list | None = None):
    """The band C ABI driven in ONE process: ``n_bands`` bands (the split
    ``n_bands`` ranks would use), each with its own context, the exchange steps
    done on the host.  ``px``: the whole image (uint8 cuda tensor).  Returns
    the stream (uint8 cuda tensor), equal to encoding the image whole.
    ``backends``: reuse contexts across calls (a list, filled on first use)."""
    import torch
    from . import _Ctx
    w, h, c, R = width, height, channels, n_bands
    N = w * h
    if backends is None:
        backends = []
    while len(backends) < R:
        be = HipBands(device)
        be.ctx = _Ctx(device)   # a context holds one band's state between the steps
        backends.append(be)
    bands = backends[:R]
    ranges = [band_tiles(w, h, r, R) for r in range(R)]
    firsts = []
    for be, (lo, hi) in zip(bands, ranges):
        p0, p1 = band_pixels(w, h, lo, hi)
        firsts.append(int(be.classify(px[p0 * c: p1 * c], p0, w, h, c, c, lo, hi)[0]))
    hist = None
    for r, be in enumerate(bands):
        later = [f for f in firsts[r + 1:] if f != NONE]
        hr = be.runs(later[0] if later else N)
        hist = hr.clone() if hist is None else hist + hr
    bits, seeds = zip(*[be.tables(hist) for be in bands])
    assert len(set(seeds)) == 1
    bit0s = [seeds[0] + sum(bits[:r]) for r in range(R)]
    words = torch.cat([be.pack(bit0s[r], bits[r]) for r, be in enumerate(bands)])
    return bands[0].assemble(words, bit0s, list(bits), w, h)
