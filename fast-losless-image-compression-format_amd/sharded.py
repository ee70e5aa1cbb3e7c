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

Steps 1-3 stay on the device: the next band's first coded pixel is reduced
on the GPU and read by ``nice_band_runs_dev``, the summed histogram goes
straight to ``nice_band_tables_dev``, whose bit count is gathered as a device
tensor.  The host reads once, after step 3 (the word counts of step 4 size
its buffers).

A band step that fails on one rank (a NiceError from the C ABI, raised before
anything is queued) is carried as an error word through every later exchange;
the rank keeps taking part with empty results, so every rank raises together
after step 3 (or, for the pack, after step 4) instead of waiting in a
collective.

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
    """Band steps on the GPU through the C ABI (include/nice.h).  Results stay
    on the device; nothing here waits for the GPU."""

    def __init__(self, device: int = 0):
        from . import _ctx, lib
        self.L = lib()
        self.ctx = _ctx(device)
        self.device = device
        L = self.L
        vp, u8, u32, u64 = ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64
        L.nice_band_classify.argtypes = [vp, vp, vp, u64, u64, u32, u32, u8, u8, u32, u32, vp]
        L.nice_band_runs_dev.argtypes = [vp, vp, vp, vp]
        L.nice_band_tables_dev.argtypes = [vp, vp, vp, vp]
        L.nice_band_words.argtypes = [u64, u64]
        L.nice_band_words.restype = u64
        L.nice_band_pack_bits.argtypes = [vp, vp, u64, u64, vp, u64]
        L.nice_band_assemble.argtypes = [vp, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64), u32, vp, u64,
                                         ctypes.POINTER(u64)]

    def _st(self):
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, rc, what):
        from . import NiceError
        if rc != 0:
            raise NiceError(rc, what)

    def _dev(self):
        return f"cuda:{self.device}"

    def classify(self, px, px0, width, height, channels, channels_out, lo, hi):
        """{first, last} coded pixel of the band (int64 device tensor, NONE: none)."""
        import torch
        edges = torch.empty(2, dtype=torch.int32, device=px.device)
        self._check(self.L.nice_band_classify(self.ctx.ptr, self._st(), ctypes.c_void_p(px.data_ptr()), px0,
                                              px.numel() // channels, width, height, channels, channels_out,
                                              lo, hi, ctypes.c_void_p(edges.data_ptr())), "nice_band_classify")
        return edges.to(torch.int64) & NONE

    def runs(self, band_next):
        """The band's histogram (858 x int32, device); ``band_next``: a 0-d
        integer tensor (any device) or an int."""
        import torch
        bn = torch.as_tensor(band_next).reshape(1).to(device=self._dev(), dtype=torch.int32)
        hist = torch.empty(858, dtype=torch.int32, device=self._dev())
        self._bn = bn   # kept alive until the kernel has read it (stream order)
        self._check(self.L.nice_band_runs_dev(self.ctx.ptr, self._st(), ctypes.c_void_p(bn.data_ptr()),
                                              ctypes.c_void_p(hist.data_ptr())), "nice_band_runs_dev")
        return hist

    def tables(self, hist_total):
        """Builds the tables; returns {band bits, data start bit} as an int64
        device tensor."""
        import torch
        # the C ABI reads the histogram on this rank's GPU (gloo reduces on the host)
        h = hist_total.to(device=self._dev(), dtype=torch.int32).contiguous()
        info = torch.empty(2, dtype=torch.int64, device=self._dev())
        self._h = h
        self._info = info   # alive until the call has copied it (stream order)
        self._check(self.L.nice_band_tables_dev(self.ctx.ptr, self._st(), ctypes.c_void_p(h.data_ptr()),
                                                ctypes.c_void_p(info.data_ptr())), "nice_band_tables_dev")
        return info

    def words(self, bit0, bits):
        return int(self.L.nice_band_words(bit0, bits))

    def pack(self, bit0, bits, out=None):
        """The band's words (``words(bit0, bits)`` int32, device); into ``out``
        when given."""
        import torch
        n = self.words(bit0, bits)
        if out is None:
            out = torch.empty(max(n, 1), dtype=torch.int32, device=self._dev())
        self._check(self.L.nice_band_pack_bits(self.ctx.ptr, self._st(), bit0, bits,
                                               ctypes.c_void_p(out.data_ptr()), n), "nice_band_pack_bits")
        return out[:n]

    def assemble(self, words_cat, bit0s, bitss, width, height):
        import torch
        from . import encode_bound
        R = len(bit0s)
        cap = encode_bound(width, height)
        out = torch.empty((cap + 3) // 4 * 4, dtype=torch.uint8, device=self._dev())
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


STEPS = ("nice_band_classify", "nice_band_runs", "nice_band_tables", "nice_band_pack")


def band_next_of(firsts, n: int):
    """For each band, the first coded pixel of the bands after it (``n``: none):
    a suffix minimum over the bands' first coded pixels (int64 tensor, NONE
    for a band without one), on the tensor's device."""
    import torch
    f = torch.where(firsts == NONE, torch.full_like(firsts, n), firsts)
    nxt = torch.cat([f[1:], f.new_full((1,), n)])
    return torch.flip(torch.cummin(torch.flip(nxt, [0]), 0).values, [0])


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
    err, err_step = 0, 0

    def note(e, k):
        nonlocal err, err_step
        if e and not err:
            err, err_step = e, k

    # 1. edges -> the first coded pixel after this band, reduced on the device
    edges, e = _step(backend.classify, px, px0, width, height, channels, co, lo, hi)
    note(e, 0)
    if edges is None:
        edges = torch.full((2,), NONE, dtype=torch.int64)
    mine = edges.to(device=dev, dtype=torch.int64)
    all_edges = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(all_edges, mine)
    band_next = band_next_of(torch.stack(all_edges)[:, 0], n)[rank]
    # 2. histogram -> identical tables everywhere
    hist, e = _step(backend.runs, band_next)
    note(e, 1)
    h = torch.zeros(858, dtype=torch.int64, device=dev)
    if hist is not None:
        h += hist.to(device=dev, dtype=torch.int64)
    dist.all_reduce(h)
    info, e = _step(backend.tables, h)
    note(e, 2)
    # 3. bit counts -> offsets (+ every rank's error word): the one host read
    b = torch.zeros(4, dtype=torch.int64, device=dev)
    if info is not None:
        b[:2] = info.to(device=dev, dtype=torch.int64)
    b[2:] = torch.tensor([err, err_step], dtype=torch.int64).to(dev)
    all_bits = [torch.empty_like(b) for _ in range(world)]
    dist.all_gather(all_bits, b)
    gb = torch.stack(all_bits).cpu()
    bad = [r for r in range(world) if int(gb[r, 2])]
    if bad:
        _raise_if(int(gb[bad[0], 2]), STEPS[int(gb[bad[0], 3])])
    bitss = [int(x) for x in gb[:, 0]]
    seed = int(gb[0, 1])
    bit0s = [seed + sum(bitss[:r]) for r in range(world)]
    words, e = _step(backend.pack, bit0s[rank], bitss[rank])
    # 4. gather-v of the band words to the root: grouped P2P, all peers at once;
    # a rank whose pack failed sends zeros of the agreed size, then the error
    # words are reduced so every rank raises together
    counts = [backend.words(bit0s[r], bitss[r]) for r in range(world)]
    if words is None:
        words = torch.zeros(counts[rank], dtype=torch.int32, device=dev)
    if rank != root:
        if counts[rank]:
            for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, words.to(dev).contiguous(), root)]):
                q.wait()
    else:
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
    pe = torch.tensor([e], dtype=torch.int64).to(dev)
    dist.all_reduce(pe, op=dist.ReduceOp.MIN)   # NiceError codes are negative
    _raise_if(int(pe), STEPS[3])
    if rank != root:
        return None
    cat = torch.cat(parts) if parts else words.new_zeros(0)
    return backend.assemble(cat.to(words.device), bit0s, bitss, width, height)


def encode_bands(px, width: int, height: int, channels: int, n_bands: int, device: int = 0,
                 backends: list | None = None, streams: list | None = None, ranges: list | None = None,
                 stats: dict | None = None):
    """The band C ABI driven in ONE process: ``n_bands`` bands (the split
    ``n_bands`` ranks would use), each with its own context and HIP stream so
    the bands' kernels overlap on the GPU; the exchanges are device tensor ops
    with one host read (the bit counts).  ``px``: the whole image (uint8 cuda
    tensor).  Returns the stream (uint8 cuda tensor), equal to encoding the
    image whole.  ``backends``/``streams``: reuse across calls (lists, filled
    on first use).  ``ranges``: the bands' tile ranges (default: the even
    split of ``band_tiles``).  ``stats``: if a dict, receives "bit0s", "bits"
    and "deferred" (bands whose trailer holds a deferred wrapped write)."""
    import torch
    from . import _Ctx
    w, h, c, R = width, height, channels, n_bands
    N = w * h
    if backends is None:
        backends = []
    if streams is None:
        streams = []
    while len(backends) < R:
        be = HipBands(device)
        be.ctx = _Ctx(device)   # a context holds one band's state between the steps
        backends.append(be)
    while len(streams) < R:
        streams.append(torch.cuda.Stream(device))
    bands, sts = backends[:R], streams[:R]
    main = torch.cuda.current_stream(device)
    if ranges is None:
        ranges = [band_tiles(w, h, r, R) for r in range(R)]
    assert len(ranges) == R
    edges = []
    for be, st, (lo, hi) in zip(bands, sts, ranges):
        st.wait_stream(main)
        with torch.cuda.stream(st):
            p0, p1 = band_pixels(w, h, lo, hi)
            edges.append(be.classify(px[p0 * c: p1 * c], p0, w, h, c, c, lo, hi))
    for st in sts:
        main.wait_stream(st)
    nxt = band_next_of(torch.stack(edges)[:, 0], N).to(torch.int32)
    hists = []
    for r, (be, st) in enumerate(zip(bands, sts)):
        st.wait_stream(main)
        with torch.cuda.stream(st):
            hists.append(be.runs(nxt[r]))
    for st in sts:
        main.wait_stream(st)
    hist = torch.stack(hists).sum(0, dtype=torch.int32)
    infos = []
    for be, st in zip(bands, sts):
        st.wait_stream(main)
        with torch.cuda.stream(st):
            infos.append(be.tables(hist))
    for st in sts:
        main.wait_stream(st)
    info = torch.stack(infos).cpu()   # the one host read
    bits = [int(x) for x in info[:, 0]]
    seed = int(info[0, 1])
    bit0s = [seed + sum(bits[:r]) for r in range(R)]
    counts = [bands[0].words(bit0s[r], bits[r]) for r in range(R)]
    words = torch.empty(max(sum(counts), 1), dtype=torch.int32, device=px.device)
    off = 0
    for r, (be, st) in enumerate(zip(bands, sts)):
        st.wait_stream(main)
        with torch.cuda.stream(st):
            be.pack(bit0s[r], bits[r], words[off: off + counts[r]])
        off += counts[r]
    for st in sts:
        main.wait_stream(st)
    if stats is not None:
        ends = [sum(counts[: r + 1]) for r in range(R)]
        stats.update(bit0s=bit0s, bits=bits, deferred=[r for r in range(R) if counts[r] and
                                                         int(words[ends[r] - 2]) & 0x80000000])
    return bands[0].assemble(words[:off], bit0s, bits, w, h)
