#!/usr/bin/env python3
"""Benchmark: NICE2 encode+decode of 4K RGBA frames resident in HBM.

One "step" encodes a batch of F synthetic 3840x2160 RGBA frames on the GPU and
decodes the resulting streams back (steady-state throughput of repeated frames,
SURVEY.md §8d; BASELINE.json metric "encode+decode MPixels/s on 4K RGBA").
Frames are independent, so N GPUs shard frames with no collective ("weak").

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (HIP
events around its launches inside the timed region; algorithmic bytes per
launch) and the CPU baseline (the oracle restatement of the
reference, single thread, on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import ctypes
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "fast-losless-image-compression-format_amd"

HBM_PEAK = 8.0e12          # B/s, MI355X HBM3E (MI355X_MICROARCH.md)
AMP = [0, 1, 2, 3, 8, 24, 64, 256]


_syn = None


def syn_lib():
    """tools/libnice_syn.so: NICE-SYN-v1 generated on the GPU (xorshift32
    jump-ahead), bit-identical to the oracle's gen_syn_v1 (tests/test_syn_gen.py)."""
    global _syn
    if _syn is None:
        _syn = ctypes.CDLL(os.path.join(ROOT, "tools", "libnice_syn.so"))
        _syn.nice_syn_v1_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    return _syn


def syn_frames(torch, n, W, H, seed0, device, channels=4):
    """n NICE-SYN-v1 frames (RGBA, or RGB with channels=3),
    seeds seed0 .. seed0+n-1, generated on `device`: [n, W*H*channels] uint8."""
    out = torch.empty((n, W * H * channels), dtype=torch.uint8, device=device)
    st = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    rc = syn_lib().nice_syn_v1_dev(ctypes.c_void_p(out.data_ptr()), out.stride(0), n, W, H, channels, seed0, st)
    if rc != 0:
        raise RuntimeError(f"nice_syn_v1_dev failed ({rc})")
    return out


def stream_check(O, px, streams, lens, W, H, idx):
    """Byte-compares the GPU streams of frames `idx` of the measured batch with
    the oracle's code::encode of the same pixels (outside the timed region)."""
    L = lens.cpu()
    for i in idx:
        want = O.encode(px[i].cpu().numpy(), W, H, 4)
        got = streams[i, :int(L[i])].cpu().numpy().tobytes()
        if got != want:
            raise AssertionError(f"frame {i}: GPU stream differs from the oracle")
    return f"oracle, {len(idx)} frames of the timed batch (indices {list(idx)}): byte-exact"


def cpu_baseline(W, H, seconds=12.0):
    """Oracle (C restatement of the reference, -O3, 1 thread): encode + decode of
    4K RGBA frames until ~`seconds` of CPU work -- the same frames as the GPU
    batch's first ones (SYN-v1 seeds 1, 2, ...).  Decode runs on the stream's
    channels=3 view (byte 12 patched), the only form the reference decodes."""
    from oracle import oracle as O
    n = 0
    t_total = 0.0
    seed = 1
    while t_total < seconds and n < 64:
        px = O.gen_syn_v1(W, H, 4, seed)
        t0 = time.perf_counter()
        s = O.encode(px, W, H, 4)
        s3 = bytearray(s)
        s3[12] = 3
        O.decode(bytes(s3))
        t_total += time.perf_counter() - t0
        n += 1
        seed += 1
    return {"value": round(n * W * H / t_total / 1e6, 3), "unit": "MPixels/s", "cores": 1,
            "kind": "port",
            "sample": f"{n} x {W}x{H} RGBA NICE-SYN-v1 frames (seeds 1..{n}: frames 0..{n - 1} of the "
                      f"GPU batch), encode+decode, {t_total:.1f} s single-thread"}


def cpu_baseline_threads(W, H, seconds=8.0):
    """The same oracle work frame-parallel on the host's CPU share (SURVEY.md
    §8d: per-image 1-thread time and frame-parallel throughput): one frame per
    thread per round, the C calls release the GIL."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    frames = [O.gen_syn_v1(W, H, 4, seed) for seed in range(1, threads + 1)]

    def work(px):
        s3 = bytearray(O.encode(px, W, H, 4))
        s3[12] = 3
        O.decode(bytes(s3))

    n = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds:
            list(ex.map(work, frames))
            n += threads
    el = time.perf_counter() - t0
    return {"value": round(n * W * H / el / 1e6, 3), "unit": "MPixels/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} x {W}x{H} RGBA NICE-SYN-v1 frames ({threads} distinct, seeds 1..{threads}), "
                      f"encode+decode, {threads} threads, {el:.1f} s"}


def timed_region(step, steps, sync, barrier):
    """Barrier + sync on both sides of exactly `steps` calls of `step`."""
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    return time.perf_counter() - t0


def max_over_ranks(value, dist, device):
    """Whole-job time is the slowest rank's (RCCL all-reduce MAX; gloo in tests)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device="cpu" if dist.get_backend() == "gloo" else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# timing phase -> the kernels that implement it (first match in the PMC summary)
PHASE_KERNELS = {"enc_classify": ["enc_classify_slide0", "enc_classify_slide1", "enc_classify_slide2",
                                  "enc_classify_slide3", "enc_classify_pair_m", "enc_classify_pair",
                                  "enc_classify_ring", "enc_classify"],
                 "enc_tilebits": ["enc_tilebits_hist", "enc_tilebits"],
                 "dec_reconstruct": ["dec_rows_flow", "dec_rows", "dec_rows_wide", "dec_reconstruct"]}


def current_profiles():
    """profiles/CURRENT.json: the counter summaries measured on the committed
    tree ({"tree": git tree hash, "pmc_traffic": file, "pmc_sq": file, ...}),
    so the bench never picks up a mid-round file by name order."""
    try:
        with open(os.path.join(ROOT, "profiles", "CURRENT.json")) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def load_traffic(phase, frames, path=None):
    """Per-launch HBM bytes of the kernel behind `phase` from the committed PMC
    summary (bytes per frame from separate FETCH_SIZE / WRITE_SIZE passes,
    gfx950-corrected; see profiles/README.md), scaled to this launch's frame
    count; None if absent."""
    if path is None:   # the summary profiles/CURRENT.json names
        name = current_profiles().get("pmc_traffic")
        if not name:
            return None, None
        path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    for k in PHASE_KERNELS.get(phase, [phase]):
        if k in d.get("kernels", {}):
            return int(d["kernels"][k]["hbm_bytes_per_frame"] * frames), os.path.basename(path)
    return None, None


SQ_KERNELS = {"classify": ["nice::enc_classify_slide0", "nice::enc_classify_slide1", "nice::enc_classify_slide2",
                           "nice::enc_classify_slide3", "nice::enc_classify_pair_m", "nice::enc_classify_pair",
                           "nice::enc_classify_ring"],
              "pack": ["nice::enc_pack"], "sync": ["nice::dec_sync"], "emit": ["nice::dec_emit"],
              "rundigits": ["nice::enc_rundigits"], "place": ["nice::dec_place"], "rows": ["nice::dec_rows_flow", "nice::dec_rows"]}


def load_sq(px_per_run=32 * 3840 * 2160, path=None):
    """VALU / SALU wave-instructions per pixel, wait share and LDS bank-conflict
    share of the hot kernels, from the newest committed SQ counter passes
    (profiles/pmc_sq_rNN*.txt: tools/pmc_kernel.sh, 32 4K frames per
    dispatch); None if absent."""
    if path is None:   # the passes profiles/CURRENT.json names
        name = current_profiles().get("pmc_sq")
        if not name:
            return None
        path = os.path.join(ROOT, "profiles", name)
    vals = {}
    try:
        with open(path) as fh:
            for line in fh:
                parts = line.split()
                if not parts:
                    continue
                d = vals.setdefault(parts[0], {})
                for kv in parts[1:]:
                    k, _, v = kv.partition("=")
                    try:
                        d[k] = float(v)
                    except ValueError:
                        pass
    except OSError:
        return None
    out = {"source": os.path.basename(path), "pixels_per_dispatch": px_per_run}
    for name, ks in SQ_KERNELS.items():
        d = next((vals[k] for k in ks if k in vals), None)
        if not d or "SQ_INSTS_VALU" not in d:
            continue
        e = {"kernel": next(k for k in ks if k in vals),
             "valu_per_px": round(d["SQ_INSTS_VALU"] / px_per_run, 3)}
        if "SQ_INSTS_SALU" in d:
            e["salu_per_px"] = round(d["SQ_INSTS_SALU"] / px_per_run, 3)
        if "SQ_INSTS_LDS" in d:
            e["lds_per_px"] = round(d["SQ_INSTS_LDS"] / px_per_run, 3)
        if d.get("SQ_ACTIVE_INST_ANY"):
            e["wait_share"] = round(d.get("SQ_WAIT_INST_ANY", 0.0) / d["SQ_ACTIVE_INST_ANY"], 3)
        if d.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_share"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"], 3)
        out[name] = e
    return out


def sharded_image(torch, nice, dist, device, side, rank, world, reps=3):
    """BASELINE config 4: one side x side RGBA image encoded by all ranks
    (bands + RCCL exchanges, fast-losless-image-compression-format_amd/sharded.py)."""
    S = importlib.import_module(PKG + ".sharded")
    W = H = side
    lo, hi = S.band_tiles(W, H, rank, world)
    p0, p1 = S.band_pixels(W, H, lo, hi)
    px = syn_frames(torch, 1, W, H, 11, device).view(-1)[p0 * 4:p1 * 4]
    be = S.HipBands(device.index or 0)
    cdev = "cpu" if dist.get_backend() == "gloo" else None   # where collective tensors live
    out = S.encode_sharded(be, dist, px, p0, W, H, 4, device=cdev)   # warmup
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = S.encode_sharded(be, dist, px, p0, W, H, 4, device=cdev)
    torch.cuda.synchronize()
    dist.barrier()
    el = max_over_ranks((time.perf_counter() - t0) / reps, dist, device)
    return {"workload": f"1 x {W}x{H} RGBA image, bands over {world} ranks, RCCL exchanges + gather-v",
            "ms": round(el * 1e3, 3), "mpix_s": round(W * H / el / 1e6, 2),
            "stream_bytes": int(out.numel()) if out is not None else None}


def config4_one_gpu(torch, nice, device, side, reps=3):
    """BASELINE config 4 on one GPU: the side x side RGBA image (SYN-v1 seed 11)
    encoded whole (one-frame batch) and through the band C ABI in 8 bands in
    this process (the 8-rank split, each band on its own HIP stream, exchanges
    as device tensor ops with one host read); both streams must be identical."""
    S = importlib.import_module(PKG + ".sharded")
    W = H = side
    img = syn_frames(torch, 1, W, H, 11, device)
    bound = (nice.encode_bound(W, H) + 255) // 256 * 256
    out = torch.empty((1, bound), dtype=torch.uint8, device=device)
    ln = torch.zeros(1, dtype=torch.int64, device=device)
    ctx = nice.Context(device.index or 0)
    nice.encode_batch(img, W, H, 4, out, ln, ctx=ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        nice.encode_batch(img, W, H, 4, out, ln, ctx=ctx)
    torch.cuda.synchronize()
    t_whole = (time.perf_counter() - t0) / reps
    flat = img.view(-1)
    bes, sts = [], []
    band = S.encode_bands(flat, W, H, 4, 8, device.index or 0, bes, sts)   # warmup (contexts, scratch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        band = S.encode_bands(flat, W, H, 4, 8, device.index or 0, bes, sts)
    torch.cuda.synchronize()
    t_band = (time.perf_counter() - t0) / reps
    n = int(ln[0])
    same = band.numel() == n and torch.equal(band, out[0, :n])
    # its decode (replicas only across GPUs: one image's rows are one chain;
    # several CUs per image through the strip-split row kernel)
    del band
    dec = torch.empty((1, W * H * 4), dtype=torch.uint8, device=device)
    st = torch.zeros(1, dtype=torch.int32, device=device)
    nice.decode_batch(out, ln, W, H, 4, dec, st, ctx=ctx)
    torch.cuda.synchronize()
    exact = int(st[0]) == 0 and torch.equal(dec.view(-1, 4)[:, :3], img.view(-1, 4)[:, :3])
    t0 = time.perf_counter()
    for _ in range(2):
        nice.decode_batch(out, ln, W, H, 4, dec, st, ctx=ctx)
    torch.cuda.synchronize()
    t_dec = (time.perf_counter() - t0) / 2
    return {"workload": f"1 x {W}x{H} RGBA SYN-v1 image on 1 GPU", "whole_frame_encode_ms": round(t_whole * 1e3, 2),
            "whole_frame_mpix_s": round(W * H / t_whole / 1e6, 1),
            "bands8_one_process_encode_ms": round(t_band * 1e3, 2),
            "band_stream_equals_whole_frame": bool(same), "stream_bytes": n,
            "whole_frame_decode_ms": round(t_dec * 1e3, 1), "decode_round_trip_exact": bool(exact)}


def rgb_leg(torch, nice, device, W, H, F, check, reps=3):
    """4K RGB input (the reference CLI's common case, main.rs:39-41 ->
    code.rs:59-64): F SYN-v1 RGB frames resident in HBM, encode-only and
    decode-only rates; one stream byte-compared with the oracle and the round
    trip checked (outside the timed regions)."""
    N = W * H
    px = syn_frames(torch, F, W, H, 5001, device, channels=3)
    stride = (nice.encode_bound(W, H) + 255) // 256 * 256
    streams = torch.empty((F, stride), dtype=torch.uint8, device=device)
    lens = torch.zeros(F, dtype=torch.int64, device=device)
    dec = torch.empty((F, N * 3), dtype=torch.uint8, device=device)
    status = torch.zeros(F, dtype=torch.int32, device=device)
    enc = lambda: nice.encode_batch(px, W, H, 3, streams, lens)
    dcd = lambda: nice.decode_batch(streams, lens, W, H, 3, dec, status)
    enc()
    dcd()
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0 and torch.equal(dec, px), "RGB round trip"
    exact = None
    if check:
        from oracle import oracle as O
        want = O.encode(px[F - 1].cpu().numpy(), W, H, 3)
        exact = streams[F - 1, :int(lens[F - 1])].cpu().numpy().tobytes() == want
        assert exact, "RGB stream differs from the oracle"

    def timed(fn):
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - a) / reps
    t_e, t_d = timed(enc), timed(dcd)
    return {"workload": f"{F} x {W}x{H} RGB SYN-v1 frames (seeds 5001..), inputs resident in HBM",
            "encode_mpix_s": round(F * N / t_e / 1e6, 1), "decode_mpix_s": round(F * N / t_d / 1e6, 1),
            "encode_decode_mpix_s": round(F * N / (t_e + t_d) / 1e6, 1),
            "bits_per_pixel": round(int(lens.sum()) * 8 / (F * N), 3),
            "stream_check": None if exact is None else "oracle, last frame: byte-exact"}


def batch_leg(torch, nice, device, W, H, F, seed0, check, reps=3, what="config3"):
    """A batch of F W x H RGBA SYN-v1 frames resident in HBM (BASELINE config 3:
    64 x 1920x1080, per-image parallelism on one GPU; also 8K UHD frames):
    encode-only, decode-only and encode-then-decode rates; the last frame's
    stream byte-compared with the oracle and the round trip checked (outside
    the timed regions)."""
    N = W * H
    px = syn_frames(torch, F, W, H, seed0, device)
    stride = (nice.encode_bound(W, H) + 255) // 256 * 256
    streams = torch.empty((F, stride), dtype=torch.uint8, device=device)
    lens = torch.zeros(F, dtype=torch.int64, device=device)
    dec = torch.empty((F, N * 4), dtype=torch.uint8, device=device)
    status = torch.zeros(F, dtype=torch.int32, device=device)
    ctx = nice.Context(device.index or 0)
    enc = lambda: nice.encode_batch(px, W, H, 4, streams, lens, ctx=ctx)
    dcd = lambda: nice.decode_batch(streams, lens, W, H, 4, dec, status, ctx=ctx)
    enc()
    dcd()
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0, f"{what}: decode status"
    assert torch.equal(dec.view(F, N, 4)[:, :, :3], px.view(F, N, 4)[:, :, :3]), f"{what}: round trip"
    exact = None
    if check:
        from oracle import oracle as O
        want = O.encode(px[F - 1].cpu().numpy(), W, H, 4)
        exact = streams[F - 1, :int(lens[F - 1])].cpu().numpy().tobytes() == want
        assert exact, f"{what}: stream differs from the oracle"

    def timed(fn):
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - a) / reps
    t_e, t_d = timed(enc), timed(dcd)
    t_ed = timed(lambda: (enc(), dcd()))
    return {"workload": f"{F} x {W}x{H} RGBA SYN-v1 frames (seeds {seed0}..{seed0 + F - 1}), inputs resident in HBM",
            "encode_mpix_s": round(F * N / t_e / 1e6, 1), "decode_mpix_s": round(F * N / t_d / 1e6, 1),
            "encode_decode_mpix_s": round(F * N / t_ed / 1e6, 1),
            "encode_ms": round(t_e * 1e3, 3), "decode_ms": round(t_d * 1e3, 3),
            "bits_per_pixel": round(int(lens.sum()) * 8 / (F * N), 3),
            "stream_check": None if exact is None else "oracle, last frame: byte-exact, round trip exact"}


def gpu_numa_cpus(torch, device):
    """(NUMA node, its CPUs) of the GPU's PCIe root from sysfs, or (None, None)."""
    try:
        pr = torch.cuda.get_device_properties(device)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as fh:
            node = int(fh.read().strip())
        if node < 0:
            return None, None
        with open(f"/sys/devices/system/node/node{node}/cpulist") as fh:
            spec = fh.read().strip()
        cpus = set()
        for part in spec.split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        return node, cpus & os.sched_getaffinity(0) or None
    except (OSError, ValueError, AttributeError):
        return None, None


def streamed(torch, nice, dist, device, px, W, H, rank, world, total, distinct=16, batch=32, depth=4,
             numa_local=True):
    """BASELINE config 5: `total` 4K RGBA frames streamed from host memory over
    the ranks (total / world each): H2D -> encode -> D2H streams, then H2D
    streams -> decode -> D2H pixels, overlapped over `depth` HIP streams
    (nice_pipe_*).  Host buffers are pinned; the frame list cycles over
    `distinct` of them (every frame is still copied and coded in full)."""
    n = total // world
    N = W * H
    k = min(distinct, px.shape[0])
    # pinned host buffers on the GPU's NUMA node: the host thread runs there
    # while they are allocated (first touch) and while the copies are issued
    node, cpus = gpu_numa_cpus(torch, device) if numa_local else (None, None)
    old_aff = os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, cpus)
    src = [px[i].cpu().pin_memory() for i in range(k)]
    p = nice.Pipeline(W, H, 4, batch=batch, depth=depth, device=device.index or 0)
    outs = [torch.empty(p.stream_stride, dtype=torch.uint8).pin_memory() for _ in range(k)]
    dec = [torch.empty(N * 4, dtype=torch.uint8).pin_memory() for _ in range(k)]
    frames = [src[i % k] for i in range(n)]
    o_list = [outs[i % k] for i in range(n)]
    d_list = [dec[i % k] for i in range(n)]
    warm = min(n, 2 * batch)
    lens = p.encode(frames[:warm], o_list[:warm])
    p.decode(o_list[:warm], lens, d_list[:warm])
    for i in range(k):
        assert torch.equal(dec[i].view(N, 4)[:, :3], src[i].view(N, 4)[:, :3]), "streamed round trip"
    barrier = (lambda: dist.barrier()) if dist is not None else (lambda: None)
    # every timed stream and decoded frame gets a device checksum (nice_pipe_
    # set_checksums, inside the timed run: part of what is measured), checked
    # below against the oracle's stream and the source pixels
    p.checksums(True)
    barrier()
    t0 = time.perf_counter()
    lens = p.encode(frames, o_list)
    t_enc = time.perf_counter() - t0
    enc_sums = p.last_sums
    barrier()
    t1 = time.perf_counter()
    st = p.decode(o_list, lens, d_list)
    t_dec = time.perf_counter() - t1
    dec_sums = p.last_sums
    assert st == [0] * n
    # the timed frames, checked outside the timed regions: every frame's stream
    # checksum equals that of the oracle's stream of its source (all n
    # encodes), every decoded frame's equals its source's, and each decode
    # buffer -- last written by the timed run -- holds its source
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    with ThreadPoolExecutor(min(k, 16)) as ex:   # ctypes calls release the GIL
        want = list(ex.map(lambda j: O.encode(src[j].numpy(), W, H, 4), range(k)))
    want_enc = [nice.checksum64(w) for w in want]
    want_dec = [nice.checksum64(src[j].numpy()) for j in range(k)]
    assert all(lens[i] == len(want[i % k]) for i in range(n)), "streamed: timed stream lengths differ from the oracle's"
    bad = [i for i in range(n) if enc_sums[i] != want_enc[i % k]]
    assert not bad, f"streamed: timed streams {bad[:8]} differ from the oracle's (checksum)"
    bad = [i for i in range(n) if dec_sums[i] != want_dec[i % k]]
    assert not bad, f"streamed: timed decodes {bad[:8]} differ from their sources (checksum)"
    for i in range(k):
        assert torch.equal(dec[i].view(N, 4)[:, :3], src[i].view(N, 4)[:, :3]), "streamed timed round trip"
    t_enc = max_over_ranks(t_enc, dist, device)
    t_dec = max_over_ranks(t_dec, dist, device)
    p.close()
    if cpus:
        os.sched_setaffinity(0, old_aff)
    px_all = n * world * N
    sb = sum(lens[:k]) / k
    return {"workload": f"{n * world} x {W}x{H} RGBA frames from pinned host memory, {n} per GPU, "
                        f"H2D/compute/D2H overlapped ({depth} slots x {batch} frames)",
            "host_numa_node": node,
            "check": f"{n} timed streams checksum-equal (device checksum64, nice.h) to the oracle's stream of "
                     f"their source ({k} distinct); {n} timed decodes checksum-equal to their source pixels; the "
                     f"{k} decode buffers after the timed run byte-equal their sources",
            "encode_mpix_s": round(px_all / t_enc / 1e6, 2),
            "decode_mpix_s": round(px_all / t_dec / 1e6, 2),
            "encode_ms": round(t_enc * 1e3, 2), "decode_ms": round(t_dec * 1e3, 2),
            "pcie_gb_s_per_gpu": {"encode": round(n * (N * 4 + sb) / t_enc / 1e9, 2),
                                  "decode": round(n * (N * 4 + sb) / t_dec / 1e9, 2)}}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(gpus, argv):
    """`--gpus N` with no WORLD_SIZE in the environment: run this script as N
    ranks under torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1) in a CHILD process -- no exec, nothing here has touched the GPU
    -- and return its exit status."""
    import subprocess
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def check_world(gpus):
    """World size from torchrun's environment; it must equal --gpus (a bench
    line's n_gpus is the world size, so a mismatch would mislabel it)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; "
                         f"launch with --nproc-per-node {gpus} or leave WORLD_SIZE unset")
    return world


def standin(args):
    """Tests only (`--standin`, CPU, gloo): the launcher, the rank harness and
    the JSON line of the real bench with a host stand-in step (a fixed amount of
    byte work per rank), so the N>1 plumbing is exercised without a GPU."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = check_world(args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    buf = np.random.default_rng(rank).integers(0, 256, 1 << 20, dtype=np.uint8)
    step = (lambda: int(np.bitwise_xor.reduce(buf)))
    for _ in range(args.warmup):
        step()
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    el = timed_region(step, args.steps, lambda: None, barrier)
    el = max_over_ranks(el, dist if world > 1 else None, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"metric": "standin", "value": round(world * args.steps * buf.size / el / 1e6, 3),
                          "unit": "MB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "scaling": "weak"}))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=512, help="frames per step per GPU")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--streamed-frames", type=int, default=1024,
                    help="config 5: frames streamed from host memory over all ranks (0: skip)")
    ap.add_argument("--sharded-side", type=int, default=16384,
                    help="config 4: one side x side image encoded across the ranks (N>1), or whole and "
                         "in 8 bands on one GPU (N=1) (0: skip)")
    ap.add_argument("--rgb-frames", type=int, default=128,
                    help="4K RGB leg: frames per GPU encoded and decoded (0: skip)")
    ap.add_argument("--config3-frames", type=int, default=64,
                    help="BASELINE config 3 leg: 1920x1080 RGBA frames per GPU (0: skip)")
    ap.add_argument("--uhd8k-frames", type=int, default=16,
                    help="8K UHD leg: 7680x4320 RGBA frames per GPU (0: skip)")
    ap.add_argument("--check-frames", type=int, default=4,
                    help="frames of the timed batch byte-compared with the oracle (rank 0)")
    ap.add_argument("--standin", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.standin:
        return standin(args)

    import torch
    world = check_world(args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # tests only: NICE_DIST_BACKEND=gloo with NICE_ONE_GPU=1 runs every rank on
    # GPU 0 (rehearses the multi-rank legs on a one-GPU box)
    gpu = 0 if os.environ.get("NICE_ONE_GPU") == "1" else local
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        backend = os.environ.get("NICE_DIST_BACKEND", "nccl")
        if backend == "nccl":   # RCCL: bind the group to this rank's GPU (eager init, no device guess)
            dist.init_process_group(backend, device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", gpu)
    torch.cuda.set_device(device)
    nice = importlib.import_module(PKG)
    L = nice.lib()
    L.nice_ctx_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.nice_ctx_read_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_uint32)]
    L.nice_phase_name.restype = ctypes.c_char_p

    W, H, F = args.width, args.height, args.frames
    N = W * H
    px = syn_frames(torch, F, W, H, seed0=1 + rank * F, device=device)
    stride = (nice.encode_bound(W, H) + 255) // 256 * 256
    streams = torch.empty((F, stride), dtype=torch.uint8, device=device)
    lens = torch.zeros(F, dtype=torch.int64, device=device)
    dec = torch.empty((F, N * 4), dtype=torch.uint8, device=device)
    status = torch.zeros(F, dtype=torch.int32, device=device)
    ctx = nice._ctx(gpu)

    def step():
        nice.encode_batch(px, W, H, 4, streams, lens)
        nice.decode_batch(streams, lens, W, H, 4, dec, status)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness of the measured work (outside the timed region)
    assert int(status.abs().sum()) == 0, "decode reported an error"
    for c in range(0, F, 64):   # chunked: a whole-batch RGB slice copy does not fit beside 1024 frames
        assert torch.equal(dec.view(F, N, 4)[c:c + 64, :, :3], px.view(F, N, 4)[c:c + 64, :, :3]), \
            "round trip mismatch"
    stream_bytes = int(lens.sum())
    check = None
    if rank == 0 and args.check_frames > 0:
        from oracle import oracle as O
        k = min(args.check_frames, F)
        idx = sorted({(F - 1) * j // max(k - 1, 1) for j in range(k)})
        check = stream_check(O, px, streams, lens, W, H, idx)

    L.nice_ctx_set_timing(ctx.ptr, 1)
    barrier = (lambda: dist.barrier()) if dist is not None else (lambda: None)
    elapsed = timed_region(step, args.steps, torch.cuda.synchronize, barrier)
    ms = (ctypes.c_double * 32)()
    cnt = (ctypes.c_uint32 * 32)()
    L.nice_ctx_read_timing(ctx.ptr, ms, cnt)
    L.nice_ctx_set_timing(ctx.ptr, 0)
    elapsed = max_over_ranks(elapsed, dist, device)

    # encode-only / decode-only rates (separate short runs, outside the main timing)
    def timed(fn, reps=2):
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - a) / reps
    t_enc = timed(lambda: nice.encode_batch(px, W, H, 4, streams, lens))
    t_dec = timed(lambda: nice.decode_batch(streams, lens, W, H, 4, dec, status))
    # single-frame latency (one 4K frame): encode, decode, encode then decode
    one_px, one_s, one_l = px[:1], streams[:1], lens[:1]
    one_d, one_st = dec[:1], status[:1]
    t_one_enc = timed(lambda: nice.encode_batch(one_px, W, H, 4, one_s, one_l), reps=5)
    t_one_dec = timed(lambda: nice.decode_batch(one_s, one_l, W, H, 4, one_d, one_st), reps=3)
    t_one = timed(lambda: (nice.encode_batch(one_px, W, H, 4, one_s, one_l),
                           nice.decode_batch(one_s, one_l, W, H, 4, one_d, one_st)), reps=2)
    # measured copy peak: device-to-device copy of the frames
    t_copy = timed(lambda: dec.copy_(px), reps=3)
    copy_gb_s = 2 * px.numel() / t_copy / 1e9
    # §8 f4: the 5x5 sub-block position map of one frame (8 B written per index)
    img = nice.Image.new(W, H, 4)
    pos = img.subblock_positions()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(20):
        img.subblock_positions(out=pos)
    ev1.record()
    torch.cuda.synchronize()
    t_pos = ev0.elapsed_time(ev1) / 20 / 1e3
    subblock = {"workload": f"calc_pos_from map of one {W}x{H} frame", "ms": round(t_pos * 1e3, 4),
                "gb_s": round(8 * N / t_pos / 1e9, 1), "frac": round(8 * N / t_pos / HBM_PEAK, 4)}
    del pos

    rgb = None
    if args.rgb_frames:
        try:
            rgb = rgb_leg(torch, nice, device, W, H, args.rgb_frames, rank == 0 and args.check_frames > 0)
        except Exception as exc:   # report, never lose the main measurement
            rgb = {"error": repr(exc)[:300]}
        torch.cuda.empty_cache()

    config3 = None
    if args.config3_frames:
        try:
            config3 = batch_leg(torch, nice, device, 1920, 1080, args.config3_frames, 1 + rank * args.config3_frames,
                                rank == 0 and args.check_frames > 0)
        except Exception as exc:   # report, never lose the main measurement
            config3 = {"error": repr(exc)[:300]}
        torch.cuda.empty_cache()
    uhd8k = None
    if args.uhd8k_frames:
        try:
            uhd8k = batch_leg(torch, nice, device, 7680, 4320, args.uhd8k_frames, 7001 + rank * args.uhd8k_frames,
                              rank == 0 and args.check_frames > 0, what="8k")
        except Exception as exc:   # report, never lose the main measurement
            uhd8k = {"error": repr(exc)[:300]}
        torch.cuda.empty_cache()

    stream_leg = None
    if args.streamed_frames:
        try:
            stream_leg = streamed(torch, nice, dist, device, px, W, H, rank, world, args.streamed_frames)
        except Exception as exc:   # report, never lose the main measurement
            stream_leg = {"error": repr(exc)[:300]}

    sharded = None
    if args.sharded_side:
        del px, streams, dec
        torch.cuda.empty_cache()
        try:
            if world > 1:
                sharded = sharded_image(torch, nice, dist, device, args.sharded_side, rank, world)
            else:
                sharded = config4_one_gpu(torch, nice, device, args.sharded_side)
        except Exception as exc:   # report, never lose the main measurement
            sharded = {"error": repr(exc)[:300]}

    names = [L.nice_phase_name(i).decode() for i in range(32)]
    phase = {names[i]: {"ms_total": round(ms[i], 3), "launches": int(cnt[i])}
             for i in range(32) if cnt[i] and names[i]}
    # dominant kernel and its algorithmic bytes per launch
    in_bytes = F * N * 4
    out_px_bytes = F * N * 4
    algo = {
        "enc_classify": in_bytes, "enc_pack": stream_bytes,
        "dec_sync": stream_bytes, "dec_resync": stream_bytes, "dec_emit": stream_bytes,
        "dec_reconstruct": out_px_bytes,
    }
    dom = max((k for k in phase if k in algo), key=lambda k: phase[k]["ms_total"])
    traffic, traffic_src = load_traffic(dom, F)
    avg_s = phase[dom]["ms_total"] / 1e3 / phase[dom]["launches"]
    achieved = algo[dom] / avg_s / 1e9
    total_px = N * F * args.steps * world
    value = total_px / elapsed / 1e6
    res = {
        "metric": "encode+decode MPixels/s on 4K RGBA at 1/2/4/8 MI355X; bitstream bit-exact",
        "value": round(value, 3),
        "unit": "MPixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: NICE-SYN-v1 RGBA frames (SURVEY.md §8d, seeds 1+rank*F ..), generated on device "
                "bit-identical to the oracle's generator",
        "config": {"workload": f"{F} x {W}x{H} RGBA frames per GPU per step, encode then decode, "
                               f"inputs resident in HBM", "width": W, "height": H,
                   "channels": 4, "frames_per_gpu_per_step": F,
                   "parallelism": f"frames sharded over {world} GPU(s), no collective"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                     "copy_peak_measured": round(copy_gb_s, 1),
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": round(achieved * 1e9 / HBM_PEAK, 5),
                     "traffic": traffic,
                     "traffic_ratio": round(traffic / algo[dom], 3) if traffic else None,
                     "traffic_source": traffic_src,
                     "sq_counters": load_sq(),
                     "algo_bytes_per_launch": algo[dom],
                     "avg_launch_ms": round(avg_s * 1e3, 4)},
        # whole path against HBM: encode (px in + stream out) + decode (stream in + px out)
        "path_roofline_frac": round(2 * (in_bytes + stream_bytes) / (elapsed / args.steps)
                                    / HBM_PEAK * world, 5),
        "encode_mpix_s": round(F * N / t_enc / 1e6, 2),
        "decode_mpix_s": round(F * N / t_dec / 1e6, 2),
        "single_frame_latency_ms": round(t_one * 1e3, 2),
        "single_frame_encode_ms": round(t_one_enc * 1e3, 3),
        "single_frame_decode_ms": round(t_one_dec * 1e3, 3),
        "stream_check": check,
        "subblock_positions": subblock,
        "rgb_4k": rgb,
        "config3_batch_1080p": config3,   # BASELINE config 3
        "uhd8k_7680x4320": uhd8k,
        "stream_bytes_per_frame": stream_bytes // F,
        "bits_per_pixel": round(stream_bytes * 8 / (F * N), 3),
        "phase_ms_timed_region": phase,
        "sharded_image_encode": sharded,   # config 4 (N>1: across ranks; N=1: one GPU)
        "streamed_host_frames": stream_leg,
        "cpu_baseline": None,
        "cpu_baseline_threads": None,
    }
    # rank 0 only, after every GPU leg (at N > 1 the other ranks wait at the
    # final barrier; their GPUs are idle by then)
    if rank == 0 and not args.no_cpu_baseline:
        from oracle import oracle as O
        try:   # the reference's release profile with target-cpu=native
            flags = O.use_native()
        except Exception:
            flags = "gcc -O3 -march=x86-64-v3 (native build failed)"
        res["cpu_baseline"] = cpu_baseline(W, H, args.cpu_seconds)
        res["cpu_baseline_threads"] = cpu_baseline_threads(W, H, min(args.cpu_seconds, 8.0))
        res["cpu_baseline"]["build"] = flags
        res["cpu_baseline_threads"]["build"] = flags
    if rank == 0:
        print(json.dumps(res))
        sys.stdout.flush()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
