"""nice_decode_batch_dev is host-asynchronous: the parse reaches its fixpoint
on the device (queued sync iterations, then dec_sync_settle for frames still
changing, code.rs:573-684 being a serial parse), so the call returns as soon
as the decode is queued.  A torch event recorded right after the call must
still be pending for a 64-frame 4K batch, and the pixels must be exact; with
host lengths (nice_decode_batch_dev_hl) the call does not even wait for the
encode queued before it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _batch(nice, O, n, w, h, c):
    import torch
    frames = np.stack([O.gen_syn_v1(w, h, c, s) for s in range(1, n + 1)])
    px = torch.from_numpy(frames).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    return frames, px, out, lens


@pytest.mark.parametrize("host_len", [False, True])
def test_decode_batch_returns_before_gpu(nice, O, host_len):
    import torch
    w, h, c, n = 3840, 2160, 4, 64
    frames, px, out, lens = _batch(nice, O, n, w, h, c)
    nice.encode_batch(px, w, h, c, out, lens)
    hl = lens.cpu().tolist() if host_len else None
    if host_len:
        nice.encode_batch(px, w, h, c, out, lens)   # queued again: the decode must not wait for it
    dec = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    nice.decode_batch(out, lens, w, h, 4, dec, status, host_len=hl)
    ev = torch.cuda.Event()
    ev.record()
    pending = not ev.query()
    torch.cuda.synchronize()
    assert pending, "decode_batch waited for the GPU"
    assert (status.cpu().numpy() == 0).all()
    assert torch.equal(dec.view(n, -1, 4)[:, :, :3], px.view(n, -1, 4)[:, :, :3])


@pytest.mark.parametrize("queued", ["1", "2"])
def test_device_settle(nice, O, queued, opts):
    """Too few queued iterations for the batch to settle: the device settle
    finds the fixpoint (frames of different content settle differently)."""
    import torch
    opts.setenv("NICE_DEC_SYNC_QUEUED", queued)
    opts.setenv("NICE_DEC_SLICE_BITS", "1024")
    w, h, c, n = 1280, 720, 4, 6
    frames, px, out, lens = _batch(nice, O, n, w, h, c)
    nice.encode_batch(px, w, h, c, out, lens)
    dec = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    nice.decode_batch(out, lens, w, h, 4, dec, status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert torch.equal(dec.view(n, -1, 4)[:, :, :3], px.view(n, -1, 4)[:, :, :3])


def test_host_len_mismatch(nice, O):
    """host lengths size the slice scratch.  A host list
    of the wrong length is refused; a host length shorter than the device's
    fails the frame (NICE_E_ARG) before any slice is written past the scratch."""
    import torch
    w, h, c, n = 640, 360, 4, 3
    frames, px, out, lens = _batch(nice, O, n, w, h, c)
    nice.encode_batch(px, w, h, c, out, lens)
    hl = lens.cpu().tolist()
    dec = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    with pytest.raises(nice.NiceError):
        nice.decode_batch(out, lens, w, h, 4, dec, status, host_len=hl[:-1])
    # every host length far below the device's: the scratch is sized for one
    # slice per frame, so every frame must fail instead of writing past it
    nice.decode_batch(out, lens, w, h, 4, dec, status, host_len=[64] * n)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == -1).all(), status
    # and the context decodes the same streams exactly afterwards
    nice.decode_batch(out, lens, w, h, 4, dec, status, host_len=hl)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert torch.equal(dec.view(n, -1, 4)[:, :, :3], px.view(n, -1, 4)[:, :, :3])


def _time_decode(nice, s, runs=3):
    import time
    import torch
    w = int.from_bytes(s[4:8], "big")
    h = int.from_bytes(s[8:12], "big")
    c = s[12]
    dev = torch.device("cuda", 0)
    st = torch.from_numpy(np.frombuffer(s + bytes(-len(s) % 256), np.uint8).copy()).view(1, -1).to(dev)
    ln = torch.tensor([len(s)], dtype=torch.int64, device=dev)
    out = torch.zeros((1, w * h * c), dtype=torch.uint8, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    ts = []
    for _ in range(runs + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nice.decode_batch(st, ln, w, h, c, out, status, host_len=[len(s)])
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    assert int(status[0]) == 0
    return sorted(ts[1:])[runs // 2], out[0].cpu().numpy()


def test_settle_slow_sync_stream(nice, O, opts, capfd):
    """a stream that needs more Jacobi iterations than are
    queued (8).  tests/crafted_streams.make_slow_sync: zero-residual RGB
    pixels are 25 zero bits, so a parse that starts at the wrong bit stays
    there until a rare SMALL_DIFF pixel moves it (re-synchronisation after
    ~7 K bits on average, ~34 K at worst: ~35 iterations of 1 K-bit slices).
    The device settle (ranges of slices per lane, consistent slices skipped)
    must decode it exactly, in at most 5x the time of an ordinary stream of
    the same shape, and the last queued iteration must still have been moving
    (so the settle, not the queue, reached the fixpoint)."""
    import crafted_streams as C
    W, H = 512, 512
    s = C.make_slow_sync(O, 5, W, H)
    ref = O.decode(s)[0]
    opts.setenv("NICE_DEC_SLICE_BITS", 1024)
    opts.setenv("NICE_DEC_STATS", 1)
    got = np.frombuffer(nice.decode_bytes(s)[0], np.uint8)
    assert np.array_equal(got, ref)
    err = capfd.readouterr().err
    line = [l for l in err.splitlines() if "sync iterations that changed an entry" in l][-1]
    flags = [int(x) for x in line.split(":")[1].split("(")[0].split()]
    queued = int(line.split("(queued")[1].split(",")[0])
    assert flags[queued - 1] == 1 and flags[16] == 1 and flags[17] == 0, line   # last queued moved; settled; final still
    opts.delenv("NICE_DEC_STATS")
    t_slow, px = _time_decode(nice, s)
    assert np.array_equal(px.reshape(-1), ref)
    normal = O.encode(O.gen_syn_v1(W, H, 3, 5), W, H, 3)
    t_norm, _ = _time_decode(nice, normal)
    print(f"slow-sync decode {t_slow * 1e3:.2f} ms, ordinary {t_norm * 1e3:.2f} ms")
    assert t_slow <= 5 * t_norm, (t_slow, t_norm)


def test_settle_4k_few_queued(nice, O, opts):
    """one 4K SYN-v1 frame with 1 K-bit slices needs 5
    Jacobi iterations; with 4 queued, the settle finishes it (round 5's serial
    settle took 3.3 s) -- exactly, and within 30 ms."""
    W, H = 3840, 2160
    px = O.gen_syn_v1(W, H, 4, 1)
    s = O.encode(px, W, H, 4)
    opts.setenv("NICE_DEC_SYNC_QUEUED", 4)
    opts.setenv("NICE_DEC_SLICE_BITS", 1024)
    t, out = _time_decode(nice, s)
    assert np.array_equal(out.reshape(-1, 4)[:, :3], px.reshape(-1, 4)[:, :3])
    print(f"4K frame, 4 queued iterations: {t * 1e3:.2f} ms")
    assert t <= 0.030, t
