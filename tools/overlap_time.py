"""Diagnostic: the bench step (encode then decode of F 4K RGBA SYN-v1 frames)
issued as one sequence on one stream, against the batch split in P parts on P
streams with a context each (part k's encode waits for part k-1's encode:
one part's decode runs beside the next part's encode).  Usage:
overlap_time.py F [reps [P]]"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
F = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
P = int(sys.argv[3]) if len(sys.argv) > 3 else 2
W, H, C = 3840, 2160, 4
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, F, W, H, 1, dev, C)
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
st = torch.empty((F, stride), dtype=torch.uint8, device=dev)
ln = torch.zeros(F, dtype=torch.int64, device=dev)
dec = torch.empty((F, W * H * C), dtype=torch.uint8, device=dev)
status = torch.zeros(F, dtype=torch.int32, device=dev)


def seq():
    nice.encode_batch(px, W, H, C, st, ln)
    nice.decode_batch(st, ln, W, H, C, dec, status)


streams = [torch.cuda.Stream(dev) for _ in range(P)]
ctxs = [nice.Context(0) for _ in range(P)]
cut = [F * k // P for k in range(P + 1)]


def split(stagger):
    main = torch.cuda.current_stream(dev)
    prev = main.record_event()
    evs = []
    for k in range(P):
        s, c, a, b = streams[k], ctxs[k], cut[k], cut[k + 1]
        s.wait_event(prev)
        nice.encode_batch(px[a:b], W, H, C, st[a:b], ln[a:b], stream=s, ctx=c)
        e = s.record_event()
        if stagger:
            prev = e
        evs.append(e)
    for k in range(P):
        s, c, a, b = streams[k], ctxs[k], cut[k], cut[k + 1]
        nice.decode_batch(st[a:b], ln[a:b], W, H, C, dec[a:b], status[a:b], stream=s, ctx=c)
    for s in streams:
        main.wait_stream(s)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for name, fn in [("sequential", seq), (f"split{P} staggered", lambda: split(True)),
                 (f"split{P} concurrent", lambda: split(False)), ("sequential", seq)]:
    dec.zero_()
    ms = timed(fn)
    assert int(status.abs().sum()) == 0
    assert torch.equal(dec, px.reshape(F, -1)), f"{name}: decoded frames differ"
    print(f"{name}: {ms:.2f} ms per step ({F * W * H / ms / 1e6:.2f} GPix/s)", flush=True)
