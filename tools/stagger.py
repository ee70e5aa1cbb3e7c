"""Diagnostic: one step of F frames as one encode+decode vs K slices pipelined
over two streams (slice k's encode on the other stream, started when slice
k-1's encode is done, runs beside slice k-1's decode)."""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
W, H = 3840, 2160
F = int(os.environ.get("NF", 512))
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, F, W, H, 1, dev)
N = W * H
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
streams = torch.empty((F, stride), dtype=torch.uint8, device=dev)
lens = torch.zeros(F, dtype=torch.int64, device=dev)
dec = torch.empty((F, N * 4), dtype=torch.uint8, device=dev)
status = torch.zeros(F, dtype=torch.int32, device=dev)
for K in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
    sts = [torch.cuda.Stream(dev) for _ in range(2)]
    ctxs = [nice.Context(0) for _ in range(2)]
    per = F // K
    def step():
        ev = None
        for k in range(K):
            s, c = sts[k % 2], ctxs[k % 2]
            sl = slice(k * per, (k + 1) * per)
            if ev is not None:
                s.wait_event(ev)   # encode of slice k after encode of slice k-1
            nice.encode_batch(px[sl], W, H, 4, streams[sl], lens[sl], stream=s, ctx=c)
            ev = torch.cuda.Event()
            ev.record(s)
            nice.decode_batch(streams[sl], lens[sl], W, H, 4, dec[sl], status[sl], stream=s, ctx=c)
    step(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 3
    ok = int(status.abs().sum()) == 0 and torch.equal(dec[:2].view(2, N, 4)[:, :, :3], px[:2].view(2, N, 4)[:, :, :3])
    print(f"K={K}: {el*1e3:.1f} ms/step  {F*N/el/1e6:.0f} MPix/s ok={ok}", flush=True)
    del ctxs
