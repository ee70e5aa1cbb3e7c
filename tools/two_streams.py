"""Diagnostic: one step of F frames as 1 stream vs S concurrent streams of F/S frames."""
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
for S in (1, 2, 4):
    sts = [torch.cuda.Stream(dev) for _ in range(S)]
    ctxs = [nice.Context(0) for _ in range(S)]
    per = F // S
    def step():
        for k in range(S):
            sl = slice(k * per, (k + 1) * per)
            with torch.cuda.stream(sts[k]):
                nice.encode_batch(px[sl], W, H, 4, streams[sl], lens[sl], stream=sts[k], ctx=ctxs[k])
                nice.decode_batch(streams[sl], lens[sl], W, H, 4, dec[sl], status[sl], stream=sts[k], ctx=ctxs[k])
    step(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 3
    ok = int(status.abs().sum()) == 0 and torch.equal(dec[:2].view(2, N, 4)[:, :, :3], px[:2].view(2, N, 4)[:, :, :3])
    print(f"S={S}: {el*1e3:.1f} ms/step  {F*N/el/1e6:.0f} MPix/s ok={ok}", flush=True)
    del ctxs
