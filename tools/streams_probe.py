"""Diagnostic: one encode+decode step of F RGBA 4K frames on one stream against
the same frames split into S parts, each on its own stream and context
(concurrent kernels of independent frames).  Usage: streams_probe.py F [S ...]"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
F = int(sys.argv[1]) if len(sys.argv) > 1 else 512
splits = [int(s) for s in sys.argv[2:]] or [1, 2, 4]
W, H = 3840, 2160
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, F, W, H, 1, dev)
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
st = torch.empty((F, stride), dtype=torch.uint8, device=dev)
ln = torch.zeros(F, dtype=torch.int64, device=dev)
dec = torch.empty((F, W * H * 4), dtype=torch.uint8, device=dev)
status = torch.zeros(F, dtype=torch.int32, device=dev)
ctxs = [nice._Ctx(0) for _ in range(max(splits))]
strs = [torch.cuda.Stream(dev) for _ in range(max(splits))]
for S in splits:
    parts = [(F * k // S, F * (k + 1) // S) for k in range(S)]
    def step():
        if S == 1:
            nice.encode_batch(px, W, H, 4, st, ln, ctx=ctxs[0])
            nice.decode_batch(st, ln, W, H, 4, dec, status, ctx=ctxs[0])
            return
        cur = torch.cuda.current_stream(dev)
        for k, (a, b) in enumerate(parts):
            strs[k].wait_stream(cur)
            with torch.cuda.stream(strs[k]):
                nice.encode_batch(px[a:b], W, H, 4, st[a:b], ln[a:b], ctx=ctxs[k])
        for k, (a, b) in enumerate(parts):
            with torch.cuda.stream(strs[k]):
                nice.decode_batch(st[a:b], ln[a:b], W, H, 4, dec[a:b], status[a:b], ctx=ctxs[k])
        for k in range(S):
            cur.wait_stream(strs[k])
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    ok = all(torch.equal(dec.view(F, -1, 4)[c:c + 64, :, :3], px.view(F, -1, 4)[c:c + 64, :, :3]) for c in range(0, F, 64))
    print(f"F={F} streams={S}: {t * 1e3:.2f} ms/step, {F * W * H / t / 1e9:.2f} GPix/s, exact={ok}", flush=True)
