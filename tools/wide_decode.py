"""Diagnostic: encode + decode one very wide RGBA SYN-v1 frame on the GPU (inputs
resident in HBM) and time the decode -- frames wider than 16384 columns go
through the strip-split row kernel in launches of at most CUs / 2 strips.
Usage: wide_decode.py [W H reps]   (default 32768 x 4096, 3 reps)"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
W = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
H = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, 1, W, H, 11, dev)
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
st = torch.empty((1, stride), dtype=torch.uint8, device=dev)
ln = torch.zeros(1, dtype=torch.int64, device=dev)
dec = torch.empty((1, W * H * 4), dtype=torch.uint8, device=dev)
status = torch.zeros(1, dtype=torch.int32, device=dev)
nice.encode_batch(px, W, H, 4, st, ln)
nice.decode_batch(st, ln, W, H, 4, dec, status)   # sizes the scratch
torch.cuda.synchronize()
assert int(status[0]) == 0
exact = bool(torch.equal(dec.view(-1, 4)[:, :3], px.view(-1, 4)[:, :3]))
t = []
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nice.decode_batch(st, ln, W, H, 4, dec, status)
    torch.cuda.synchronize()
    t.append(time.perf_counter() - t0)
print(f"{W}x{H} RGBA: stream {int(ln[0])} bytes, decode {min(t) * 1e3:.1f} ms "
      f"({W * H / min(t) / 1e6:.0f} MPix/s, {min(t) / H * 1e6:.1f} us per row), round trip exact: {exact}")
