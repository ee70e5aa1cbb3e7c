"""Diagnostic: encode + decode one batch of F synthetic 4K frames once (for
rocprofv3 counter runs: every dispatch is a batch dispatch)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module(bench.PKG)
F = int(os.environ.get("F", 32))
W, H = 3840, 2160
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, F, W, H, 1, dev)
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
streams = torch.empty((F, stride), dtype=torch.uint8, device=dev)
lens = torch.zeros(F, dtype=torch.int64, device=dev)
dec = torch.empty((F, W * H * 4), dtype=torch.uint8, device=dev)
status = torch.zeros(F, dtype=torch.int32, device=dev)
for _ in range(int(os.environ.get("REPS", 1))):
    nice.encode_batch(px, W, H, 4, streams, lens)
    nice.decode_batch(streams, lens, W, H, 4, dec, status)
torch.cuda.synchronize()
print("ok", bool(torch.equal(dec.view(F, -1, 4)[:, :, :3], px.view(F, -1, 4)[:, :, :3])))
