"""Diagnostic: encode N 4K RGBA SYN-v1 frames through the device batch path."""
import importlib, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
nice = importlib.import_module("fast-losless-image-compression-format_amd")
from oracle import oracle as O
w, h, n = 3840, 2160, int(os.environ.get("NF", 8))
frames = np.stack([O.gen_syn_v1(w, h, 4, s) for s in range(1, n + 1)])
px = torch.from_numpy(frames).cuda()
bound = (nice.encode_bound(w, h) + 255) // 256 * 256
out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
lens = torch.zeros(n, dtype=torch.int64, device="cuda")
for _ in range(2):
    nice.encode_batch(px, w, h, 4, out, lens)
torch.cuda.synchronize()
print("enc ok", int(lens[0]) == len(O.encode(frames[0], w, h, 4)))
