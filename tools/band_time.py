"""Times config 4 on one GPU: the 16384^2 image whole and through the band
C ABI in R bands in one process (sharded.encode_bands).  Usage:
python tools/band_time.py [side R reps]"""
import importlib, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import bench
nice = importlib.import_module(bench.PKG)
side = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda:0")
res = bench.config4_one_gpu(torch, nice, dev, side, reps)
print(res)
S = importlib.import_module(bench.PKG + ".sharded")
img = bench.syn_frames(torch, 1, side, side, 11, dev).view(-1)
bes, sts = [], []
S.encode_bands(img, side, side, 4, R, 0, bes, sts)
torch.cuda.synchronize()
for k in range(3):
    t0 = time.perf_counter()
    S.encode_bands(img, side, side, 4, R, 0, bes, sts)
    torch.cuda.synchronize()
    print(f"bands{R} {1e3 * (time.perf_counter() - t0):.2f} ms")
