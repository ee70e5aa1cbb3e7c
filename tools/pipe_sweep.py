"""Diagnostic: streamed (host-memory) encode/decode of 4K RGBA frames for
several pipeline shapes.  Usage: pipe_sweep.py TOTAL batch,depth ..."""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
total = int(sys.argv[1])
W, H = 3840, 2160
N = W * H
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, 16, W, H, 1, dev)
for spec in sys.argv[2:]:
    b, d = (int(x) for x in spec.split(","))
    numa = os.environ.get("NUMA", "1") == "1"
    r = bench.streamed(torch, nice, None, dev, px, W, H, 0, 1, total, batch=b, depth=d, numa_local=numa)
    import gc; gc.collect()
    print(f"numa {r['host_numa_node']} batch {b} depth {d}: enc {r['encode_mpix_s']:.0f} "
          f"dec {r['decode_mpix_s']:.0f} MPix/s  pcie {r['pcie_gb_s_per_gpu']}", flush=True)
