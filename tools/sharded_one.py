"""Diagnostic: bench.sharded_image with a one-rank RCCL group (config 4 path on one GPU)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import bench
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29571")
os.environ.setdefault("RANK", "0"); os.environ.setdefault("WORLD_SIZE", "1")
dist.init_process_group("nccl")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
nice = importlib.import_module(bench.PKG)
side = int(os.environ.get("SIDE", 16384))
print(bench.sharded_image(torch, nice, dist, dev, side, 0, 1))
dist.destroy_process_group()
