"""Diagnostic: encode phase times only (no decode, no output checks) -- for
timing builds with parts of a kernel disabled.  Usage: enc_only.py F [reps]"""
import ctypes, importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
F = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
W, H = 3840, 2160
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, F, W, H, 1, dev)
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
st = torch.empty((F, stride), dtype=torch.uint8, device=dev)
ln = torch.zeros(F, dtype=torch.int64, device=dev)
L = nice.lib()
L.nice_ctx_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.nice_ctx_read_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
L.nice_phase_name.restype = ctypes.c_char_p
ctx = nice._ctx(0)
nice.encode_batch(px, W, H, 4, st, ln)
torch.cuda.synchronize()
L.nice_ctx_set_timing(ctx.ptr, 1)
for _ in range(reps):
    nice.encode_batch(px, W, H, 4, st, ln)
ms = (ctypes.c_double * 32)(); cnt = (ctypes.c_uint32 * 32)()
L.nice_ctx_read_timing(ctx.ptr, ms, cnt)
print({L.nice_phase_name(i).decode(): round(ms[i] / reps, 3) for i in range(32) if cnt[i]}, flush=True)
