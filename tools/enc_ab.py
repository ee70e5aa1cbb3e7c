"""Diagnostic: encoder A/B (ring-staged classify vs window classify): identical
streams and per-phase time on N device-generated 4K frames."""
import ctypes, importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
W, H, n = 3840, 2160, int(os.environ.get("NF", 128))
px = bench.syn_frames(torch, n, W, H, 1, torch.device("cuda", 0))
bound = (nice.encode_bound(W, H) + 255) // 256 * 256
L = nice.lib()
L.nice_ctx_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.nice_ctx_read_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
outs = {}
for mode in ("window", "ring"):
    if mode == "window": os.environ["NICE_ENC_NO_RING"] = "1"
    else: os.environ.pop("NICE_ENC_NO_RING", None)
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    nice.encode_batch(px, W, H, 4, out, lens)
    torch.cuda.synchronize()
    ctx = nice._ctx(0)
    L.nice_ctx_set_timing(ctx.ptr, 1)
    t0 = time.perf_counter()
    for _ in range(3):
        nice.encode_batch(px, W, H, 4, out, lens)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 3
    ms = (ctypes.c_double * 32)(); cnt = (ctypes.c_uint32 * 32)()
    L.nice_ctx_read_timing(ctx.ptr, ms, cnt)
    L.nice_ctx_set_timing(ctx.ptr, 0)
    print(f"encode {n} x 4K {mode}: {el*1e3:.2f} ms; classify {ms[0]/max(cnt[0],1):.2f} ms/launch", flush=True)
    outs[mode] = (out, lens)
same = torch.equal(outs["window"][1], outs["ring"][1]) and all(
    torch.equal(outs["window"][0][i, :int(outs["window"][1][i])], outs["ring"][0][i, :int(outs["ring"][1][i])]) for i in range(n))
print("identical streams:", same)
