"""Diagnostic: per-phase HIP-event times of encode + decode for a batch of F
RGBA SYN-v1 frames (F=1: single-frame latency).  Usage: phase_time.py F [reps [W H [C]]]
(C = 3: RGB input frames, decoded to RGB)"""
import ctypes, importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import opts as _opts  # noqa: E402
_opts.apply_env(nice)
F = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
W = int(sys.argv[3]) if len(sys.argv) > 4 else 3840
H = int(sys.argv[4]) if len(sys.argv) > 4 else 2160
C = int(sys.argv[5]) if len(sys.argv) > 5 else 4
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, F, W, H, 1, dev, C)
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
st = torch.empty((F, stride), dtype=torch.uint8, device=dev)
ln = torch.zeros(F, dtype=torch.int64, device=dev)
dec = torch.empty((F, W * H * C), dtype=torch.uint8, device=dev)
status = torch.zeros(F, dtype=torch.int32, device=dev)
L = nice.lib()
L.nice_ctx_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.nice_ctx_read_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
L.nice_phase_name.restype = ctypes.c_char_p
ctx = nice._ctx(0)
ENC_ONLY = bool(os.environ.get("NICE_PT_ENC_ONLY"))   # (probe builds whose streams are not valid)
for _ in range(2):
    nice.encode_batch(px, W, H, C, st, ln)
    if not ENC_ONLY:
        nice.decode_batch(st, ln, W, H, C, dec, status)
torch.cuda.synchronize()
assert int(status.abs().sum()) == 0
if not os.environ.get("NICE_PT_NOCHECK") and not ENC_ONLY:   # (timing-only experiment builds)
    assert torch.equal(dec.reshape(F, -1), px.reshape(F, -1)), "decoded frames differ from the input"
for what, fn in [("encode", lambda: nice.encode_batch(px, W, H, C, st, ln)),
                 ("decode", lambda: nice.decode_batch(st, ln, W, H, C, dec, status))][:1 if ENC_ONLY else 2]:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    L.nice_ctx_set_timing(ctx.ptr, 1)
    for _ in range(reps):
        fn()
    ms = (ctypes.c_double * 32)(); cnt = (ctypes.c_uint32 * 32)()
    L.nice_ctx_read_timing(ctx.ptr, ms, cnt)
    L.nice_ctx_set_timing(ctx.ptr, 0)
    ph = {L.nice_phase_name(i).decode(): round(ms[i] / reps, 4) for i in range(32) if cnt[i]}
    print(f"{what} F={F}: wall {wall * 1e3:.3f} ms/call ({F * W * H / wall / 1e9:.2f} GPix/s)  phases(ms): {ph}")
