"""Diagnostic: encode + decode time per phase for N device-generated 4K frames,
and a digest of the streams (A/B builds via NICE_LIB_PATH must agree)."""
import ctypes, hashlib, importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import opts as _opts  # noqa: E402
_opts.apply_env(nice)
W, H, n = 3840, 2160, int(os.environ.get("NF", 256))
tag = os.environ.get("NICE_LIB_PATH", "in-tree")
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, n, W, H, 1, dev)
bound = (nice.encode_bound(W, H) + 255) // 256 * 256
out = torch.zeros((n, bound), dtype=torch.uint8, device=dev)
lens = torch.zeros(n, dtype=torch.int64, device=dev)
dec = torch.empty((n, W * H * 4), dtype=torch.uint8, device=dev)
st = torch.zeros(n, dtype=torch.int32, device=dev)
L = nice.lib()
L.nice_ctx_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.nice_ctx_read_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
L.nice_phase_name.restype = ctypes.c_char_p
nice.encode_batch(px, W, H, 4, out, lens)
nice.decode_batch(out, lens, W, H, 4, dec, st)
torch.cuda.synchronize()
ok = int(st.abs().sum()) == 0 and torch.equal(dec.view(n, -1, 4)[:, :, :3], px.view(n, -1, 4)[:, :, :3])
h = hashlib.sha256()
for i in range(min(n, 16)):
    h.update(out[i, :int(lens[i])].cpu().numpy().tobytes())
ctx = nice._ctx(0)
L.nice_ctx_set_timing(ctx.ptr, 1)
R = 3
t0 = time.perf_counter()
for _ in range(R):
    nice.encode_batch(px, W, H, 4, out, lens)
torch.cuda.synchronize()
te = (time.perf_counter() - t0) / R
t0 = time.perf_counter()
for _ in range(R):
    nice.decode_batch(out, lens, W, H, 4, dec, st)
torch.cuda.synchronize()
td = (time.perf_counter() - t0) / R
ms = (ctypes.c_double * 32)(); cnt = (ctypes.c_uint32 * 32)()
L.nice_ctx_read_timing(ctx.ptr, ms, cnt)
ph = {L.nice_phase_name(i).decode(): round(ms[i] / R, 2) for i in range(32) if cnt[i]}
print(f"[{tag}] {n} x 4K: encode {te*1e3:.2f} ms decode {td*1e3:.2f} ms ok={ok} "
      f"digest={h.hexdigest()[:16]} {ph}", flush=True)
