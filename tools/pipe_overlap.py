"""Diagnostic: F frames per step, sequential (encode all, then decode all, one
stream) vs two half-batches on two streams offset by one encode, so that one
half's decode (latency-bound dec_rows, one block per CU at F/2 = 256) runs
beside the other half's encode.  Usage: NF=512 python tools/pipe_overlap.py"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
nice = importlib.import_module("fast-losless-image-compression-format_amd")
W, H = 3840, 2160
F = int(os.environ.get("NF", 512))
R = int(os.environ.get("REPS", 4))
dev = torch.device("cuda", 0)
px = bench.syn_frames(torch, F, W, H, 1, dev)
N = W * H
stride = (nice.encode_bound(W, H) + 255) // 256 * 256
streams = torch.empty((F, stride), dtype=torch.uint8, device=dev)
lens = torch.zeros(F, dtype=torch.int64, device=dev)
dec = torch.empty((F, N * 4), dtype=torch.uint8, device=dev)
status = torch.zeros(F, dtype=torch.int32, device=dev)
ref_lens = None


def check(tag):
    ok = int(status.abs().sum()) == 0 and torch.equal(dec[::97].view(-1, N, 4)[:, :, :3], px[::97].view(-1, N, 4)[:, :, :3])
    same = ref_lens is None or torch.equal(lens, ref_lens)
    print(f"  {tag}: ok={ok} same_lens={same}", flush=True)


# sequential
s0 = torch.cuda.Stream(dev)
c0 = nice.Context(0)
def seq_step():
    nice.encode_batch(px, W, H, 4, streams, lens, stream=s0, ctx=c0)
    nice.decode_batch(streams, lens, W, H, 4, dec, status, stream=s0, ctx=c0)
seq_step(); torch.cuda.synchronize()
ref_lens = lens.clone()
t0 = time.perf_counter()
for _ in range(R):
    seq_step()
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / R
print(f"sequential: {el*1e3:.1f} ms/step  {F*N/el/1e6:.0f} MPix/s", flush=True)
check("sequential")

# two offset half-batches
half = F // 2
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
ca, cb = nice.Context(0), nice.Context(0)
A, B = slice(0, half), slice(half, F)
def enc(sl, s, c):
    nice.encode_batch(px[sl], W, H, 4, streams[sl], lens[sl], stream=s, ctx=c)
def dcd(sl, s, c):
    nice.decode_batch(streams[sl], lens[sl], W, H, 4, dec[sl], status[sl], stream=s, ctx=c)
for warm in (True, False):
    lens.zero_(); status.fill_(7)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 1 if warm else R
    enc(A, sa, ca)
    ev = torch.cuda.Event()
    ev.record(sa)
    sb.wait_event(ev)
    for r in range(reps):
        if r:
            enc(A, sa, ca)
        dcd(A, sa, ca)
        enc(B, sb, cb)
        dcd(B, sb, cb)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    if not warm:
        print(f"two offset streams: {el*1e3:.1f} ms/step  {F*N/el/1e6:.0f} MPix/s", flush=True)
        check("offset")
