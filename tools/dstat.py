import sys, importlib, numpy as np, os
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else '.')
nice = importlib.import_module("fast-losless-image-compression-format_amd")
from oracle import oracle as O
for (w,h,seed) in [(3840,2160,1),(1920,1080,2)]:
    px = O.gen_syn_v1(w,h,4,seed)
    s = O.encode(px,w,h,4)
    d,_ = nice.decode_bytes(s)
    print(w,h,'ok', np.array_equal(np.frombuffer(d,np.uint8).reshape(-1,4)[:,:3], px.reshape(-1,4)[:,:3]), flush=True)
