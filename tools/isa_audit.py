"""Diagnostic: per-kernel instruction audit of the device assembly (spill
reloads, quarter-rate multiplies, exec-mask branches, scratch, VALU count),
and the first vmcnt wait after each outermost loop head ("heads=..."): a
vmcnt(0) there in a loop that prefetches its next loads means the compiler
found a path with loads but no counted store behind them, and the wait drains
the prefetch and the stores ("waits").
Usage: python tools/isa_audit.py [source.hip ...]"""
import re, subprocess, sys, os
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
srcs = sys.argv[1:] or ["nice_encode.hip", "nice_decode.hip"]
for src in srcs:
    path = os.path.join(root, "fast-losless-image-compression-format_amd", "csrc", os.path.basename(src))
    asm = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                          "-Wno-unused-function", "--cuda-device-only", "-S", path, "-o", "-"],
                         capture_output=True, text=True, check=True).stdout
    kernels = re.split(r"\n(?=_ZN4nice[A-Za-z0-9_]+:)", asm)
    for k in kernels[1:]:
        name = re.match(r"_ZN4nice\d+([A-Za-z0-9_]+?)E", k)
        body = k.split(".Lfunc_end")[0]
        c = lambda pat: len(re.findall(pat, body, re.M))
        pats = {"valu": r"^\s+v_", "salu": r"^\s+s_", "readlane": r"v_readlane_b32", "writelane": r"v_writelane_b32",
                "mul_lo": r"v_mul_lo_u32|v_mul_hi_u32", "b64": r"v_(lshlrev|lshrrev|ashrrev)_b64|v_cmp_[a-z]+_u64",
                "saveexec": r"s_and_saveexec", "scratch": r"scratch_", "swappc": r"s_swappc"}
        counts = " ".join(f"{k}={c(v)}" for k, v in pats.items())
        lines = body.split("\n")
        heads = []
        for i, l in enumerate(lines):
            if "Loop Header: Depth=1" in l:
                w = next((re.search(r"vmcnt\((\d+)\)", x).group(1) for x in lines[i:i + 40]
                          if re.search(r"s_waitcnt vmcnt\(\d+\)$", x.strip())), "-")
                heads.append(w)
        print(f"{(name.group(1) if name else k[:30]):22s} {counts} heads={','.join(heads) or '-'}")
