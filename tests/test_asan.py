"""Host code under ASan + UBSan: the oracle restatement and the
CLI's PNG scanline unfilter, built with gcc -fsanitize=address,undefined and
run on KATs, synthetic / random / long-code frames, every decode mode,
truncated and bit-flipped streams (tests/asan_driver.c)."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG_NAME, ROOT


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="needs gcc")
def test_host_code_asan_ubsan(tmp_path):
    exe = tmp_path / "asan_driver"
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1"]
    objs = []
    for src, cc, std in [(os.path.join(ROOT, "oracle", "nice_oracle.c"), "gcc", "-std=c11"),
                         (os.path.join(ROOT, "tests", "asan_driver.c"), "gcc", "-std=c11"),
                         (os.path.join(ROOT, PKG_NAME, "csrc", "nice_png.cpp"), "g++", "-std=c++17")]:
        o = tmp_path / (os.path.basename(src) + ".o")
        subprocess.run([cc, std, *san, "-c", src, "-o", str(o)], check=True, capture_output=True)
        objs.append(str(o))
    subprocess.run(["g++", *san, *objs, "-o", str(exe)], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), (r.stdout[-2000:], r.stderr[-4000:])
