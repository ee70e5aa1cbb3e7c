"""The row kernels' spread-form arithmetic after round 5's instruction cuts
(ivs_avg, rows_step, rows_step_exact in nice_decode.hip) equals the forms it
replaced: tools/rows_arith_check.cpp, compiled here with g++ (CPU only)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_rows_arith_equal(tmp_path):
    exe = str(tmp_path / "rows_arith_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", exe,
                           os.path.join(ROOT, "tools", "rows_arith_check.cpp")])
    out = subprocess.run([exe, "3000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "average 0, step 0, exact 0 mismatches" in out.stdout
