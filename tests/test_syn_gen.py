"""The on-device NICE-SYN-v1 generator (tools/libnice_syn.so, used by bench.py
for the measured batch) must equal the oracle's generator byte for byte, so the
benchmark's inputs are the SURVEY.md §8d workload and the CPU baseline times
the same frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(3840, 2160, 4, 1, 3), (333, 77, 3, 9, 2), (17, 5, 4, 4, 1), (1920, 1080, 4, 64, 2)])
def test_syn_gen_matches_oracle(O, shape):
    import torch
    import bench
    w, h, c, seed0, n = shape
    out = torch.empty((n, w * h * c), dtype=torch.uint8, device="cuda")
    import ctypes
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert bench.syn_lib().nice_syn_v1_dev(ctypes.c_void_p(out.data_ptr()), out.stride(0), n, w, h, c, seed0, st) == 0
    got = out.cpu().numpy()
    for f in range(n):
        assert np.array_equal(got[f], O.gen_syn_v1(w, h, c, seed0 + f)), f
