"""5x5 sub-block traversal, image.rs:45-102 Image::calc_pos_from.

CPU: the oracle restatement against the reference's own known answers
(image.rs:110-112) and the structure of the map on shapes without leftovers.
GPU: nice_subblock_positions_dev equals the oracle index for index, on shapes
with every combination of width / height leftovers, windows not starting at 0,
indices past the image, and the 32-bit / 64-bit arithmetic paths.
"""
import numpy as np
import pytest


def test_oracle_reference_kat(O):
    # image.rs:110-112: Image::new(4000, 3000, 3); the test divides byte offsets by 3
    assert O.calc_pos_from(4000, 3000, 25) == 48015 // 3
    assert O.calc_pos_from(4000, 3000, 49) == 27 // 3


def test_oracle_structure(O):
    # 10 x 10: block 0 walked top-down, rows alternating; block 1 bottom-up
    m = [O.calc_pos_from(10, 10, i) for i in range(100)]
    assert m[:10] == [0, 1, 2, 3, 4, 14, 13, 12, 11, 10]
    assert m[25:30] == [45, 46, 47, 48, 49]      # block 1 starts on its last row
    assert sorted(m) == list(range(100))
    for w, h in [(5, 5), (15, 10), (20, 3), (4, 3), (1, 9)]:   # at most one leftover: a permutation
        assert sorted(O.calc_pos_from(w, h, i) for i in range(w * h)) == list(range(w * h))


def test_oracle_reference_quirks(O):
    # the reference map is not a bijection when both leftovers are nonzero, and
    # leaves the image for w = 7 (the codec never calls it; we keep it exact)
    assert len({O.calc_pos_from(13, 11, i) for i in range(13 * 11)}) < 13 * 11
    assert max(O.calc_pos_from(7, 2, i) for i in range(14)) == 14


SHAPES = [(4000, 3000), (10, 10), (13, 11), (7, 2), (1, 9), (4, 3), (5, 5), (3840, 2161), (1, 1),
          (17, 4), (1021, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_gpu_positions_match_oracle(nice, O, shape):
    w, h = shape
    img = nice.Image.new(w, h, 3)
    n = w * h
    # whole image, plus a window running 37 indices past its end
    got = img.subblock_positions().cpu().numpy()
    idx = np.unique(np.concatenate([np.arange(min(n, 4096)), np.linspace(0, n - 1, 2048).astype(np.int64),
                                    np.arange(max(n - 256, 0), n)]))
    want = np.array([O.calc_pos_from(w, h, int(i)) for i in idx], np.uint64)
    assert np.array_equal(got[idx].astype(np.uint64), want)
    i0 = max(n - 40, 0)
    want_tail = np.array([O.calc_pos_from(w, h, i0 + k) for k in range(77)], np.uint64)
    tail = img.subblock_positions(i0, 77).cpu().numpy().astype(np.uint64)
    assert np.array_equal(tail, want_tail)
    # an output only 8-byte aligned takes the one-index-per-thread kernel
    import torch
    buf = torch.full((80,), -1, dtype=torch.int64, device="cuda:0")
    img.subblock_positions(i0, 77, out=buf[1:])
    got8 = buf.cpu().numpy()
    assert got8[0] == -1 and (got8[78:] == -1).all()
    assert np.array_equal(got8[1:78].astype(np.uint64), want_tail)


@pytest.mark.gpu
def test_gpu_calc_pos_from_kat(nice):
    img = nice.Image.new(4000, 3000, 3)
    assert img.calc_pos_from(25) == 16005
    assert img.calc_pos_from(49) == 9


@pytest.mark.gpu
def test_gpu_positions_64bit_path(nice, O):
    # indices beyond 2^32 take the 64-bit kernel: 70000 x 70000 = 4.9e9 pixels
    w = h = 70000
    img = nice.Image.new(w, h, 4)
    for i0 in [(1 << 32) - 50, w * h - 100, w * h + 5]:
        got = img.subblock_positions(i0, 200).cpu().numpy().astype(np.uint64)
        want = np.array([O.calc_pos_from(w, h, i0 + k) for k in range(200)], np.uint64)
        assert np.array_equal(got, want), i0


@pytest.mark.gpu
def test_gpu_positions_full_4k_permutation(nice, O):
    # 3840 x 2160 has no height leftover: the map is a permutation of the frame
    import torch
    w, h = 3840, 2160
    pos = nice.Image.new(w, h, 4).subblock_positions()
    torch.cuda.synchronize()
    seen = torch.zeros(w * h, dtype=torch.int32, device=pos.device)
    seen.index_add_(0, pos, torch.ones_like(pos, dtype=torch.int32))
    assert bool((seen == 1).all())
    probe = torch.randint(0, w * h, (512,), generator=torch.Generator().manual_seed(3))
    want = np.array([O.calc_pos_from(w, h, int(i)) for i in probe], np.int64)
    assert np.array_equal(pos[probe.to(pos.device)].cpu().numpy(), want)


@pytest.mark.gpu
def test_gpu_positions_errors(nice):
    with pytest.raises(nice.NiceError):
        nice.Image.new(0, 5, 3).subblock_positions(0, 4)
