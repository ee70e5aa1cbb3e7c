"""nice_decode_batch_dev is host-asynchronous: the parse reaches its fixpoint
on the device (queued sync iterations, then dec_sync_settle for frames still
changing, code.rs:573-684 being a serial parse), so the call returns as soon
as the decode is queued.  A torch event recorded right after the call must
still be pending for a 64-frame 4K batch, and the pixels must be exact; with
host lengths (nice_decode_batch_dev_hl) the call does not even wait for the
encode queued before it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _batch(nice, O, n, w, h, c):
    import torch
    frames = np.stack([O.gen_syn_v1(w, h, c, s) for s in range(1, n + 1)])
    px = torch.from_numpy(frames).cuda()
    bound = (nice.encode_bound(w, h) + 255) // 256 * 256
    out = torch.zeros((n, bound), dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int64, device="cuda")
    return frames, px, out, lens


@pytest.mark.parametrize("host_len", [False, True])
def test_decode_batch_returns_before_gpu(nice, O, host_len):
    import torch
    w, h, c, n = 3840, 2160, 4, 64
    frames, px, out, lens = _batch(nice, O, n, w, h, c)
    nice.encode_batch(px, w, h, c, out, lens)
    hl = lens.cpu().tolist() if host_len else None
    if host_len:
        nice.encode_batch(px, w, h, c, out, lens)   # queued again: the decode must not wait for it
    dec = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    nice.decode_batch(out, lens, w, h, 4, dec, status, host_len=hl)
    ev = torch.cuda.Event()
    ev.record()
    pending = not ev.query()
    torch.cuda.synchronize()
    assert pending, "decode_batch waited for the GPU"
    assert (status.cpu().numpy() == 0).all()
    assert torch.equal(dec.view(n, -1, 4)[:, :, :3], px.view(n, -1, 4)[:, :, :3])


@pytest.mark.parametrize("queued", ["1", "2"])
def test_device_settle(nice, O, queued, monkeypatch):
    """Too few queued iterations for the batch to settle: the device settle
    finds the fixpoint (frames of different content settle differently)."""
    import torch
    monkeypatch.setenv("NICE_DEC_SYNC_QUEUED", queued)
    monkeypatch.setenv("NICE_DEC_SLICE_BITS", "1024")
    w, h, c, n = 1280, 720, 4, 6
    frames, px, out, lens = _batch(nice, O, n, w, h, c)
    nice.encode_batch(px, w, h, c, out, lens)
    dec = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    nice.decode_batch(out, lens, w, h, 4, dec, status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert torch.equal(dec.view(n, -1, 4)[:, :, :3], px.view(n, -1, 4)[:, :, :3])
