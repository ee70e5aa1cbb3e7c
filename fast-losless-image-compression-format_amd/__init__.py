"""MI355X-native NICE2 codec: host-side mirror of the reference codec API.

The reference (Rust, wouter-rombouts/fast-losless-image-compression-format)
exposes its codec path as

* ``image::Image::new(width, height, channels)``          image.rs:22-43
* ``code::encode(input_bytes, image_header, channels_out, output_writer)``
                                                            code.rs:59-64
* ``code::decode(image_reader, channels_out, output_vec) -> Image``
                                                            code.rs:464-468

This package keeps those names and argument meanings and forwards to the C ABI
in ``libnice_hip.so`` (include/nice.h), whose kernels run on the GPU.  There is
no CPU fallback: if the library or a gfx950 device is missing, every call raises.

Device-resident batches (the benchmark path) go through ``encode_batch`` and
``decode_batch`` which take torch tensors already on the GPU.
"""
from __future__ import annotations

import ctypes
import io
import os
from dataclasses import dataclass

__all__ = [
    "Image", "encode", "decode", "encode_bytes", "decode_bytes", "encode_bound",
    "encode_batch", "decode_batch", "Context", "Pipeline", "NiceError", "lib", "LIB_PATH",
    "DEC_STRICT_REFERENCE", "DEC_ALPHA_FILL_FF", "DEC_TOLERANT_HEADER",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# NICE_LIB_PATH: an alternative build of the same library (tools/ A/B timing)
LIB_PATH = os.environ.get("NICE_LIB_PATH") or os.path.join(_HERE, "libnice_hip.so")

OK, E_ARG, E_HIP, E_NODEV, E_CAPACITY, E_FORMAT, E_UNSUPPORTED = 0, -1, -2, -3, -4, -5, -6
_ERRNAMES = {E_ARG: "bad argument", E_HIP: "HIP runtime failure", E_NODEV: "no gfx950 device",
             E_CAPACITY: "output buffer too small",
             E_FORMAT: "malformed stream (the reference decoder would panic)",
             E_UNSUPPORTED: "stream outside the reference decoder's domain"}
DEC_STRICT_REFERENCE = 0x1
DEC_ALPHA_FILL_FF = 0x2
DEC_TOLERANT_HEADER = 0x4   # repair spilled 5-bit max fields (small / flat images)

EXPORTS = [
    "nice_version", "nice_device_count", "nice_encode_bound", "nice_encode", "nice_peek_header",
    "nice_decode", "nice_ctx_create", "nice_ctx_destroy", "nice_ctx_reserve",
    "nice_encode_batch_dev", "nice_decode_batch_dev", "nice_decode_batch_dev_hl",
    "nice_band_classify", "nice_band_runs", "nice_band_tables", "nice_band_words", "nice_band_pack",
    "nice_band_runs_dev", "nice_band_tables_dev", "nice_band_pack_bits",
    "nice_band_assemble", "nice_tile_pixels",
    "nice_pipe_create", "nice_pipe_destroy", "nice_pipe_stream_stride", "nice_pipe_encode",
    "nice_pipe_decode", "nice_pipe_set_checksums",
]


class NiceError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {_ERRNAMES.get(code, 'error')} ({code})")


_lib = None


def lib():
    """Load libnice_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NiceError(E_NODEV, f"{LIB_PATH} missing (run __graft_entry__.build())")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7; load it
    # first so libnice_hip.so binds to the same runtime (same SONAME) and device
    # pointers / streams are shared with torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    u8p = ctypes.c_void_p
    sz = ctypes.c_size_t
    u32 = ctypes.c_uint32
    u64 = ctypes.c_uint64
    L.nice_version.restype = ctypes.c_char_p
    L.nice_encode_bound.restype = sz
    L.nice_encode_bound.argtypes = [u32, u32]
    L.nice_encode.argtypes = [u8p, sz, u32, u32, ctypes.c_uint8, ctypes.c_uint8, u8p, sz,
                              ctypes.POINTER(sz)]
    L.nice_peek_header.argtypes = [u8p, sz, ctypes.POINTER(u32), ctypes.POINTER(u32),
                                   ctypes.POINTER(ctypes.c_uint8)]
    L.nice_decode.argtypes = [u8p, sz, u8p, sz, u32, ctypes.POINTER(sz)]
    L.nice_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.nice_ctx_destroy.argtypes = [ctypes.c_void_p]
    L.nice_ctx_reserve.argtypes = [ctypes.c_void_p, u32, u32, u32]
    L.nice_encode_batch_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u8p, u64, u32, u32, u32,
                                        ctypes.c_uint8, ctypes.c_uint8, u8p, u64, u8p]
    L.nice_decode_batch_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u8p, u64, u8p, u32, u32,
                                        u32, ctypes.c_uint8, u8p, u64, u32, u8p]
    L.nice_decode_batch_dev_hl.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u8p, u64, u8p, ctypes.c_void_p, u32,
                                           u32, u32, ctypes.c_uint8, u8p, u64, u32, u8p]
    L.nice_pipe_create.argtypes = [ctypes.c_int, u32, u32, ctypes.c_uint8, u32, u32,
                                   ctypes.POINTER(ctypes.c_void_p)]
    L.nice_pipe_destroy.argtypes = [ctypes.c_void_p]
    L.nice_pipe_stream_stride.restype = u64
    L.nice_pipe_stream_stride.argtypes = [ctypes.c_void_p]
    L.nice_pipe_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u32, ctypes.c_uint8,
                                   ctypes.c_void_p, u64, ctypes.c_void_p]
    L.nice_pipe_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, u32,
                                   ctypes.c_uint8, ctypes.c_void_p, u32, ctypes.c_void_p]
    L.nice_pipe_set_checksums.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.nice_subblock_positions_dev.argtypes = [ctypes.c_int, ctypes.c_void_p, u32, u32, u64, u64,
                                              ctypes.c_void_p]
    _lib = L
    return L


def _check(rc: int, what: str):
    if rc != OK:
        raise NiceError(rc, what)


@dataclass
class Image:
    """image.rs:5-43 -- only width/height/channels are used on the codec path."""
    width: int
    height: int
    channels: int

    @staticmethod
    def new(width: int, height: int, channels: int) -> "Image":
        return Image(width, height, channels)

    def subblock_positions(self, index0: int = 0, count: int | None = None, device: int = 0, out=None):
        """image.rs:45-102 calc_pos_from for indices [index0, index0 + count)
        (default: the whole image), computed on the GPU into an int64 cuda
        tensor (``out`` or a new one); asynchronous on the current stream."""
        import torch
        n = self.width * self.height - index0 if count is None else count
        if out is None:
            out = torch.empty(max(n, 0), dtype=torch.int64, device=f"cuda:{device}")
        if out.numel() < n or out.dtype != torch.int64 or not out.is_contiguous():
            raise NiceError(E_ARG, "out: contiguous int64 with >= count elements")
        rc = lib().nice_subblock_positions_dev(device, _stream_ptr(torch, out.device), self.width, self.height,
                                               index0, n, ctypes.c_void_p(out.data_ptr()))
        _check(rc, "nice_subblock_positions_dev")
        return out

    def calc_pos_from(self, index: int) -> int:
        """image.rs:45-102: raster position of traversal index ``index``."""
        return int(self.subblock_positions(index, 1)[0])


def encode_bound(width: int, height: int) -> int:
    return int(lib().nice_encode_bound(width, height))


def _as_buffer(data):
    """(ctypes pointer, nbytes, keepalive) for bytes / bytearray / numpy / memoryview."""
    mv = memoryview(data).cast("B")
    if mv.readonly:
        buf = (ctypes.c_uint8 * mv.nbytes).from_buffer_copy(mv)
    else:
        buf = (ctypes.c_uint8 * mv.nbytes).from_buffer(mv)
    return ctypes.cast(buf, ctypes.c_void_p), mv.nbytes, buf


def encode_bytes(input_bytes, width: int, height: int, channels: int,
                 channels_out: int | None = None) -> bytes:
    ptr, n, keep = _as_buffer(input_bytes)
    cap = encode_bound(width, height)
    out = (ctypes.c_uint8 * cap)()
    out_len = ctypes.c_size_t()
    co = channels if channels_out is None else channels_out
    rc = lib().nice_encode(ptr, n, width, height, channels, co, out, cap, ctypes.byref(out_len))
    _check(rc, "nice_encode")
    del keep
    return bytes(out[: out_len.value])


def encode(input_bytes, image_header: Image, channels_out: int, output_writer) -> None:
    """code::encode (code.rs:59-64): appends the stream to ``output_writer``
    (a bytearray, or any object with ``write``)."""
    data = encode_bytes(input_bytes, image_header.width, image_header.height,
                        image_header.channels, channels_out)
    if isinstance(output_writer, bytearray):
        output_writer.extend(data)
    else:
        output_writer.write(data)


def decode_bytes(stream, flags: int = DEC_ALPHA_FILL_FF):
    """Returns (pixels: bytes, Image)."""
    ptr, n, keep = _as_buffer(stream)
    w, h, ch = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint8()
    _check(lib().nice_peek_header(ptr, n, ctypes.byref(w), ctypes.byref(h), ctypes.byref(ch)),
           "nice_peek_header")
    cap = w.value * h.value * max(ch.value, 1)
    out = (ctypes.c_uint8 * max(cap, 1))()
    px_len = ctypes.c_size_t()
    rc = lib().nice_decode(ptr, n, out, cap, flags, ctypes.byref(px_len))
    _check(rc, "nice_decode")
    del keep
    return bytes(out[: px_len.value]), Image(w.value, h.value, ch.value)


def decode(image_reader, channels_out: int, output_vec: bytearray) -> Image:
    """code::decode (code.rs:464-468).  ``channels_out`` is accepted and ignored,
    as in the reference (main.rs:88 passes 3; code.rs never reads it).  The
    output replaces ``output_vec``'s contents."""
    del channels_out
    data = image_reader.read() if hasattr(image_reader, "read") else bytes(image_reader)
    px, img = decode_bytes(data)
    output_vec[:] = px
    return img


# ---- device-resident batches (torch tensors on the GPU) ---------------------
class _Ctx:
    def __init__(self, device: int):
        self.ptr = ctypes.c_void_p()
        _check(lib().nice_ctx_create(device, ctypes.byref(self.ptr)), "nice_ctx_create")

    def __del__(self):
        try:
            if self.ptr:
                lib().nice_ctx_destroy(self.ptr)
        except Exception:
            pass


_ctxs: dict = {}


def _ctx(device: int) -> _Ctx:
    if device not in _ctxs:
        _ctxs[device] = _Ctx(device)
    return _ctxs[device]


def _stream_ptr(torch, device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Context(_Ctx):
    """A device context with its own scratch arena: calls on different torch
    streams need different contexts to run concurrently."""


def encode_batch(px, width: int, height: int, channels: int, out, out_len,
                 channels_out: int | None = None, stream=None, ctx: "_Ctx | None" = None) -> None:
    """Encode ``px`` (uint8 cuda tensor [n_frames, W*H*channels]) into ``out``
    (uint8 cuda tensor [n_frames, stride >= encode_bound]); lengths into
    ``out_len`` (int64 cuda tensor [n_frames]).  Asynchronous on the current
    torch stream (or ``stream``: a torch.cuda.Stream)."""
    import torch
    dev = px.device.index or 0
    n = px.shape[0]
    st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else _stream_ptr(torch, px.device)
    rc = lib().nice_encode_batch_dev(
        (ctx or _ctx(dev)).ptr, st, ctypes.c_void_p(px.data_ptr()), px.stride(0), n, width, height,
        channels, channels if channels_out is None else channels_out,
        ctypes.c_void_p(out.data_ptr()), out.stride(0), ctypes.c_void_p(out_len.data_ptr()))
    _check(rc, "nice_encode_batch_dev")


def decode_batch(streams, stream_len, width: int, height: int, out_channels: int, px, status,
                 flags: int = DEC_ALPHA_FILL_FF, stream=None, ctx: "_Ctx | None" = None,
                 host_len=None) -> None:
    """Decode ``streams`` (uint8 cuda [n, stride]) with byte lengths ``stream_len``
    (int64 cuda [n]) into ``px`` (uint8 cuda [n, >= W*H*out_channels]); per-frame
    status codes into ``status`` (int32 cuda [n]).  Asynchronous: returns once
    the work is queued.  ``host_len`` (the same lengths on the host: a sequence,
    numpy array or CPU tensor) spares the call its one device read (the lengths
    size the scratch), so it never waits for earlier work on the stream."""
    import torch
    dev = streams.device.index or 0
    n = streams.shape[0]
    st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else _stream_ptr(torch, streams.device)
    args = ((ctx or _ctx(dev)).ptr, st, ctypes.c_void_p(streams.data_ptr()), streams.stride(0),
            ctypes.c_void_p(stream_len.data_ptr()))
    tail = (n, width, height, out_channels, ctypes.c_void_p(px.data_ptr()), px.stride(0), flags,
            ctypes.c_void_p(status.data_ptr()))
    if host_len is None:
        rc = lib().nice_decode_batch_dev(*args, *tail)
    else:
        hl_list = [int(x) for x in host_len]
        if len(hl_list) != n:   # a short list would be zero padded: lengths the device does not hold
            raise NiceError(E_ARG, f"host_len has {len(hl_list)} entries for {n} frames")
        hl = (ctypes.c_uint64 * n)(*hl_list)
        rc = lib().nice_decode_batch_dev_hl(*args, ctypes.cast(hl, ctypes.c_void_p), *tail)
    _check(rc, "nice_decode_batch_dev")


def checksum64(buf) -> int:
    """nice_checksum64 (include/nice.h) of a byte buffer, on the host."""
    import numpy as np
    b = np.frombuffer(bytes(buf), np.uint8) if not hasattr(buf, "dtype") else np.asarray(buf, np.uint8).reshape(-1)
    pad = (-b.size) % 4
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    w = b.view("<u4").astype(np.uint64)
    with np.errstate(over="ignore"):
        A = int(w.sum(dtype=np.uint64))
        B = int((w * np.arange(1, w.size + 1, dtype=np.uint64)).sum(dtype=np.uint64))
    return (A + 0x9E3779B97F4A7C15 * B) % (1 << 64)


# ---- streamed host pipeline (config 5: H2D / compute / D2H overlapped) ------
def _host_ptr(buf):
    """Address of a host buffer: numpy array, bytearray or CPU torch tensor."""
    if hasattr(buf, "data_ptr"):
        return buf.data_ptr()
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data
    return ctypes.addressof((ctypes.c_uint8 * len(buf)).from_buffer(buf))


class Pipeline:
    """Streamed encode/decode of host frames (include/nice.h ``nice_pipe_*``):
    ``depth`` slots of ``batch`` frames, each with its own HIP stream, so H2D
    copies, kernels and D2H copies of different slots overlap.  Host buffers
    may be pinned (``torch.empty(..., pin_memory=True)``: asynchronous copies)
    or pageable (numpy / bytearray)."""

    def __init__(self, width: int, height: int, channels: int, batch: int = 16, depth: int = 3,
                 device: int = 0):
        self.width, self.height, self.channels = width, height, channels
        self.ptr = ctypes.c_void_p()
        _check(lib().nice_pipe_create(device, width, height, channels, batch, depth,
                                      ctypes.byref(self.ptr)), "nice_pipe_create")
        self.stream_stride = int(lib().nice_pipe_stream_stride(self.ptr))

    def close(self):
        if self.ptr:
            lib().nice_pipe_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def checksums(self, on: bool = True):
        """From the next call on, encode / decode also record each frame's
        checksum64 (computed on the device; ``last_sums`` after the call)."""
        self._ck = on

    def _sums(self, n, enc):
        if not getattr(self, "_ck", False):
            lib().nice_pipe_set_checksums(self.ptr, None, None)
            return None
        buf = (ctypes.c_uint64 * max(n, 1))()
        _check(lib().nice_pipe_set_checksums(self.ptr, buf if enc else None, None if enc else buf),
               "nice_pipe_set_checksums")
        return buf

    def _sums_done(self, buf, n):
        if buf is not None:
            lib().nice_pipe_set_checksums(self.ptr, None, None)
            self.last_sums = [int(buf[i]) for i in range(n)]

    def encode(self, frames, outs, channels_out: int | None = None):
        """frames[f] -> outs[f] (host buffers of >= stream_stride bytes); returns
        the stream lengths."""
        n = len(frames)
        sums = self._sums(n, True)
        src = (ctypes.c_void_p * max(n, 1))(*[_host_ptr(f) for f in frames])
        dst = (ctypes.c_void_p * max(n, 1))(*[_host_ptr(o) for o in outs])
        caps = [o.numel() if hasattr(o, "numel") else len(o) for o in outs]
        lens = (ctypes.c_uint64 * max(n, 1))()
        co = self.channels if channels_out is None else channels_out
        try:
            rc = lib().nice_pipe_encode(self.ptr, src, n, co, dst, min(caps) if caps else 0, lens)
        finally:   # the pipe must not keep pointing at `sums` once it is freed
            self._sums_done(sums, n)
        _check(rc, "nice_pipe_encode")
        return [int(lens[i]) for i in range(n)]

    def decode(self, streams, lengths, outs, out_channels: int | None = None,
               flags: int = DEC_ALPHA_FILL_FF, raise_on_error: bool = True):
        """streams[f] (lengths[f] bytes) -> outs[f] (W*H*out_channels bytes);
        returns the per-frame statuses.  A frame's error raises NiceError unless
        raise_on_error is False (outs[f] is undefined where status[f] != 0)."""
        n = len(streams)
        sums = self._sums(n, False)
        src = (ctypes.c_void_p * max(n, 1))(*[_host_ptr(s) for s in streams])
        dst = (ctypes.c_void_p * max(n, 1))(*[_host_ptr(o) for o in outs])
        ln = (ctypes.c_uint64 * max(n, 1))(*lengths)
        status = (ctypes.c_int32 * max(n, 1))()
        oc = self.channels if out_channels is None else out_channels
        try:
            rc = lib().nice_pipe_decode(self.ptr, src, ln, n, oc, dst, flags, status)
        finally:
            self._sums_done(sums, n)
        st = [int(status[i]) for i in range(n)]
        if rc != 0 and (raise_on_error or rc not in st):
            _check(rc, "nice_pipe_decode")
        return st
