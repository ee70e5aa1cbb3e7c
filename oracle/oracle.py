"""ctypes front-end for the CPU restatement (oracle/nice_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg, as the checker.  The product package never
imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

STREAM_N = [256, 13, 64, 32, 11, 343, 64, 32, 32, 11]
DEC_REFERENCE = 0
DEC_STRIDE = 1          # "intent" decode: pixel stride = channels, correct bit reader
DEC_TOLERANT = 2        # DEC_STRIDE + tolerant table header (spilled max fields repaired)
E_PANIC, E_DOMAIN, E_HANG = -3, -4, -5


class OracleDecodeError(RuntimeError):
    def __init__(self, rc):
        self.rc = rc
        what = {E_PANIC: "reference would panic", E_DOMAIN: "tables outside the decodable domain",
                E_HANG: "reference decoder would never terminate"}.get(rc, "error")
        super().__init__(f"oracle decode failed rc={rc} ({what})")


class Stats(ctypes.Structure):
    _fields_ = [
        ("max_aob", ctypes.c_uint8 * 10),
        ("max_emitted_aob", ctypes.c_uint8),
        ("n_symbols", ctypes.c_uint64),
        ("n_coded", ctypes.c_uint64),
        ("n_backref", ctypes.c_uint64),
        ("n_smalldiff", ctypes.c_uint64),
        ("n_luma2", ctypes.c_uint64),
        ("n_luma", ctypes.c_uint64),
        ("n_rgb", ctypes.c_uint64),
        ("n_run_pixels", ctypes.c_uint64),
        ("header_end", ctypes.c_uint64),
        ("hist_total", ctypes.c_uint64),
        ("hist", ctypes.c_uint64 * 858),
        ("aob", ctypes.c_uint8 * 858),
        ("n_long_emits", ctypes.c_uint64),
        ("n_wrapped_emits", ctypes.c_uint64),
    ]


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB_PATH


def use_native() -> str:
    """Switch to the -march=native build (the timed CPU baseline), compiled on
    this machine; returns the build's flags, or raises if it cannot be built."""
    global _lib, _LIB_PATH
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle_native.so"], timeout=120)
    _LIB_PATH = os.path.join(_HERE, "liboracle_native.so")
    _lib = None
    lib()
    return "gcc -O3 -march=native"


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.nice_oracle_encode.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint8, ctypes.c_uint8,
                                         ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(Stats)]
        L.nice_oracle_decode.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(u8p),
                                         ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint8)]
        L.nice_oracle_free.argtypes = [ctypes.c_void_p]
        L.nice_oracle_code_lengths.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, u8p]
        L.nice_oracle_canonical.argtypes = [u8p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.nice_oracle_kat_writer.argtypes = [u8p, ctypes.c_int]
        L.nice_oracle_kat_reader.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_uint32)]
        L.nice_oracle_kat_hfe.argtypes = [ctypes.POINTER(ctypes.c_size_t), u8p]
        L.nice_oracle_gen_syn_v1.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_uint32]
        L.nice_oracle_gen_gradient.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_uint32]
        L.nice_oracle_calc_pos_from.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.nice_oracle_calc_pos_from.restype = ctypes.c_uint64
        L.nice_oracle_gen_deep_codes.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.nice_oracle_gen_deep_codes_at.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
        L.nice_oracle_encode_bitpos.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint8, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                                ctypes.POINTER(ctypes.c_uint64)]
        L.nice_oracle_gen_deep_codes_flat.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                      ctypes.c_uint32, ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                                      ctypes.c_uint32, ctypes.c_uint32]
        L.nice_oracle_gen_rgb_field.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]
        _lib = L
    return _lib


def _u8p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def encode(px: np.ndarray, width: int, height: int, channels: int, channels_out=None,
           with_stats: bool = False):
    """code::encode (code.rs:59-457) on a raster of ``channels`` bytes per pixel."""
    L = lib()
    px = np.ascontiguousarray(px, dtype=np.uint8).reshape(-1)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    st = Stats()
    rc = L.nice_oracle_encode(_u8p(px), px.size, width, height, channels,
                              channels if channels_out is None else channels_out,
                              ctypes.byref(out), ctypes.byref(n), ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed rc={rc}")
    try:
        data = bytes(ctypes.string_at(out, n.value))
    finally:
        L.nice_oracle_free(out)
    return (data, st) if with_stats else data


def encode_bitpos(px: np.ndarray, width: int, height: int, channels: int):
    """encode() plus, per pixel, the stream bit where its first symbol starts
    (2**64-1 for run members), then the data end bit: (stream, uint64 array
    of W*H + 1)."""
    L = lib()
    px = np.ascontiguousarray(px, dtype=np.uint8).reshape(-1)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    bits = np.zeros(width * height + 1, dtype=np.uint64)
    rc = L.nice_oracle_encode_bitpos(_u8p(px), px.size, width, height, channels, ctypes.byref(out),
                                     ctypes.byref(n), bits.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed rc={rc}")
    try:
        data = bytes(ctypes.string_at(out, n.value))
    finally:
        L.nice_oracle_free(out)
    return data, bits


def decode(stream: bytes, mode: int = DEC_REFERENCE):
    """code::decode (code.rs:464-687).  Returns (pixels, (w, h, ch)); raises on a
    condition where the reference would panic."""
    L = lib()
    buf = np.frombuffer(stream, dtype=np.uint8).copy()
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    w, h, ch = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint8()
    rc = L.nice_oracle_decode(_u8p(buf), buf.size, mode, ctypes.byref(out), ctypes.byref(n),
                              ctypes.byref(w), ctypes.byref(h), ctypes.byref(ch))
    if rc != 0:
        raise OracleDecodeError(rc)
    try:
        px = np.frombuffer(ctypes.string_at(out, n.value), dtype=np.uint8).copy()
    finally:
        L.nice_oracle_free(out)
    return px, (w.value, h.value, ch.value)


def code_lengths(counts) -> np.ndarray:
    counts = np.ascontiguousarray(counts, dtype=np.uint64)
    aob = np.zeros(counts.size, dtype=np.uint8)
    lib().nice_oracle_code_lengths(counts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                   counts.size, _u8p(aob))
    return aob


def canonical(aob) -> np.ndarray:
    aob = np.ascontiguousarray(aob, dtype=np.uint8)
    code = np.zeros(aob.size, dtype=np.uint64)
    lib().nice_oracle_canonical(_u8p(aob), aob.size,
                                code.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    return code


def gen_syn_v1(width: int, height: int, channels: int, seed: int) -> np.ndarray:
    """NICE-SYN-v1 photo-like synthetic frame."""
    px = np.zeros(width * height * channels, dtype=np.uint8)
    lib().nice_oracle_gen_syn_v1(_u8p(px), width, height, channels, seed)
    return px


def gen_gradient(width: int, height: int, channels: int) -> np.ndarray:
    px = np.zeros(width * height * channels, dtype=np.uint8)
    lib().nice_oracle_gen_gradient(_u8p(px), width, height, channels)
    return px


def gen_deep_codes(width: int, height: int, channels: int, seed: int = 1, k: int = 32) -> np.ndarray:
    """Small-diff frame with Fibonacci-skewed symbol counts: emitted codes of
    up to about k-1 bits (test input for the long-code writer path)."""
    px = np.zeros(width * height * channels, dtype=np.uint8)
    lib().nice_oracle_gen_deep_codes(_u8p(px), width, height, channels, seed, k)
    return px


def gen_deep_codes_at(width: int, height: int, channels: int, seed: int, k: int, force) -> np.ndarray:
    """gen_deep_codes whose pixels ``force`` (indices) take the rarest symbols
    (longest codes) first: a band starting at such a pixel begins with a long
    payload code."""
    px = np.zeros(width * height * channels, dtype=np.uint8)
    f = np.ascontiguousarray(sorted(force), dtype=np.uint64)
    lib().nice_oracle_gen_deep_codes_at(_u8p(px), width, height, channels, seed, k,
                                        f.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), f.size)
    return px


def gen_deep_codes_flat(width: int, height: int, channels: int, seed: int, k: int, force,
                        flat_rows) -> np.ndarray:
    """gen_deep_codes_at with rows [flat_rows[0], flat_rows[1]) one flat colour
    (a single run, generated without disturbing the symbol counts)."""
    px = np.zeros(width * height * channels, dtype=np.uint8)
    f = np.ascontiguousarray(sorted(force), dtype=np.uint64)
    lib().nice_oracle_gen_deep_codes_flat(_u8p(px), width, height, channels, seed, k,
                                          f.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), f.size,
                                          flat_rows[0], flat_rows[1])
    return px


def gen_rgb_field(width: int, height: int, channels: int, seed: int, noise_rows) -> np.ndarray:
    """RGB-mode frame (geometric residuals per channel) with uniform-noise rows
    ``noise_rows``: the noise pixels cost over 32 bits each."""
    px = np.zeros(width * height * channels, dtype=np.uint8)
    r = np.ascontiguousarray(sorted(noise_rows), dtype=np.uint32)
    lib().nice_oracle_gen_rgb_field(_u8p(px), width, height, channels, seed,
                                    r.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), r.size)
    return px


def calc_pos_from(width: int, height: int, index: int) -> int:
    """image.rs:45-102 Image::calc_pos_from (2^64-1 where the reference panics)."""
    return int(lib().nice_oracle_calc_pos_from(width, height, index))


def kat_writer() -> bytes:
    buf = np.zeros(16, dtype=np.uint8)
    n = lib().nice_oracle_kat_writer(_u8p(buf), 16)
    return bytes(buf[:n])


def kat_reader(data: bytes, ops, bits):
    arr = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    n = len(ops)
    o = (ctypes.c_int * n)(*ops)
    b = (ctypes.c_int * n)(*bits)
    res = (ctypes.c_uint32 * n)()
    rc = lib().nice_oracle_kat_reader(_u8p(arr), arr.size, o, b, n, res)
    if rc != 0:
        raise RuntimeError("reader KAT hit EOF")
    return list(res)


def kat_hfe():
    n = ctypes.c_size_t()
    mx = ctypes.c_uint8()
    rc = lib().nice_oracle_kat_hfe(ctypes.byref(n), ctypes.byref(mx))
    return rc, n.value, mx.value
