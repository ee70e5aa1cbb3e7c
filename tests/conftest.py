"""Shared test setup: markers, repo paths, and loaders for the product package
(hyphenated directory, imported with importlib) and the oracle (checker only)."""
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKG_NAME = "fast-losless-image-compression-format_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def nice_pkg():
    return importlib.import_module(PKG_NAME)


def oracle_mod():
    from oracle import oracle as O
    return O


@pytest.fixture(scope="session")
def O():
    return oracle_mod()


@pytest.fixture(scope="session")
def nice():
    return nice_pkg()


def band_encode(nice, t, w, h, c, R):
    """One image through the band C ABI in one process (sharded.encode_bands)."""
    S = importlib.import_module(PKG_NAME + ".sharded")
    return S.encode_bands(t, w, h, c, R)


def set_hooks(nice, ctx, split_absent=0, pack_cap_bpp=0):
    """The library's per-context test hooks (nice_test_set_hooks)."""
    import ctypes
    L = nice.lib()
    L.nice_test_set_hooks.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    assert L.nice_test_set_hooks(ctx.ptr, split_absent, pack_cap_bpp) == 0


# include/nice_test.h ids (the library reads no environment variables)
OPT_IDS = {"NICE_DEC_SLICE_BITS": 0, "NICE_DEC_SINGLE_WAVE": 1, "NICE_DEC_SEG": 2, "NICE_DEC_SPLIT": 3,
           "NICE_DEC_FLOW": 4, "NICE_DEC_NO_EVENTS": 5, "NICE_DEC_EV_CAP": 6, "NICE_DEC_SLOW_PARSE": 7,
           "NICE_DEC_STATS": 8, "NICE_DEC_SYNC_QUEUED": 9, "NICE_DEC_REC_CLEAR": 10, "NICE_ENC_NO_RING": 11,
           "NICE_ENC_NO_PAIR": 12, "NICE_ENC_NO_SLIDE": 13,
           "NICE_TEST_FLOW_ABSENT": 14}


class Opts:
    """Test / A/B options of libnice_hip.so (nice_test_set_option), undone at teardown."""

    def __init__(self, nice):
        import ctypes
        self.L = nice.lib()
        self.L.nice_test_set_option.argtypes = [ctypes.c_int, ctypes.c_int64]

    def setenv(self, name, value):
        assert self.L.nice_test_set_option(OPT_IDS[name], int(value)) == 0

    def delenv(self, name):
        assert self.L.nice_test_set_option(OPT_IDS[name], -1) == 0

    def reset(self):
        self.L.nice_test_reset_options()


@pytest.fixture
def opts(nice):
    o = Opts(nice)
    o.reset()
    yield o
    o.reset()
