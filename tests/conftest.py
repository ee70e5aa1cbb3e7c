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
