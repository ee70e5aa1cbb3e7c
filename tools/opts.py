"""Diagnostic tools only: forwards NICE_DEC_* / NICE_ENC_* variables of the
tool's environment to the library's test options (include/nice_test.h,
nice_test_set_option) -- the library itself reads no environment."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import OPT_IDS  # noqa: E402


def apply_env(nice):
    L = nice.lib()
    L.nice_test_set_option.argtypes = [ctypes.c_int, ctypes.c_int64]
    for name, oid in OPT_IDS.items():
        v = os.environ.get(name)
        if v is not None:
            assert L.nice_test_set_option(oid, int(v) if v.strip() else 1) == 0, name
