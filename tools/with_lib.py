#!/usr/bin/env python3
"""Run a script against a variant build of the HIP library (developer A/B
measurements only): `python tools/with_lib.py VARIANT.so bench.py ARGS...`.
Points diplomjourney_amd.native.LIB_PATH at the variant in this process, then
runs the script as __main__ — the product loader itself has no override."""
import ctypes
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diplomjourney_amd import native  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])


class _Tolerant(ctypes.CDLL):
    """An older variant may lack entry points added since: they resolve to a
    stub returning MPC_ERR_UNSUPPORTED (-4) instead of failing the binding."""

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            if name.startswith("__"):
                raise
            def stub(*_a):
                return -4
            setattr(self, name, stub)
            return stub


ctypes.CDLL = _Tolerant
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
