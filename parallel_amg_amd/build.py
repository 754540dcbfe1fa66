"""Build helpers: libpamg.so (hipcc for gfx950 + g++/OpenMP), in-tree."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libpamg.so")


def build(jobs: int = 4, arch: str = "gfx950") -> str:
    """Compile every HIP/C++ source of libpamg for ``arch``; returns the library path."""
    subprocess.run(["make", "-s", "-C", CSRC, f"-j{jobs}", f"ARCH={arch}"], check=True)
    if not os.path.exists(LIB):
        raise RuntimeError("libpamg.so was not produced")
    return LIB
