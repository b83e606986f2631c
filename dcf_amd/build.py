"""Build the in-tree HIP library ``dcf_amd/libdcf_hip.so`` for gfx950.

Plain ``hipcc -shared``: the C ABI (include/dcf_hip.h) has no torch types, so
no torch extension machinery is involved.  The .so is git-ignored but travels
to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dcf_amd")
SRC = os.path.join(PKG, "csrc", "dcf_hip.hip")
HDR = os.path.join(ROOT, "include", "dcf_hip.h")
LIB = os.path.join(PKG, "libdcf_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DCF_OFFLOAD_ARCH", "gfx950")


def _sources():
    csrc = os.path.join(PKG, "csrc")
    return [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".hpp"))] + [HDR]


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in _sources())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", LIB + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
