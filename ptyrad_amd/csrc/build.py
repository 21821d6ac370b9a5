"""Build libptyx.so for gfx950 with hipcc (in-tree, so the .so travels with the repo snapshot).

    python -m ptyrad_amd.csrc.build [--force] [--only-n 128]
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
OUT = os.path.join(PKG, "lib", "libptyx.so")
SOURCES = [os.path.join(HERE, "ptyx_kernels.hip")]
DEPS = SOURCES + glob.glob(os.path.join(HERE, "*.hpp")) + [os.path.join(ROOT, "include", "ptyx.h")]
ARCH = os.environ.get("PTYX_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build libptyx.so)")


def up_to_date(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, only_n: int | None = None, out: str = OUT, extra=None, verbose=True) -> str:
    if not force and only_n is None and up_to_date(out):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp", *SOURCES]
    if only_n:
        cmd.insert(2, f"-DPTYX_ONLY_N={only_n}")
    if extra:
        cmd[2:2] = list(extra)
    if verbose:
        print("[ptyx build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only-n", type=int, default=None)
    a = ap.parse_args()
    print(build(a.force, a.only_n))
    sys.exit(0)
