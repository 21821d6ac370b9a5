"""Build libptyx.so for gfx950 with hipcc (in-tree, so the .so travels with the repo snapshot).

    python -m ptyrad_amd.csrc.build [--force] [--only-n 128]

Each translation unit compiles to its own object under build/obj/ (in parallel, and only when
it or a header is newer than its object), then one hipcc -shared link.

Freshness is keyed on CONTENT, not mtimes: the sha1 of every source and header (plus the flags)
is compiled into the library (ptyx_build_id(), a generated one-line translation unit), so
``up_to_date`` rebuilds whenever the library was built from other sources, and ``_lib.load()``
refuses a library whose build id does not match the sources next to it.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
OUT = os.path.join(PKG, "lib", "libptyx.so")
OBJ = os.path.join(ROOT, "build", "obj")
SOURCES = [os.path.join(HERE, "ptyx_kernels.hip"), os.path.join(HERE, "ptyx_constraints.hip"),
           os.path.join(HERE, "ptyx_ingest.hip"), os.path.join(HERE, "ptyx_optim.hip")]
GEN_SOURCE = os.path.join(HERE, "ptyx_gen.hip")


MAX_RADIX = 49


def plan_r1(n: int) -> int:
    """ptyx_fft.hpp plan_r1: the first-pass radix of the two-pass plan (0: none)."""
    fixed = {16: 16, 32: 8, 64: 8, 128: 16, 256: 16}
    if n in fixed:
        return fixed[n]
    if n > 256:
        r = next(r for r in range(2, n + 1) if n % r == 0 and r * r >= n)
        return r if r <= MAX_RADIX else 0
    for r in list(range(16, 1, -1)) + list(range(17, MAX_RADIX + 1)):
        if n % r == 0 and n // r <= 16:
            return r
    return 0


def smooth_sizes(lo: int = 32, hi: int = 512):
    """Every 2·3·5·7-smooth N in [lo, hi] with a two-pass plan: the general engine's supported
    sizes (all of them: the largest radix needed is 49, for 343 = 49·7)."""
    out = []
    for n in range(lo, hi + 1):
        m = n
        for f in (2, 3, 5, 7):
            while m % f == 0:
                m //= f
        if m == 1 and plan_r1(n):
            out.append(n)
    return out


GEN_SIZES = smooth_sizes()
# size groups of the general engine, one ptyx_gen.hip object each (compiled in parallel): dealt
# round-robin over the sizes in descending order so every group gets a similar mix
N_GEN_GROUPS = 16
GEN_GROUPS = [sorted(GEN_SIZES[::-1][g::N_GEN_GROUPS]) for g in range(N_GEN_GROUPS)]
HEADERS = glob.glob(os.path.join(HERE, "*.hpp")) + [os.path.join(ROOT, "include", "ptyx.h")]
DEPS = SOURCES + [GEN_SOURCE] + HEADERS
ARCH = os.environ.get("PTYX_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fno-slp-vectorize", "-fPIC"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build libptyx.so)")


def source_hash(defs=()) -> str:
    """sha1 over the contents of every source / header and the compile flags."""
    h = hashlib.sha1()
    for d in sorted(DEPS, key=os.path.basename):
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    h.update(" ".join([ARCH, *FLAGS, *defs]).encode())
    return h.hexdigest()


def library_build_id(path: str = OUT) -> str | None:
    """The build id compiled into a built library (without loading HIP): the marker string."""
    if not os.path.exists(path):
        return None
    data = open(path, "rb").read()
    i = data.find(b"PTYX_BUILD_ID=")
    return data[i + 14:i + 54].decode() if i >= 0 else None


def up_to_date(out: str = OUT) -> bool:
    return library_build_id(out) == source_hash()


def _headers_of(src: str):
    """Headers a translation unit depends on (the constraints unit includes only its own)."""
    if os.path.basename(src) == "ptyx_constraints.hip":
        return [os.path.join(HERE, "ptyx_constraints.hpp"), os.path.join(HERE, "ptyx_abi.hpp"),
                os.path.join(ROOT, "include", "ptyx.h")]
    gen = [os.path.join(HERE, h) for h in ("ptyx_general.hpp", "ptyx_single.hpp")]
    if os.path.basename(src) == "ptyx_gen.hip":
        return gen + [os.path.join(HERE, h) for h in ("ptyx_common.hpp", "ptyx_fft.hpp", "ptyx_genops.hpp")] + \
            [os.path.join(ROOT, "include", "ptyx.h")]
    if os.path.basename(src) == "ptyx_kernels.hip":
        return [h for h in HEADERS if h not in gen]
    if os.path.basename(src) == "ptyx_ingest.hip":
        return [os.path.join(HERE, "ptyx_abi.hpp"), os.path.join(ROOT, "include", "ptyx.h")]
    return HEADERS


def _stale(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + _headers_of(src))


def build(force: bool = False, only_n: int | None = None, out: str = OUT, extra=None, verbose=True) -> str:
    if not force and only_n is None and not extra and up_to_date(out):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    defs = ([f"-DPTYX_ONLY_N={only_n}"] if only_n else []) + list(extra or [])
    tag = "default" if not defs else "v" + hashlib.sha1(" ".join(defs).encode()).hexdigest()[:10]
    odir = os.path.join(OBJ, tag)
    os.makedirs(odir, exist_ok=True)
    cc = hipcc()

    groups = [[only_n]] if only_n else GEN_GROUPS
    units = [(src, os.path.basename(src), []) for src in SOURCES]
    units += [(GEN_SOURCE, f"ptyx_gen_{'_'.join(map(str, g))}.hip",
               [f"-DPTYX_GEN_SIZES={','.join(map(str, g))}"]) for g in groups]

    def compile_one(unit):
        src, name, udefs = unit
        obj = os.path.join(odir, name + ".o")
        if force or _stale(obj, src):
            cmd = [cc, f"--offload-arch={ARCH}", *FLAGS, *defs, *udefs, "-I", os.path.join(ROOT, "include"), "-c",
                   src, "-o", obj + ".tmp"]
            if verbose:
                print("[ptyx build]", " ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(obj + ".tmp", obj)
        return obj

    jobs = int(os.environ.get("PTYX_BUILD_JOBS", "0")) or min(len(units), os.cpu_count() or 4, 16)
    # the two slowest units first, so they do not start last
    order = sorted(range(len(units)), key=lambda i: 0 if units[i][1] == "ptyx_kernels.hip" else 1)
    with ThreadPoolExecutor(jobs) as ex:
        done = dict(zip(order, ex.map(compile_one, [units[i] for i in order])))
    objs = [done[i] for i in range(len(units))]
    # build id: the content hash of the sources this library is made of
    bid = source_hash(defs)
    bsrc = os.path.join(odir, "ptyx_build_id.cpp")
    with open(bsrc, "w") as f:
        f.write('static const char kId[] = "PTYX_BUILD_ID=%s";\n'
                'extern "C" const char* ptyx_build_id(void) { return kId + 14; }\n' % bid)
    bobj = bsrc + ".o"
    subprocess.run([cc, "-fPIC", "-O2", "-c", bsrc, "-o", bobj], check=True)
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, bobj, "-o", out + ".tmp"]
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
