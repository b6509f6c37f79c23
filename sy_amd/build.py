"""Build libsydelta.so (gfx950 HIP kernels + C ABI) in-tree.

    python -m sy_amd.build            # incremental
    python -m sy_amd.build --force
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libsydelta.so")
SOURCES = ["sydelta_kernels.hip", "sydelta_filewalk.hip", "sydelta_api.cpp", "sydelta_wire.cpp", "sydelta_local.cpp", "sydelta_integrity.cpp"]
HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith(".hpp")) + [os.path.join("..", "..", "include", "sydelta.h")]
# objects stay in build/obj (the host sanitizer test links sydelta_kernels.o)
OBJDIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("SYDELTA_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    jobs = []
    os.makedirs(OBJDIR, exist_ok=True)
    # an object is rebuilt when its source, or any header, is newer (or on --force)
    t_hdr = max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS)
    for src in SOURCES:
        obj = os.path.join(OBJDIR, src.rsplit(".", 1)[0] + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(t_hdr, os.path.getmtime(
                os.path.join(CSRC, src))):
            continue
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
               "-I", os.path.join(ROOT, "include"), "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
        jobs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    for j in jobs:
        out, _ = j.communicate()
        if j.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{out}")
        if verbose and out:
            print(out)
    tmp = LIB + ".tmp"
    link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(link, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
