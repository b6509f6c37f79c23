"""The library's host logic end to end on the CPU (no GPU): the C ABI's host translation
units (sydelta_api/wire/local/integrity.cpp) linked against a host emulation of the
device layer (tests/csrc/fake_device.cpp: HIP runtime calls on host memory, the
launch_* contracts computed with the C oracle's hashes) into build/emu/
libsydelta_emu.so, driven through sy_amd.delta's bindings by tests/csrc/
emulated_checks.py and compared with the C oracle.

This checks the code around the kernels — classification bookkeeping (probe, ranges,
on-demand scans), the sequential and split walks, the chunked and streamed path API,
the in-memory generator, the path-level change ratio, 10 concurrent callers — before it
reaches a GPU.  It says nothing about the kernels (tests/test_gpu_*.py do), and the
emulation library is test infrastructure: the product module never loads it.
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sy_amd", "csrc")
OUT = os.path.join(ROOT, "build", "emu")
HOST_TUS = ["sydelta_api.cpp", "sydelta_wire.cpp", "sydelta_local.cpp", "sydelta_integrity.cpp"]


def _build() -> str:
    os.makedirs(OUT, exist_ok=True)
    flags = ["-std=c++17", "-O1", "-g", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
             "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    jobs = [(["g++"] + flags + ["-c", os.path.join(CSRC, f), "-o", os.path.join(OUT, f[:-4] + ".o")])
            for f in HOST_TUS]
    jobs.append(["g++"] + flags + ["-c", os.path.join(ROOT, "tests", "csrc", "fake_device.cpp"), "-o",
                                   os.path.join(OUT, "fake_device.o")])
    jobs.append(["gcc", "-O2", "-fPIC", "-c", os.path.join(ROOT, "oracle", "sydelta_oracle.c"), "-o",
                 os.path.join(OUT, "oracle.o")])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-4000:]

    with ThreadPoolExecutor(min(6, os.cpu_count() or 1)) as ex:
        list(ex.map(run, jobs))
    lib = os.path.join(OUT, "libsydelta_emu.so")
    objs = [os.path.join(OUT, f[:-4] + ".o") for f in HOST_TUS] + [os.path.join(OUT, "fake_device.o"),
                                                                   os.path.join(OUT, "oracle.o")]
    run(["g++", "-shared", "-o", lib] + objs + ["-Wl,-Bsymbolic", "-Wl,--no-undefined", "-lpthread", "-lm"])
    return lib


@pytest.mark.timeout(1200)
def test_host_logic_on_emulated_device():
    if shutil.which("g++") is None or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("needs g++ and the HIP headers")
    lib = _build()
    # SYDELTA_CHUNK_SEG_LAST: the pipelined chunk checks' last part in 16-block segments
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "csrc", "emulated_checks.py"), ROOT, lib],
                       capture_output=True, text=True, timeout=1100, cwd="/tmp",
                       env=dict(os.environ, SYDELTA_CHUNK_SEG_LAST="16"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "emulated host checks ok" in r.stdout


@pytest.mark.timeout(600)
def test_multi_device_host_logic_on_emulated_devices():
    """Four emulated devices (EMU_DEVICES=4): the path API's per-thread device binding and
    the in-process multi-device chunked match (peer-copied signature, chained walks)."""
    if shutil.which("g++") is None or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("needs g++ and the HIP headers")
    lib = _build()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "csrc", "emulated_checks.py"), ROOT, lib, "multi"],
                       capture_output=True, text=True, timeout=550, cwd="/tmp", env=dict(os.environ, EMU_DEVICES="4"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "emulated multi-device checks ok" in r.stdout
