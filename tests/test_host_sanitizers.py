"""The library's host code under AddressSanitizer + UndefinedBehaviorSanitizer, on CPU
(VERDICT r01 item 9).  tests/csrc/host_fuzz.cpp is linked against the C ABI's host
translation units rebuilt with g++ -fsanitize=address,undefined (the kernels' object
from sy_amd.build supplies the launch symbols; no GPU call is made) and runs:

* the greedy walk (sydelta_walk.hpp) on 3000 random synthetic hit lists -- probed and
  unprobed sources, on-demand classification, phase-probed windows, entries inside the
  source, final/non-final chunks, the tail rule -- against a restated greedy walk
  (generator.rs:116-221 / 283-379), and its split form over 2, 3 and 8 segments;
* sydelta_delta_append (the chunk join) against a restated merge;
* the serde_json parsers on malformed, mutated, deeply nested and huge inputs, with
  writer -> parser -> writer round trips (ssh.rs:967-1003, sy-remote.rs:146-175);
* sydelta_delta_from_ops validation.

tests/csrc/kernel_bodies_fuzz.cpp (test_kernel_bodies_under_asan_ubsan) drives the
per-thread bodies of the device walk (sydelta_chain.hpp) and the zstd block coder
(sydelta_zstd.hpp) with every array allocated at its exact size, so an index a GPU
kernel would take out of its array is a report here, and checks them against walk_src
and the sequential stream writer.

Any sanitizer report (including leaks) fails the run.
"""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sy_amd", "csrc")
OUT = os.path.join(ROOT, "build", "asan")
HOST_SOURCES = ["sydelta_api.cpp", "sydelta_wire.cpp", "sydelta_local.cpp", "sydelta_integrity.cpp"]
FLAGS = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
         "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


KERNEL_SOURCES = ["sydelta_kernels.hip", "sydelta_filewalk.hip"]


def _kernels_objects() -> list:
    """The kernel translation units' objects from sy_amd.build (the launch symbols)."""
    from sy_amd import build as b

    objs = [os.path.join(b.OBJDIR, f.rsplit(".", 1)[0] + ".o") for f in KERNEL_SOURCES]
    if not os.path.exists(b.LIB) or any(not os.path.exists(o) or os.path.getmtime(o) < os.path.getmtime(
            os.path.join(CSRC, f)) for o, f in zip(objs, KERNEL_SOURCES)):
        b.build(force=True)
    return objs


@pytest.mark.timeout(900)
def test_host_code_under_asan_ubsan():
    if shutil.which("g++") is None or not os.path.exists("/opt/rocm/lib/libamdhip64.so"):
        pytest.skip("needs g++ and the ROCm runtime library")
    kobjs = _kernels_objects()
    os.makedirs(OUT, exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in HOST_SOURCES] + [os.path.join(ROOT, "tests", "csrc", "host_fuzz.cpp")]

    def compile_one(src):
        obj = os.path.join(OUT, os.path.basename(src).rsplit(".", 1)[0] + ".o")
        r = subprocess.run(["g++"] + FLAGS + ["-c", src, "-o", obj], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-4000:]
        return obj

    with ThreadPoolExecutor(min(5, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    exe = os.path.join(OUT, "host_fuzz")
    r = subprocess.run(["g++", "-fsanitize=address,undefined", "-o", exe] + objs +
                       kobjs + ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "3000"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "host_fuzz ok" in r.stdout
    assert "runtime error" not in r.stderr  # UBSan reports


@pytest.mark.timeout(600)
def test_host_pool_under_tsan():
    """The shared host pool and the split walk from 10 caller threads at once under
    ThreadSanitizer (tests/csrc/pool_tsan.cpp): no data race, results equal the serial
    walk."""
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "pool_tsan")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I" + os.path.join(ROOT, "include"),
                        "-I" + CSRC, os.path.join(ROOT, "tests", "csrc", "pool_tsan.cpp"), "-o", exe, "-lpthread"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1", SYDELTA_HOST_THREADS="6")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=500)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "pool_tsan ok" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr


@pytest.mark.timeout(900)
def test_kernel_bodies_under_asan_ubsan():
    """K5b's chain bodies on 2000 random classified sources (marking threads shuffled)
    against walk_src, and K7z's block coder plus a thread-by-thread replica of its
    parallel bit scatter on random texts, all under ASan + UBSan."""
    if shutil.which("g++") is None or not os.path.exists("/opt/rocm/include/hip/hip_runtime.h"):
        pytest.skip("needs g++ and the HIP headers")
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "kernel_bodies_fuzz")
    r = subprocess.run(["g++"] + FLAGS + [os.path.join(ROOT, "tests", "csrc", "kernel_bodies_fuzz.cpp"), "-o", exe,
                                          "-lpthread"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "2000"], capture_output=True, text=True, env=env, timeout=800)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "kernel bodies ok" in r.stdout
    assert "runtime error" not in r.stderr
