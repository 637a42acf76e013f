"""Build ``libfpm_hip.so`` (HIP kernels for gfx950 + host C++) in-tree with hipcc.

    python fingerprint-matching-code_amd/build.py [--jobs N] [--debug] [--asan]

Objects go to ``csrc/build/``; the shared library lands next to this file so it travels to the
GPU box with the repo snapshot.  Incremental: a source is recompiled when it (or a header) is
newer than its object.

``--asan``: a host-only build of the C-ABI's CPU code (``csrc/lsa.cpp``, ``csrc/sparse_host.cpp``)
with AddressSanitizer + UBSan, linked with the driver ``tests/asan/host_driver.cpp`` into
``csrc/build/asan_host_driver`` (run by ``tests/test_asan_host.py``); ``--tsan``: the same with
ThreadSanitizer (``tsan_host_driver``, the LSA thread pool).  GPU sanitizers are not
available on the pool; the device code is not part of this build.
"""
import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(CSRC, "build")
LIB = os.path.join(HERE, "libfpm_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("FPM_ARCH", "gfx950")

COMMON = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
          "-Wno-unused-lambda-capture", "-I" + CSRC, "-I" + os.path.join(os.path.dirname(HERE), "include")]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _needs(src, obj, headers_mtime):
    if not os.path.exists(obj):
        return True
    m = os.path.getmtime(obj)
    return os.path.getmtime(src) > m or headers_mtime > m


def _compile(src, debug):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    cmd = [HIPCC] + COMMON
    if src.endswith(".hip"):
        cmd += ["--offload-arch=" + ARCH, "-munsafe-fp-atomics", "-x", "hip"]
    else:
        cmd += ["-pthread", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-x", "c++"]
    if debug:
        cmd += ["-g"]
    cmd += ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr))
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    return obj


ASAN_SRCS = ("lsa.cpp", "sparse_host.cpp")
SANITIZERS = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
              "tsan": ["-fsanitize=thread"]}


def build_asan(verbose=True, kind="asan"):
    """Host-only sanitizer build of the CPU sources + the C driver (g++, no HIP).  ``kind``:
    "asan" (AddressSanitizer + UBSan) or "tsan" (ThreadSanitizer, for the LSA thread pool)."""
    os.makedirs(OBJ, exist_ok=True)
    ASAN_BIN = os.path.join(OBJ, "%s_host_driver" % kind)
    repo = os.path.dirname(HERE)
    driver = os.path.join(repo, "tests", "asan", "host_driver.cpp")
    srcs = [os.path.join(CSRC, f) for f in ASAN_SRCS] + [driver]
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(repo, "include", "*.h"))
    newest = max(os.path.getmtime(f) for f in srcs + hdrs)
    if os.path.exists(ASAN_BIN) and os.path.getmtime(ASAN_BIN) >= newest:
        return ASAN_BIN
    cmd = [os.environ.get("CXX", "g++"), "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer"] + SANITIZERS[kind] + [
           "-pthread",
           "-I" + CSRC, "-I" + os.path.join(repo, "include")] + srcs + ["-o", ASAN_BIN + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("asan build failed: %s\n%s" % (" ".join(cmd), r.stderr))
    os.replace(ASAN_BIN + ".tmp", ASAN_BIN)
    if verbose:
        print("built %s" % ASAN_BIN)
    return ASAN_BIN


def build(jobs=8, debug=False, force=False, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(os.path.dirname(HERE), "include", "*.h"))
    hm = max([os.path.getmtime(h) for h in hdrs] + [0])
    srcs = _sources()
    todo = [s for s in srcs if force or _needs(s, os.path.join(OBJ, os.path.basename(s) + ".o"), hm)]
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda s: _compile(s, debug), todo))
    objs = [os.path.join(OBJ, os.path.basename(s) + ".o") for s in srcs]
    if todo or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", LIB + ".tmp"] + objs + ["-pthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stderr))
        os.replace(LIB + ".tmp", LIB)
    if verbose:
        print("built %s (%d recompiled)" % (LIB, len(todo)))
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-only ASan/UBSan build of the CPU sources + driver")
    ap.add_argument("--tsan", action="store_true", help="host-only ThreadSanitizer build of the same")
    a = ap.parse_args()
    if a.asan or a.tsan:
        if a.asan:
            build_asan(kind="asan")
        if a.tsan:
            build_asan(kind="tsan")
    else:
        build(a.jobs, a.debug, a.force)
