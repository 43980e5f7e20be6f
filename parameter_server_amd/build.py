"""In-tree build of the HIP library (gfx950) and the C++ host programs.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the resulting .so files travel to the GPU box with the repo.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

LIB_SOURCES = ["pskv_kernels.hip", "pskv_shard.cpp", "pskv_frames.cpp"]
LIB_OUT = os.path.join(PKG, "libpskv.so")
CPP_TESTS = {  # program -> (source in tests/cpp, links the oracle checker)
    "hip_storage_test": ("hip_storage_test.cpp", False),
    "ssp_replay": ("ssp_replay.cpp", True),
    "kv_client_table_test": ("kv_client_table_test.cpp", False),
}
ORACLE_DIR = os.path.join(ROOT, "oracle")
BIN_DIR = os.path.join(PKG, "bin")


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed: " + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force=False):
    srcs = [os.path.join(CSRC, s) for s in LIB_SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in ("pskv_internal.h", "pskv_frames.h", "pskv_queues.h")] + [os.path.join(INCLUDE, "pskv.h")]
    if force or _stale(LIB_OUT, deps):
        # built beside, then renamed over: a reader (a test, a GPU-box upload)
        # never sees a half-written library
        tmp = LIB_OUT + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-I", INCLUDE, "-I", CSRC, *srcs, "-o", tmp])
        os.replace(tmp, LIB_OUT)
    return LIB_OUT


def build_cpp_tests(force=False):
    os.makedirs(BIN_DIR, exist_ok=True)
    outs = []
    hdrs = [os.path.join(INCLUDE, "ps", h) for h in os.listdir(os.path.join(INCLUDE, "ps"))]
    for prog, (src, with_oracle) in CPP_TESTS.items():
        s = os.path.join(ROOT, "tests", "cpp", src)
        out = os.path.join(BIN_DIR, prog)
        deps = [s, LIB_OUT] + hdrs
        extra = []
        if with_oracle:  # test programs only: the checker is linked beside the product
            deps.append(os.path.join(ORACLE_DIR, "liboracle.so"))
            extra = ["-L", ORACLE_DIR, "-loracle", "-Wl,-rpath,$ORIGIN/../../oracle"]
        if force or _stale(out, deps):
            # host-only C++ against the C ABI: the program never sees HIP types
            _run(["g++", "-O2", "-std=c++11", "-pthread", "-I", INCLUDE, s, "-o", out,
                  "-L", PKG, "-lpskv", "-Wl,-rpath,$ORIGIN/..", *extra])
        outs.append(out)
    return outs


def build_oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle  # noqa: WPS433  (test infrastructure: the checker, built beside the product)

        return oracle.build()
    finally:
        sys.path.pop(0)


RA_SRC = os.path.join(ROOT, "tools", "micro", "random_access.hip")
RA_OUT = os.path.join(ROOT, "tools", "micro", "librandom_access.so")


def build_random_access(force=False):
    """bench.py's random-access calibration (not part of libpskv)."""
    if force or _stale(RA_OUT, [RA_SRC]):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", RA_SRC, "-o", RA_OUT])
    return RA_OUT


def build_all(force=False):
    lib = build_lib(force)
    orc = build_oracle()
    progs = build_cpp_tests(force)
    ra = build_random_access(force)
    return {"lib": lib, "cpp": progs, "oracle": orc, "random_access": ra}


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv))
