"""Build libuampath.so for gfx950 in-tree with hipcc (no JIT cache: the .so travels with the
repo snapshot to the GPU box)."""
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "uampath.hip")
SRCS = [SRC, os.path.join(HERE, "csrc", "polyproc.cpp"), os.path.join(HERE, "csrc", "tiles.cpp")]
DEPS = SRCS + [os.path.join(HERE, "csrc", "polyproc.h"), os.path.join(HERE, "csrc", "ccl_tile.inc")]
HEADER = os.path.join(ROOT, "include", "uampath.h")
OUT = os.path.join(HERE, "lib", "libuampath.so")
ARCH = os.environ.get("UAM_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: every product/sum separately rounded, in the reference's order (bit-exact
# parity with the float64 oracle).  No fast-math.
HIPCC_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
               f"--offload-arch={ARCH}", "-Wall"]


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libuampath.so)")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in (*DEPS, HEADER, __file__))


def build_library(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    # UAM_HIPCC_EXTRA: extra flags for tuning experiments (e.g. "-DUAM_RF_WAVES=3")
    extra = os.environ.get("UAM_HIPCC_EXTRA", "").split()
    cmd = [hipcc(), *HIPCC_FLAGS, *extra, "-o", tmp, *SRCS, "-lz"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
