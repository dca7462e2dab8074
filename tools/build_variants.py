#!/usr/bin/env python3
"""Tuning builds of libuampath for tools/k2s_tbits.sh: build/var/libuampath_<name>.so with the
product's hipcc flags plus the -D flags of each variant, compiled in parallel on the CPU.
usage: python tools/build_variants.py name='-DUAM_SEG_CH1=8' [name2='...' ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from uam_path_planning_amd import build as b

    os.makedirs(os.path.join(ROOT, "build", "var"), exist_ok=True)
    procs = []
    for arg in sys.argv[1:]:
        name, flags = arg.split("=", 1)
        out = os.path.join(ROOT, "build", "var", f"libuampath_{name}.so")
        cmd = [b.hipcc(), *b.HIPCC_FLAGS, *flags.split(), "-o", out, *b.SRCS]
        procs.append((name, subprocess.Popen(cmd)))
    bad = [n for n, p in procs if p.wait() != 0]
    if bad:
        sys.exit(f"failed: {bad}")


if __name__ == "__main__":
    main()
