#!/usr/bin/env python3
"""K3b diagnostics (GPU box): builds libuampath with -DUAM_K3B_DIAG into build/k3b_diag/, loads
it (UAM_LIB_PATH) and reports, for the cfg3 analytic workload, the kernel time with and without
the evaluation phase and the sorted chunks' coherence: distinct grid slots per 64-point chunk,
union-walk steps vs. each lane's own list entries (table 0 = region penalty, obstacle walk).
usage: python tools/probe_k3b.py [--seg 8] [--pairs 100000]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seg", type=int, default=8)
    ap.add_argument("--cpl", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from uam_path_planning_amd import build as B
    out = os.environ.get("K3B_DIAG_LIB") or os.path.join(ROOT, "build", "k3b_diag", "libuampath.so")
    if not os.path.exists(out) or os.environ.get("UAM_REBUILD"):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run([B.hipcc(), *B.HIPCC_FLAGS, "-DUAM_K3B_DIAG", "-o", out, *B.SRCS],
                       check=True)
    os.environ["UAM_LIB_PATH"] = out
    import torch
    from uam_path_planning_amd import _lib
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements)
    from uam_path_planning_amd.synthetic import random_pairs

    lib = _lib.load()
    lib.uam_k3b_diag.restype = ctypes.c_int
    lib.uam_k3b_diag.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    spec = canonical_spec(nfz_polygons=CONFIGS["cfg3"]["nfz_polygons"])
    params = canonical_params(spec, N=80, altitude=320.0)
    e = Engine(0)
    e.set_option("k3b_segment", a.seg)
    e.set_option("k3b_points_per_lane", a.cpl)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(params)
    ut = e.tensor(arc_table(80, displacements(5)), torch.float64)
    pairs = e.tensor(random_pairs(a.pairs, seed=0), torch.float64)
    outs = e.outputs(a.pairs * 5, 82, n_pairs=a.pairs)
    buf = (ctypes.c_uint64 * 24)()
    for skip, name in ((0, "counters"), (2, "full"), (3, "no-eval"), (6, "no-table0"), (10, "no-obstacles"), (14, "no-walks")):
        lib.uam_k3b_diag(buf, skip)
        e.eval_generated(pairs, ut, outputs=outs)   # warm-up (and the counters of one launch)
        torch.cuda.synchronize()
        lib.uam_k3b_diag(buf, skip)
        c = list(buf)
        e.kernel_timing(True)
        for _ in range(a.reps):
            e.eval_generated(pairs, ut, outputs=outs)
        ms, n = e.kernel_time()
        e.kernel_timing(False)
        lib.uam_k3b_diag(buf, 0)
        line = f"seg {a.seg} cpl {a.cpl} {name}: {ms / n:.3f} ms"
        if skip == 0 and c[0]:
            line += (f"; chunks {c[0]}, distinct slots/chunk {c[1] / c[0]:.2f}, "
                     f"table-0 union steps/chunk {c[2] / c[0]:.2f} vs lane entries/point "
                     f"{c[3] / (64 * c[0]):.2f}, obstacle union steps/chunk {c[4] / c[0]:.2f} vs "
                     f"lane entries/point {c[5] / (64 * c[0]):.2f}, points re-walked "
                     f"{c[6]} (more than K3B_KT terms: {c[7]}), points with terms {c[14]}, terms {c[15]}")
        tot = sum(c[8:14]) or 1
        line += "; workgroup phase shares (thread 0 cycles): " + ", ".join(
            f"{n} {v / tot:.1%}" for n, v in zip(("pass1", "keys", "scan+scatter", "eval",
                                                  "ordered sums", "output"), c[8:14]))
        if skip == 2 and c[21]:
            n = c[21]
            line += (f"; per chunk (wave cycles): load+point {c[18] / n:.0f}, walk "
                     f"{c[19] / n:.0f} (table 0 {c[16] / n:.0f}, obstacles {c[17] / n:.0f}), "
                     f"park {c[20] / n:.0f}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
