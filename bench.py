#!/usr/bin/env python3
"""Headline benchmark: candidate-paths/s (+ waypoint-evals/s) of the batched candidate-path
cost evaluation on an R x R DEM cost raster (BASELINE.json metric), MI355X.

One "step" = one pass of the hot path over the batch resident in HBM: the fused kernel
(arc generator K4 + raster gather / cost reduction K2) over every pair x displacement, then
the reference's candidate selection (argmin on fval and on length, K5).  Default workload:
BASELINE config 3 (4096^2 DEM + 69 no-fly shapes, 100k start/goal pairs x 5 displacements =
500k paths x 82 waypoints per GPU; weak scaling: every rank gets its own 100k pairs).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process
per GPU, RCCL; rank 0 builds the cost raster (K1) and broadcasts it once over xGMI (timed
separately, outside the step); pairs are sharded with no collective in the hot loop.

Prints ONE JSON line (rank 0).  Also reports the dominant kernel's roofline (algorithmic bytes
/ HIP-event kernel time vs 8 TB/s HBM) and a CPU baseline: the C oracle (oracle/, a "port")
timed on this host on a bounded sample of the same workload -- one thread first (which
doubles as a bit-exact parity check of the GPU outputs on that sample), then the sample over
the host's CPU share in contiguous pair shards; `cores` is that thread count.
"""
import argparse
import concurrent.futures
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "candidate-paths/sec + waypoint-evals/sec on N×N DEM at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# independent random 16-B gathers from a 256 MiB table, one MI355X (profiles/r01/gather_ceiling.log)
RANDOM_GATHER_CEILING = 55.5e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--mode", default=None, choices=["raster", "analytic", "volume"],
                    help="default: the workload's mode (raster; volume for cfg5)")
    ap.add_argument("--pairs", type=int, default=None, help="override pairs per GPU")
    ap.add_argument("--R", type=int, default=None, help="override raster size")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads for the CPU baseline (0: the box's CPU share, "
                         "OMP_NUM_THREADS capped by the affinity mask and 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variant", type=int, default=0, help="uam_set_tuning kernel variant")
    ap.add_argument("--no-skip", action="store_true",
                    help="K2 without the gather-skip summary (A/B; results are identical)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one GPU per rank; UAM_BENCH_RANKS_PER_GPU > 1 packs ranks onto fewer GPUs (rehearsal of
    # the N-rank path on a 1-GPU box, with UAM_DIST_BACKEND=gloo since RCCL needs a GPU per
    # rank)
    per_gpu = max(1, int(os.environ.get("UAM_BENCH_RANKS_PER_GPU", "1")))
    backend = None
    local = local // per_gpu
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("UAM_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)

    from uam_path_planning_amd import build
    from uam_path_planning_amd import distributed as udist
    build.build_library()
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import CostRaster, Engine, RiskVolume, VolumeGeo
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, layer_weights,
                                                raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, random_pairs3d, synthetic_dem

    cfg = dict(CONFIGS[args.workload])
    if args.pairs:
        cfg["pairs"] = args.pairs
    if args.R:
        cfg["R"] = args.R
    R, Q, D, N = cfg["R"], cfg["pairs"], cfg["D"], cfg["N"]
    W = N + 2
    mode = args.mode or cfg["mode"]
    args.mode = mode
    raster_mode = mode == "raster"
    volume_mode = mode == "volume"

    spec = canonical_spec(nfz_polygons=cfg["nfz_polygons"])
    geom = compile_map(build_region_map(spec))
    params = canonical_params(spec, N=N, altitude=320.0)
    eng = Engine(local)
    eng.set_geometry(geom)
    eng.set_params(params)
    ut_host = arc_table(N, displacements(D))

    # ---- cost raster / volume: rank 0 builds (K1), one RCCL broadcast --------------------
    setup = {}
    if world > 1:
        setup["dist_backend"] = backend
        setup["ranks_per_gpu"] = per_gpu
    geo = raster_geo(R)
    raster = volume = None
    if raster_mode or volume_mode:
        t0 = time.perf_counter()
        if rank == 0:
            dem = synthetic_dem(R)
            setup["dem_gen_s"] = round(time.perf_counter() - t0, 3)
            dem_dev = eng.tensor(dem, torch.float32)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            raster = eng.raster_build(geo, dem_dev)
            torch.cuda.synchronize()
            setup["raster_build_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
            if volume_mode:
                t2 = time.perf_counter()
                volume = eng.volume_build(raster, cfg["nz"], cfg["z0"], cfg["dz"],
                                          layer_weights(cfg["nz"]))
                torch.cuda.synchronize()
                setup["volume_build_ms"] = round((time.perf_counter() - t2) * 1e3, 3)
            del dem_dev
        else:
            raster = CostRaster(geo, eng.empty((R, R, 4), torch.int32))
            if volume_mode:
                vg = VolumeGeo(R, R, cfg["nz"], geo.x0, geo.y_top, geo.dx, geo.dy, cfg["z0"],
                               cfg["dz"])
                volume = RiskVolume(vg, eng.empty((R, R, cfg["nz"], 4), torch.int32))
        if world > 1:
            dist.barrier()
            table = volume.vox if volume_mode else raster.rec
            secs = udist.broadcast_raster(table, src=0)
            setup["raster_bcast_ms"] = round(secs * 1e3, 3)
            setup["raster_bytes"] = table.numel() * 4
            if raster_mode and rank > 0:
                eng.raster_summary(raster)   # each rank derives the skip table locally
        if raster_mode and args.no_skip:
            raster.summary = None

    # ---- this rank's shard of pairs (weak scaling) -----------------------------------------
    if volume_mode:
        pairs_host = udist.weak_shard(random_pairs3d(Q * world, seed=0), Q, rank, world)
    else:
        pairs_host = udist.weak_shard(random_pairs(Q * world, seed=0), Q, rank, world)
    pairs = eng.tensor(pairs_host, torch.float64)
    ut = eng.tensor(ut_host, torch.float64)
    P = Q * D
    outs = eng.outputs(P, W, n_pairs=Q)
    o = outs[0]
    if args.variant:
        eng.set_tuning(args.variant)

    def step(ev=None):
        # one launch: arc generation + gather + cost reduction + candidate selection
        if ev is not None:
            ev[0].record()
        if volume_mode:
            eng.eval_generated3d(pairs, ut, volume, outputs=outs)
        else:
            eng.eval_generated(pairs, ut, raster=raster, outputs=outs)
        if ev is not None:
            ev[1].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    if world > 1:
        elapsed, kern_ms = udist.max_over_ranks([elapsed, kern_ms], device=eng.torch_device)

    total_paths = P * world * args.steps
    value = total_paths / elapsed
    # algorithmic bytes per launch of the dominant kernel
    gather_b = 16 * W if (raster_mode or volume_mode) else 0
    pair_b = (48.0 if volume_mode else 32.0) / D
    # 6 f64 + 3 i32 per path (nfz_hits, offmap, below_terrain), 2 i32 best indices per pair
    out_b = 6 * 8 + 3 * 4 + 8.0 / D
    bytes_per_path = gather_b + pair_b + out_b
    launch_bytes = bytes_per_path * P
    achieved = launch_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            key = f"{args.workload}:{args.mode}:R{R}:Q{Q}"
            traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    # which kernel the library picks (uampath.hip want_wave: tuning 9, or auto for batches of
    # at most 16384 paths in raster / volume mode; 10 = never)
    wave = args.mode != "analytic" and (args.variant == 9 or (args.variant == 0 and P <= 16384))
    kernel_name = (f"k_eval_wave<{mode}> (one wave per path)" if wave else
                   "k_bin_count/k_bin_scatter/k_bin_gather + k_eval_pairs<records> (variant 11,"
                   " binned)" if (args.variant == 11 and raster_mode) else
                   f"k_eval_pairs<{mode}>" + (f" (variant {args.variant or 2})"
                                              if raster_mode else ""))
    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "candidate-paths/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (DEM seed 1 with the Nagasaki DEM's statistics, pairs seed 0, "
                "NFZ polygons seed 2; canonical map geometry from the reference data files)",
        "config": {"workload": f"{args.workload}: {workload_name(cfg['name'], world)}",
                   "dem": f"{R}x{R}", "pairs_per_gpu": Q, "displacements": D,
                   "waypoints_per_path": W, "paths_per_gpu": P, "mode": args.mode,
                   "no_fly_shapes": geom.n_obstacles, "region_shapes":
                   int(geom.region_first[-1] - geom.region_first[0]),
                   "parallelism": f"pair-sharded dp{world}, raster broadcast once"},
        "waypoint_evals_per_s": round(value * W, 1),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel": kernel_name,
                     "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_path": bytes_per_path,
                     "algorithmic_bytes_per_launch": launch_bytes,
                     "traffic_frac": (round(traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                      if traffic else None),
                     "gathers_per_s": round(P * W / (kern_ms * 1e-3), 1) if gather_b else None,
                     "random_gather_ceiling_per_s": RANDOM_GATHER_CEILING if gather_b else None,
                     "note": ("each 16-B record gather moves one 128-B line (PMC); the measured "
                              "random-gather ceiling (tools/gather_ceiling.hip) bounds the "
                              "kernel, see DESIGN.md §5") if gather_b else
                             ("analytic mode reads only the pairs and writes the results, so "
                              "the HBM fraction is not its bound: the f64 shape walk and lane "
                              "divergence are (vector f64, not MFMA), see DESIGN.md §4 K3")},
        "setup": setup,
    }

    # ---- CPU baseline + parity sample (rank 0, N=1 only) ----------------------------------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        O.build()
        orc = O.Oracle(O.compile_spec(spec), N, spec["options"], spec["maxratio"],
                       spec["maxalpha"], spec["enlargement"], spec["weights"],
                       altitude=params.altitude)
        rd = rec = vd = vox = None
        if raster_mode:
            rd = O.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                      geo.nodata, geo.dem_threshold)
            rec = raster.rec.cpu().numpy().view(np.float32)
        if volume_mode:
            g3 = volume.geo
            vd = O.volume_desc(g3.nx, g3.ny, g3.nz, g3.x0, g3.y_top, g3.dx, g3.dy, g3.z0, g3.dz)
            vox = volume.vox.cpu().numpy().view(np.float32)
        gpu_cost = o["cost"].cpu().numpy()
        gpu_best = o["best_fval_idx"].cpu().numpy()
        chunk = 50 if mode == "analytic" else 2000
        done, t_cpu, mism, bmis = 0, 0.0, 0, 0
        while done < Q and t_cpu < args.cpu_seconds:
            sl = pairs_host[done:done + chunk]
            ts = time.perf_counter()
            if volume_mode:
                r = orc.eval_paths3d(O.gen_paths3d(sl, ut_host), vd, vox)
            else:
                r = orc.eval_paths(O.gen_paths(sl, ut_host), mode=mode, rdesc=rd, rec=rec)
            t_cpu += time.perf_counter() - ts
            mism += int(np.sum(r["cost"] != gpu_cost[done * D:(done + len(sl)) * D]))
            bmis += int(np.sum(O.argmin(r["cost"], D, True) != gpu_best[done:done + len(sl)]))
            done += len(sl)
        one_core = done * D / t_cpu
        # the same sample over `threads` contiguous pair shards (ctypes drops the GIL inside
        # the C oracle, so the shards run on separate cores); passes repeat to >= 2 s wall
        threads = cpu_threads(args.cpu_threads)
        sample = pairs_host[:done]

        def shard(lo, hi):
            for c0 in range(lo, hi, chunk):
                sl = sample[c0:min(hi, c0 + chunk)]
                if volume_mode:
                    orc.eval_paths3d(O.gen_paths3d(sl, ut_host), vd, vox)
                else:
                    orc.eval_paths(O.gen_paths(sl, ut_host), mode=mode, rdesc=rd, rec=rec)

        bounds = np.linspace(0, done, threads + 1).astype(int)
        passes, wall = 0, 0.0
        with concurrent.futures.ThreadPoolExecutor(threads) as ex:
            while passes < 1 or (wall < 2.0 and passes < 20):
                ts = time.perf_counter()
                list(ex.map(lambda k: shard(bounds[k], bounds[k + 1]), range(threads)))
                wall += time.perf_counter() - ts
                passes += 1
        result["cpu_baseline"] = {
            "value": round(passes * done * D / wall, 1), "unit": "candidate-paths/s",
            "cores": threads, "kind": "port", "single_core_value": round(one_core, 1),
            "cpu_model": cpu_model(),
            "sample": f"first {done} of {Q} pairs x {D} displacements ({done * D} paths) "
                      f"through oracle/uam_oracle.c (gcc -O2): arc generation + {mode} "
                      f"evaluation + cost reduction; {threads} threads over contiguous pair "
                      f"shards, {passes} pass(es) in {wall:.2f} s; 1 thread: {t_cpu:.1f} s"}
        result["parity"] = {"paths_checked": done * D, "cost_mismatches": mism,
                            "best_index_mismatches": bmis,
                            "rule": "bit-exact float64 vs CPU oracle"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def workload_name(name, world):
    """The BASELINE config's name with its GPU count replaced by this run's (weak scaling:
    the per-GPU workload is the config's, the job spans `world` GPUs)."""
    import re

    base = re.sub(r",\s*\d+\s*(x|\u00d7)?\s*(MI355X|GPUs?)\s*$", "", name)
    return f"{base}, {world} GPU" + ("s" if world > 1 else "")


def cpu_threads(requested):
    """Threads for the CPU baseline: the request, else the box's CPU share (OMP_NUM_THREADS,
    which the GPU box sets to the process's share), capped by the affinity mask and 16."""
    avail = len(os.sched_getaffinity(0))
    if requested > 0:
        return max(1, min(requested, avail))
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        share = 0
    return max(1, min(share or avail, avail, 16))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
