#!/usr/bin/env python3
"""Headline benchmark: candidate-paths/s (+ waypoint-evals/s) of the batched candidate-path
cost evaluation on an R x R DEM cost raster (BASELINE.json metric), MI355X.

One "step" = one pass of the hot path over the batch resident in HBM: the spatial pair order
(K2o) and the fused kernel (arc generator K4 + raster gather / cost reduction K2) over every
pair x displacement, with the reference's candidate selection (argmin on fval and on length,
K5) fused in.  Workloads (--workload; BASELINE.json configs):

  cfg3 (default)  4096^2 DEM + 70 no-fly shapes, 100k start/goal pairs x 5 displacements =
                  500k paths x 82 waypoints PER GPU (weak scaling: every rank its own 100k
                  pairs).  The config the north_star target is quoted on.
  cfg4            8192^2 DEM written as 225 x 150 GeoTIFF tiles (mergeLL.vrt layout) and
                  ingested on rank 0, 1M paths TOTAL sharded over the GPUs (strong scaling).
  cfg5            1024 x 1024 x 64 risk volume, 100k pairs per GPU (weak scaling).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process
per GPU.  Rank 0 builds the cost raster (K1) and broadcasts it once with libuampath's RCCL
broadcast over xGMI (uam_bcast_raster; timed separately, outside the step); each rank derives
the gather-skip bitmap locally; pairs are sharded with no collective in the hot loop.  Every
rank checks the first pairs of its shard bit for bit against the CPU oracle; the mismatch
counts are summed over ranks into the line's "parity".

Prints ONE JSON line (rank 0).  roofline: algorithmic bytes per launch of the dominant kernel
(16 B per waypoint gather + 16 B of outputs per path = 16 W + 16 B/path) / its
HIP-event time vs 8 TB/s; "traffic" = the PMC-measured L2->fabric bytes per launch of the same
kernel (profiles/traffic.json, written by tools/pmc_traffic.py from the rocprofv3 passes of
this build; they include Infinity-Cache hits).  cpu_baseline: the C oracle (oracle/, a "port")
timed on this host on a bounded sample of the same workload -- one thread first (which doubles
as the bit-exact parity check on that sample), then the sample over the host's CPU share in
contiguous pair shards; `cores` is that thread count.
"""
import argparse
import concurrent.futures
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "candidate-paths/sec + waypoint-evals/sec on N×N DEM at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# independent random 16-B gathers from a 256 MiB table, one MI355X (profiles/r01/gather_ceiling.log)
RANDOM_GATHER_CEILING = 55.5e9
F64_PEAK_TFLOPS = 78.6  # MI355X f64 vector (FMA) spec; tools/f64_peak.hip measures 74.5
PARITY_PAIRS_PER_RANK = 200   # oracle check of every rank's first pairs at N > 1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg3", choices=["cfg2", "cfg3", "cfg4", "cfg5"])
    ap.add_argument("--mode", default=None, choices=["raster", "analytic", "volume"],
                    help="default: the workload's mode (raster; volume for cfg5)")
    ap.add_argument("--shard", choices=("spatial", "index"), default="spatial",
                    help="cfg4's strong-scaling shards: by space (Hilbert order of the pairs' "
                         "midpoints) or by index")
    ap.add_argument("--share", default=None,
                    help="cfg4 rehearsal on one process: R/N = rank R's shard of N ranks")
    ap.add_argument("--pairs", type=int, default=None,
                    help="override the pair count (per GPU, or in total for cfg4)")
    ap.add_argument("--R", type=int, default=None, help="override raster size")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads for the CPU baseline (0: the box's CPU share, "
                         "OMP_NUM_THREADS capped by the affinity mask and 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--group", type=int, default=None,
                    help="K2g waypoints per group (uam_set_option UAM_OPT_GROUP; 0 = K2s); "
                         "default: the library's")
    ap.add_argument("--no-skip", action="store_true",
                    help="K2 without the gather-skip bitmap (A/B; results are identical)")
    ap.add_argument("--no-pack", action="store_true",
                    help="K2s gathers the 16-B records instead of the packed copy "
                         "(uam_raster_pack: 8-B phi/terrain plane outside the no-fly blocks; "
                         "A/B, results are identical)")
    ap.add_argument("--cells", action="store_true",
                    help="also return every waypoint's raster cell index (outputs cells "
                         "[P, W] int32, the reference's returned waypoints); priced at "
                         "16 W + 16 + 4 W B/path (SURVEY §8(d))")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="libuampath context option (uam_set_option; names in _lib.OPTIONS), "
                         "repeatable: measurement sweeps of forms that give the same outputs")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived L2->fabric bytes per launch (tools/pmc_traffic.py)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one GPU per rank; UAM_BENCH_RANKS_PER_GPU > 1 packs ranks onto fewer GPUs (a rehearsal of
    # the N-rank path on a 1-GPU box, with UAM_DIST_BACKEND=gloo since RCCL needs a GPU per
    # rank).  n_gpus always reports physical GPUs.
    per_gpu = max(1, int(os.environ.get("UAM_BENCH_RANKS_PER_GPU", "1")))
    n_gpus = max(1, world // per_gpu)
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
    from uam_path_planning_amd.engine import CostRaster, Engine, VolumeGeo
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
    R, D, N = cfg["R"], cfg["D"], cfg["N"]
    W = N + 2
    mode = args.mode or cfg["mode"]
    args.mode = mode
    raster_mode = mode == "raster"
    volume_mode = mode == "volume"
    strong = args.workload == "cfg4"      # 1M paths in total, sharded over the GPUs
    Q_total = cfg["pairs"] if strong else cfg["pairs"] * world

    spec = canonical_spec(nfz_polygons=cfg["nfz_polygons"])
    geom = compile_map(build_region_map(spec))
    params = canonical_params(spec, N=N, altitude=320.0)
    eng = Engine(local)
    eng.set_geometry(geom)
    eng.set_params(params)
    ut_host = arc_table(N, displacements(D))

    # ---- cost raster / volume: rank 0 builds (K1), one RCCL broadcast --------------------
    setup = {}
    rccl = world > 1 and backend == "nccl" and per_gpu == 1
    if world > 1:
        setup["dist_backend"] = backend
        setup["ranks_per_gpu"] = per_gpu
        setup["raster_broadcast"] = ("uam_bcast_raster (RCCL, libuampath C-ABI)" if rccl else
                                     "torch.distributed.broadcast (rehearsal: ranks share a GPU)")
        if rccl:
            udist.init_raster_comm(eng)
    geo = raster_geo(R)
    raster = volume = None
    if raster_mode or volume_mode:
        t0 = time.perf_counter()
        if rank == 0:
            dem = synthetic_dem(R)
            setup["dem_gen_s"] = round(time.perf_counter() - t0, 3)
            if args.workload == "cfg4":
                # the config's "real GeoTIFF DEM": the DEM as 225 x 150 Float32 GeoTIFF tiles +
                # VRT in the mergeLL.vrt layout, read back through DataManager (device mosaic)
                from uam_path_planning_amd.map_generation import DataManager, write_tiled_dem
                tdir = tempfile.mkdtemp(prefix="uam_tiles_")
                try:
                    t1 = time.perf_counter()
                    vrt = write_tiled_dem(dem, (geo.x0, geo.dx, 0.0, geo.y_top, 0.0, -geo.dy),
                                          tdir)
                    setup["tiles_written_s"] = round(time.perf_counter() - t1, 3)
                    t1 = time.perf_counter()
                    dem_dev, g2 = DataManager(eng).load_dem(vrt)
                    torch.cuda.synchronize()
                    setup["tiles_ingest_s"] = round(time.perf_counter() - t1, 3)
                    setup["tiles"] = len(os.listdir(tdir)) - 1
                    geo = g2
                finally:
                    shutil.rmtree(tdir, ignore_errors=True)
            else:
                dem_dev = eng.tensor(dem, torch.float32)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            raster = eng.raster_build(geo, dem_dev, summary=False)
            torch.cuda.synchronize()
            setup["raster_build_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
            # K1 alone, warm (5 more builds into the same records, the median), HIP events on
            # its stream: 4 B of DEM read + 16 B of record written per cell
            k1_runs = []
            for _ in range(5):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                eng.raster_build(geo, dem_dev, out=raster.rec, summary=False)
                e1.record()
                torch.cuda.synchronize()
                k1_runs.append(e0.elapsed_time(e1))
            k1_ms = sorted(k1_runs)[len(k1_runs) // 2]
            cells = geo.nx * geo.ny
            setup["raster_build"] = {
                "cells": cells, "k1_ms": round(k1_ms, 4),
                "cells_per_s": round(cells / (k1_ms * 1e-3), 1), "bytes_per_cell": 20,
                "k1_frac_of_hbm": round(20 * cells / (k1_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)}
            if "tiles_ingest_s" in setup:
                setup["raster_build"]["tiles_ingest_plus_k1_ms"] = round(
                    setup["tiles_ingest_s"] * 1e3 + k1_ms, 3)
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
                volume = eng.volume_alloc(vg)
        if world > 1:
            dist.barrier()
            table = volume.buf if volume_mode else raster.rec
            secs = udist.broadcast_raster(table, src=0, engine=eng if rccl else None)
            setup["raster_bcast_ms"] = round(secs * 1e3, 3)
            setup["raster_bytes"] = table.numel() * 4
        if volume_mode and not args.no_pack:
            t1 = time.perf_counter()
            # every rank derives K4h's packed copy (uam_volume_pack) locally
            eng.volume_pack(volume)
            torch.cuda.synchronize()
            setup["volume_pack_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
        if raster_mode and not args.no_skip:
            t1 = time.perf_counter()
            # every rank derives the skip bitmap (and K2s's packed copy) locally
            eng.raster_summary(raster, packed=not args.no_pack)
            torch.cuda.synchronize()
            setup["skip_bitmap_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
            setup["skip_block"] = raster.block

    # ---- this rank's shard of pairs ------------------------------------------------------
    gen = random_pairs3d if volume_mode else random_pairs
    all_pairs = gen(Q_total, seed=0)
    if strong:
        # by space (distributed.spatial_shard): each rank's paths cover a compact part of the
        # raster; --share R/N rehearses rank R of an N-rank run on this one process
        srank, sworld = rank, world
        if args.share:
            srank, sworld = (int(v) for v in args.share.split("/"))
        if args.shard == "spatial":
            pairs_host, _ = udist.spatial_shard(all_pairs, srank, sworld)
        else:
            lo, hi = udist.shard_range(Q_total, srank, sworld)
            pairs_host = all_pairs[lo:hi]
    else:
        pairs_host = udist.weak_shard(all_pairs, cfg["pairs"], rank, world)
    del all_pairs
    Q = len(pairs_host)
    pairs = eng.tensor(pairs_host, torch.float64)
    ut = eng.tensor(ut_host, torch.float64)
    P = Q * D
    outs = eng.outputs(P, W, n_pairs=Q, want_cells=args.cells and not volume_mode)
    o = outs[0]
    if args.group is not None:
        eng.set_option("group", args.group)
    for kv in args.opt:
        name, val = kv.split("=", 1)
        eng.set_option(name.strip(), int(val))

    def step():
        # one call: sort + arc generation + gather + cost reduction + selection
        if volume_mode:
            eng.eval_generated3d(pairs, ut, volume, outputs=outs)
        else:
            eng.eval_generated(pairs, ut, raster=raster, outputs=outs)

    def run_steps(n):
        for _ in range(n):
            step()

    run_steps(args.warmup)
    torch.cuda.synchronize()
    # the timed region: ONE HIP event pair on the launch stream (libuampath enqueues on torch's
    # current stream) around all K steps, so no per-step marker perturbs the launches
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    run_steps(args.steps)
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    # cross-check after the timed region: the library's own HIP-event pair around each call's
    # launch sequence (uam_kernel_timing), same steps
    eng.kernel_timing(True)
    run_steps(args.steps)
    k_total, k_launches = eng.kernel_time()
    eng.kernel_timing(False)
    seq_ms = k_total / k_launches if k_launches == args.steps else None
    if world > 1:
        elapsed, kern_ms = udist.max_over_ranks([elapsed, kern_ms], device=eng.torch_device)

    # (a --share rehearsal processes one rank's shard only: its own paths)
    total_paths = (Q if args.share else Q_total) * D * args.steps
    value = total_paths / elapsed
    last = eng.last_kernel()   # which evaluation the library ran (uam_last_kernel)
    wave = last in ("K2w", "K4w")
    skip = raster_mode and not args.no_skip and raster.summary is not None
    # UAM_OPT_K2H_TERRAIN / UAM_OPT_K4H_TERRAIN: the terrain form K2h / K4h ran
    te = eng.get_option("k4h_terrain" if volume_mode else "k2h_terrain") == 1
    if last.startswith("K4h"):
        ktag = last.lower() + ("" if te else ":bounds")
        kernel_name = ("K4h sequence (k_v_hist / k_scan / k_g_scatter (+ the unit-arc sums), k_v_eval "
                       "over every (path, group) item: points, one packed voxel per waypoint"
                       + (" with its column's terrain" if te else
                          ", the column terrain where it could still decide an output") +
                       "; k_v_final: the similarity-form geometry, grouped sums, selection)")
    elif last.startswith("K2h"):
        ktag = last.lower() + ("" if te else ":bounds")
        kernel_name = ("K2h sequence (k_g_hist / k_scan / k_g_scatter (+ the unit-arc sums), "
                       "k_h_eval over every (path, group) item: points, cells, packed entries"
                       + (" with the terrain" if te else
                          " and the terrain where its bound could be the path maximum") +
                       "; k_h_final: the similarity-form geometry, grouped sums, selection)")
    elif last.startswith("K2g"):
        ktag = last.lower()
        kernel_name = ("K2g sequence (k_g_hist / k_scan / k_g_scatter, k_g_eval over every "
                       "(path, group) item with its share of pass 1, k_g_final)")
    elif last.startswith("K2s"):
        ktag = last.lower()
        kernel_name = (f"{last} sequence (k_seg_hist / k_scan / k_seg_scatter, k_seg_eval<FIRST> "
                       f"fused with pass 1, k_seg_eval, k_seg_final)")
    else:
        ktag = "wave" if wave else ("raster+skip" if skip else mode)
        kernel_name = (f"k_eval_wave<{mode}> (one wave per path)" if wave else
                       f"k_eval_pairs<{ktag}>")
    pkey = f"{args.workload}:{mode}:R{R}:Q{Q}:{ktag}" + (":cells" if args.cells else "")
    prof = {}
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                prof = json.load(f).get(pkey) or {}
        except (OSError, ValueError):
            prof = {}
    if mode == "analytic":
        roofline = analytic_roofline(prof, P, kern_ms, kernel_name)
    else:
        roofline = gather_roofline(prof, P, W, kern_ms, kernel_name,
                                   packed=last in ("K2s+pack", "K2g+pack", "K2h+pack"),
                                   kernel_tag=last,
                                   volume=volume_mode,
                                   cells=args.cells and not volume_mode,
                                   terrain_entry=te)
    roofline["kernel_ms_source"] = ("one HIP event pair (torch.cuda.Event on the launch "
                                    "stream) around the K timed steps / K: the whole launch "
                                    "sequence of every step (sorts, evaluation, output "
                                    "launch) and the GPU's gaps between steps")
    roofline["sequence_ms_library_events"] = (round(seq_ms, 4) if seq_ms is not None else None)
    roofline["library_kernel"] = last
    group = eng.last_group()   # the sum order the library used (0 = sequential)
    roofline["sum_group"] = group
    roofline["profile_key"] = pkey
    if args.opt:
        roofline["options"] = list(args.opt)
    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "candidate-paths/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (DEM seed 1 with the Nagasaki DEM's statistics, pairs seed 0, "
                "NFZ polygons seed 2; canonical map geometry from the reference data files)",
        "config": {"workload": f"{args.workload}: {workload_name(cfg, n_gpus, Q_total * D)}",
                   "dem": f"{R}x{R}", "pairs_total": Q_total, "pairs_this_rank": Q,
                   "displacements": D, "waypoints_per_path": W, "paths_total": Q_total * D,
                   "mode": mode, "no_fly_shapes": geom.n_obstacles,
                   "region_shapes": int(geom.region_first[-1] - geom.region_first[0]),
                   "parallelism": (f"pair-sharded dp{world}, raster broadcast once" +
                                   (f", {args.shard} shards" if strong else "") +
                                   (f" ({world} ranks on {n_gpus} GPU(s), rehearsal)"
                                    if world != n_gpus else "") +
                                   (f"; rank share {args.share} rehearsed on one process "
                                    f"(value: this shard's paths)" if args.share else ""))},
        "waypoint_evals_per_s": round(value * W, 1),
        "roofline": roofline,
        "setup": setup,
    }
    if world > 1:
        result["ranks"] = world

    # ---- parity at N > 1: every rank checks the first pairs of its shard --------------------
    if world > 1:
        mism = rank_parity(eng, spec, params, mode, geo, raster, volume, pairs_host, ut_host, o,
                           D, N, group)
        t = torch.tensor(mism, dtype=torch.float64,
                         device=eng.torch_device if backend == "nccl" else "cpu")
        dist.all_reduce(t)
        m = [int(x) for x in t.cpu()]
        result["parity"] = {"paths_checked": m[0], "cost_mismatches": m[1],
                            "best_index_mismatches": m[2], "ranks": world,
                            "rule": f"bit-exact float64 vs CPU oracle (sum order: "
                                    f"{order_name(group, last)}), first "
                                    f"{PARITY_PAIRS_PER_RANK} pairs of every rank's shard"}

    # ---- CPU baseline + parity sample (rank 0, N=1 only) ----------------------------------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        O.build()
        orc = O.Oracle(O.compile_spec(spec), N, spec["options"], spec["maxratio"],
                       spec["maxalpha"], spec["enlargement"], spec["weights"],
                       altitude=params.altitude)
        rd, rec, vd, vox = oracle_inputs(O, geo, raster, volume, mode)
        gpu_cost = o["cost"].cpu().numpy()
        gpu_best = o["best_fval_idx"].cpu().numpy()
        gpu_cells = o["cells"].cpu().numpy() if "cells" in o else None
        gpu_other = {k: o[k].cpu().numpy() for k in ("min_clearance", "nfz_hits", "length")}
        chunk = 50 if mode == "analytic" else 2000
        done, t_cpu, mism, bmis, cmis, omis = 0, 0.0, 0, 0, 0, 0
        while done < Q and t_cpu < args.cpu_seconds:
            sl = pairs_host[done:done + chunk]
            ts = time.perf_counter()
            r = oracle_eval(O, orc, sl, ut_host, mode, rd, rec, vd, vox, group,
                            want_cells=gpu_cells is not None, kernel=last)
            t_cpu += time.perf_counter() - ts
            mism += int(np.sum(r["cost"] != gpu_cost[done * D:(done + len(sl)) * D]))
            for gk, rk in (("min_clearance", "min_clearance"), ("nfz_hits", "nfz_hits"),
                           ("length", "length")):
                g_o = gpu_other[gk][done * D:(done + len(sl)) * D]
                omis += int(np.sum(~((r[rk] == g_o) | (np.isnan(r[rk]) & np.isnan(g_o)))))
            bmis += int(np.sum(O.argmin(r["cost"], D, True) != gpu_best[done:done + len(sl)]))
            if gpu_cells is not None:
                cmis += int(np.sum(r["cells"].reshape(-1, W) !=
                                   gpu_cells[done * D:(done + len(sl)) * D]))
            done += len(sl)
        one_core = done * D / t_cpu
        # the same sample over `threads` contiguous pair shards (ctypes drops the GIL inside
        # the C oracle, so the shards run on separate cores); passes repeat to >= 2 s wall
        threads = cpu_threads(args.cpu_threads)
        sample = pairs_host[:done]

        def shard(lo, hi):
            for c0 in range(lo, hi, chunk):
                oracle_eval(O, orc, sample[c0:min(hi, c0 + chunk)], ut_host, mode, rd, rec, vd,
                            vox, group, kernel=last)

        bounds = np.linspace(0, done, threads + 1).astype(int)
        passes, wall = 0, 0.0
        with concurrent.futures.ThreadPoolExecutor(threads) as ex:
            while passes < 1 or (wall < 2.0 and passes < 20):
                ts = time.perf_counter()
                list(ex.map(lambda k: shard(bounds[k], bounds[k + 1]), range(threads)))
                wall += time.perf_counter() - ts
                passes += 1
            seq = None
            if group and mode in ("raster", "volume"):
                # every pair of the batch through the reference's sequential order (threads
                # over pair shards): how far the grouped sums move the costs and whether they
                # move either selection
                sb = np.linspace(0, Q, threads + 1).astype(int)

                def seq_shard(k):
                    return oracle_eval(O, orc, pairs_host[sb[k]:sb[k + 1]], ut_host, mode, rd,
                                       rec, vd, vox, 0)

                parts = list(ex.map(seq_shard, range(threads)))
                seq = {key: np.concatenate([pp[key] for pp in parts])
                       for key in ("cost", "length")}
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
                            "clearance_hits_length_mismatches": omis,
                            "rule": f"bit-exact float64 vs CPU oracle (sum order: "
                                    f"{order_name(group, last)}) on the cpu_baseline sample"}
        if gpu_cells is not None:
            result["parity"]["cell_index_mismatches"] = cmis
        if seq is not None:
            ok = np.isfinite(seq["cost"])
            rel = np.abs(gpu_cost[ok] - seq["cost"][ok]) / np.maximum(np.abs(seq["cost"][ok]),
                                                                      1e-300)
            glen = o["length"].cpu().numpy()
            result["parity"]["vs_sequential_order"] = {
                "paths": int(Q * D),
                "max_rel_cost": float(rel.max()) if rel.size else 0.0,
                "max_rel_length": float(np.max(np.abs(glen[ok] - seq["length"][ok]) /
                                               np.maximum(seq["length"][ok], 1e-300))),
                "best_fval_idx_disagreements": int(np.sum(
                    O.argmin(seq["cost"], D, True) != gpu_best)),
                "best_length_idx_disagreements": int(np.sum(
                    O.argmin(seq["length"], D, False) != o["best_length_idx"].cpu().numpy())),
                "rule": "the whole batch through the reference's sequential sums "
                        "(problem.py:38-44, 130-146) against the GPU's grouped sums; "
                        "north_star tolerance 1e-5 relative on cost"}
            result["parity"]["tolerance_vs_reference"] = 1e-5
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def gather_roofline(prof, P, W, kern_ms, kernel_name, packed=False, volume=False, cells=False,
                    kernel_tag="", terrain_entry=True):
    """HBM roofline of the raster / volume kernel.  Algorithmic bytes (the one
    definition used in SURVEY, DESIGN §4 and here): raster, one 16-B record gather per waypoint
    + 16 B of outputs per path = 16 W + 16 B/path; volume, one 8-B voxel {risk, psi_nfz} + a
    4-B DEM per waypoint + 16 B of outputs = 12 W + 16.  `traffic`: L2->fabric bytes per launch of the same
    kernel from this build's rocprofv3 PMC passes (tools/pmc_traffic.py ->
    profiles/traffic.json; 2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md §HBM), which
    include Infinity-Cache hits: they are not proven DRAM bytes."""
    bytes_per_path = (12 if volume else 16) * W + 16 + (4 * W if cells else 0)
    launch_bytes = bytes_per_path * P
    achieved = launch_bytes / (kern_ms * 1e-3) / 1e9
    traffic = prof.get("l2_fabric_bytes_per_launch")
    r = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
         "traffic_label": ("L2->fabric bytes per launch (rocprofv3 PMC: 2 x FETCH_SIZE + "
                           "WRITE_SIZE; includes Infinity-Cache hits)") if traffic else None,
         "traffic_source": prof.get("source"),
         "kernel": kernel_name, "kernel_ms": round(kern_ms, 4),
         "algorithmic_bytes_per_path": bytes_per_path,
         "algorithmic_bytes_def": ("SURVEY.md §8(d), 3-D: 8-B voxel {risk, psi_nfz} + 4-B DEM "
                                   "per waypoint + 16 B output per path (12 W + 16)" if volume
                                   else "SURVEY.md §8(d): 16 B record gather per waypoint + "
                                   "16 B output per path + 4 B waypoint index per waypoint "
                                   "(16 W + 16 + 4 W)" if cells
                                   else "SURVEY.md §8(d): 16 B record gather per waypoint + "
                                   "16 B output per path (16 W + 16)"),
         "algorithmic_bytes_per_launch": launch_bytes,
         "traffic_over_algorithmic": round(traffic / launch_bytes, 2) if traffic else None,
         "l2_hit_rate": prof.get("l2_hit_rate"),
         "gathers_per_s": round(P * W / (kern_ms * 1e-3), 1),
         "random_gather_ceiling_per_s": RANDOM_GATHER_CEILING,
         "record_source": record_source(volume, packed, terrain_entry),
         "note": roofline_note(kernel_tag, prof, P, W, terrain_entry, cells)}
    return r


def record_source(volume, packed, terrain_entry):
    """The entries the evaluation that ran reads (UAM_OPT_K2H_TERRAIN picks the form)."""
    if volume:
        if terrain_entry:
            return ("packed volume (uam_volume_pack): 8-B {risk, column terrain} voxels in 4 x "
                    "4-column blocks per layer outside the no-fly / psi columns, 16-B voxels "
                    "inside them")
        return ("packed volume (uam_volume_pack): 4-B risk and 8-B {risk, psi|nfz} voxels by "
                "column-block code, 16-B voxels where a psi is negative, the 4-B column terrain "
                "only where a waypoint could still decide an output")
    if not packed:
        return "16-B records"
    tail = ("; the algorithmic bytes keep SURVEY's 16 B per waypoint, the information each "
            "waypoint consumes")
    if terrain_entry:
        return ("packed (uam_raster_pack): 8-B {phi, terrain} entries in 4 x 4-cell blocks (16 "
                "cells per line) outside the no-fly / psi blocks, 16-B records inside them, "
                "nothing in blocks of phi, psi +-0 and terrain +0.0" + tail)
    return ("packed (uam_raster_pack): 4-B phi entries (32 cells per line) and 8-B {phi, "
            "psi|nfz} entries (16 per line) by block code, 16-B records where a psi is "
            "negative, the 4-B terrain plane where a waypoint's bound could be the path "
            "maximum" + tail)


def roofline_note(kernel, prof, P, W, terrain_entry=True, cells=False):
    """What bounds the kernel that ran, from this build's own PMC key when there is one."""
    miss = prof.get("tcc_miss")
    hits = prof.get("tcc_hit")
    tail = ""
    if miss and hits:
        tail = (f" This build's PMC (profiles/traffic.json, {prof.get('source')}): "
                f"{(miss + hits) / 1e6:.1f}M L2 requests per step for {P * W / 1e6:.1f}M "
                f"waypoints, {miss / 1e6:.2f}M of them misses.")
    if kernel.startswith("K2h"):
        what = ("one 128-B line request per waypoint's packed entry, terrain included (none "
                "in code-0 blocks)" if terrain_entry else
                "one 128-B line request per waypoint's packed entry (none in code-0 blocks) "
                "plus one per terrain fetch (only where the waypoint's bound could still be the "
                "path maximum)")
        cells = (" The waypoint cells come from k_cells beside the evaluation (a lowest-"
                 "priority side stream; runs of 4 cells per path by 8-B streaming stores)."
                 if cells else "")
        return ("K2h: " + what + "; hits come from L2, misses from the Infinity Cache / HBM "
                "at <= 55-59 G lines/s (tools/gather_ceiling.hip); DESIGN.md §4-5." + cells +
                tail)
    if kernel.startswith("K4h"):
        return ("K4h: one 128-B line request per waypoint's packed voxel; misses from the "
                "Infinity Cache / HBM at <= 55-59 G lines/s; DESIGN.md §4-5." + tail)
    return ("each gathered entry costs one 128-B line request: an L2 hit or a line from the "
            "Infinity Cache / HBM; the measured random-gather ceiling (tools/gather_ceiling.hip) "
            "bounds a kernel gathering in random order (K2); DESIGN.md §4-5." + tail)


def analytic_roofline(prof, P, kern_ms, kernel_name):
    """f64 roofline of K3 (analytic mode reads 32 B per pair and writes 16 B per path, so HBM
    does not bound it): f64 FLOP per launch from this build's rocprofv3 PMC pass
    (64 lanes x (2 FMA + ADD + MUL + TRANS) per f64 VALU instruction, tools/pmc_traffic.py
    --flops) / the kernel's HIP-event time vs the f64 vector FMA peak."""
    flops = prof.get("f64_flop_per_launch")
    r = {"bound": "f64-valu", "unit": "TFLOP/s", "peak": F64_PEAK_TFLOPS,
         "kernel": kernel_name, "kernel_ms": round(kern_ms, 4),
         "achieved": round(flops / (kern_ms * 1e-3) / 1e12, 3) if flops else None,
         "frac": round(flops / (kern_ms * 1e-3) / 1e12 / F64_PEAK_TFLOPS, 4) if flops else None,
         "f64_flop_per_launch": flops, "f64_flop_per_path": (flops / P) if flops else None,
         "flop_source": prof.get("source"),
         "wait_any_frac": prof.get("wait_any_frac"), "valu_busy_frac": prof.get("valu_frac"),
         "traffic": prof.get("l2_fabric_bytes_per_launch"),
         "peak_note": "MI355X f64 vector FMA spec 78.6 TFLOP/s; tools/f64_peak.hip measures "
                      "74.5 (DESIGN.md §5)"}
    return r


def oracle_inputs(O, geo, raster, volume, mode):
    rd = rec = vd = vox = None
    if mode == "raster":
        rd = O.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                  geo.nodata, geo.dem_threshold)
        rec = raster.rec.cpu().numpy().view(np.float32)
    if mode == "volume":
        g3 = volume.geo
        vd = O.volume_desc(g3.nx, g3.ny, g3.nz, g3.x0, g3.y_top, g3.dx, g3.dy, g3.z0, g3.dz)
        vox = (volume.vox.cpu().numpy().view(np.float32),
               volume.cols.cpu().numpy().view(np.float32))
    return rd, rec, vd, vox


def oracle_eval(O, orc, pairs, ut_host, mode, rd, rec, vd, vox, group=0, want_cells=False,
                kernel=None):
    """The oracle's statement of what `kernel` (uam_last_kernel) computes: K2h -> the
    similarity form with grouped raster sums (orc_eval_generated_h), K2g -> the grouped order
    (orc_eval_paths_g), otherwise / kernel=None with group 0 -> the reference's sequential
    order."""
    if mode == "volume":
        if kernel == "K4h+pack":
            return orc.eval_generated_h(pairs, ut_host, mode="volume", vdesc=vd, vol=vox,
                                        group=group)
        return orc.eval_paths3d(O.gen_paths3d(pairs, ut_host), vd, vox)
    if kernel and kernel.startswith("K2h"):
        return orc.eval_generated_h(pairs, ut_host, rdesc=rd, rec=rec, group=group,
                                    want_cells=want_cells)
    return orc.eval_paths(O.gen_paths(pairs, ut_host), mode=mode, rdesc=rd, rec=rec,
                          group=group, want_cells=want_cells)


def order_name(group, kernel=None):
    if kernel == "K4h+pack":
        return (f"volume sums as per-path partial sums over groups of {group} waypoints, added "
                f"in group order; the geometry terms in the similarity form (oracle "
                f"orc_eval_generated_h, volume mode)")
    if kernel and kernel.startswith("K2h"):
        return (f"raster sums as per-path partial sums over groups of {group} waypoints, added "
                f"in group order; the geometry terms in the similarity form (oracle "
                f"orc_eval_generated_h)")
    return (f"per-path partial sums over groups of {group} waypoints, added in group order "
            f"(oracle orc_eval_paths_g)" if group else "sequential, the reference's")


def rank_parity(eng, spec, params, mode, geo, raster, volume, pairs_host, ut_host, o, D, N,
                group=0):
    """[paths checked, cost mismatches, best-index mismatches] of this rank's first pairs
    against the CPU oracle (the checker; run after the timed region)."""
    from oracle import oracle as O
    O.build()
    orc = O.Oracle(O.compile_spec(spec), N, spec["options"], spec["maxratio"],
                   spec["maxalpha"], spec["enlargement"], spec["weights"],
                   altitude=params.altitude)
    n = min(PARITY_PAIRS_PER_RANK, len(pairs_host))
    rd, rec, vd, vox = oracle_inputs(O, geo, raster, volume, mode)
    r = oracle_eval(O, orc, pairs_host[:n], ut_host, mode, rd, rec, vd, vox, group,
                    kernel=eng.last_kernel())
    cost = o["cost"][:n * D].cpu().numpy()
    best = o["best_fval_idx"][:n].cpu().numpy()
    return [float(n * D), float(np.sum(r["cost"] != cost)),
            float(np.sum(O.argmin(r["cost"], D, True) != best))]


def workload_name(cfg, n_gpus, paths_total):
    """The BASELINE config's name for this run: its GPU count is the run's physical GPUs."""
    import re

    base = re.sub(r",\s*\d+\s*(x|×)?\s*(MI355X|GPUs?)\s*$", "", cfg["name"])
    if cfg.get("R") == 8192:   # strong scaling: the total is fixed
        return f"{base}: {paths_total / 1e6:g}M paths over {n_gpus} GPU" + \
            ("s" if n_gpus > 1 else "")
    return f"{base}, {n_gpus} GPU" + ("s" if n_gpus > 1 else "")


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
