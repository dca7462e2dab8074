"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL over xGMI on the GPU box,
gloo for CPU tests).

The path shards with no data-path collective: pairs are independent and every displacement of a
pair stays on one rank, so the reference's per-pair selection (main.py:175-180) is local.  The
only exchange is the one-time broadcast of the cost raster from the rank that built it, plus
scalar max/all-gather reductions outside the timed region.
"""
import os
import time


def _dist():
    import torch.distributed as dist

    return dist


def env_rank():
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single rank)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n, rank, world):
    """Contiguous shard [lo, hi) of n items for rank r of world (sizes differ by <= 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} of world {world}")
    return n * rank // world, n * (rank + 1) // world


def hilbert_keys(x, y, bits=10):
    """Hilbert-curve index of points (x, y) on a 2^bits x 2^bits grid over their bounding box
    (host numpy; NaN coordinates sort last)."""
    import numpy as np

    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    ok = np.isfinite(x) & np.isfinite(y)
    n = 1 << bits
    if ok.any():
        x0, x1, y0, y1 = x[ok].min(), x[ok].max(), y[ok].min(), y[ok].max()
    else:
        x0 = x1 = y0 = y1 = 0.0
    sx = (n - 1) / (x1 - x0) if x1 > x0 else 0.0
    sy = (n - 1) / (y1 - y0) if y1 > y0 else 0.0
    xi = np.where(ok, np.clip((x - x0) * sx, 0, n - 1), 0).astype(np.int64)
    yi = np.where(ok, np.clip((y - y0) * sy, 0, n - 1), 0).astype(np.int64)
    d = np.zeros(len(x), np.int64)
    s = n >> 1
    while s > 0:  # the classic xy -> d walk, vectorised
        rx = (xi & s) > 0
        ry = (yi & s) > 0
        d += s * s * ((3 * rx) ^ ry)
        flip = ~ry
        swap_x = np.where(flip & rx, s - 1 - xi, xi)
        swap_y = np.where(flip & rx, s - 1 - yi, yi)
        xi, yi = np.where(flip, swap_y, xi), np.where(flip, swap_x, yi)
        s >>= 1
    return np.where(ok, d, np.int64(1) << (2 * bits))


def spatial_shard(global_pairs, rank, world, bits=10):
    """Strong scaling by space: the pairs in the order of their midpoints on a Hilbert curve,
    cut into world contiguous shards (sizes differ by <= 1), so a rank's paths cover a compact
    part of the raster and its sorted evaluation keeps the single-GPU problem's density of
    paths per raster line.  Returns (this rank's pairs, their indices in global_pairs)."""
    import numpy as np

    pr = np.asarray(global_pairs)
    ex = 3 if pr.shape[1] == 6 else 2  # (pairs3d: x0 y0 z0 xf yf zf)
    mx = 0.5 * (pr[:, 0] + pr[:, ex])
    my = 0.5 * (pr[:, 1] + pr[:, ex + 1])
    order = np.argsort(hilbert_keys(mx, my, bits), kind="stable")
    lo, hi = shard_range(len(pr), rank, world)
    idx = order[lo:hi]
    return pr[idx], idx


def weak_shard(global_pairs, per_rank, rank, world):
    """Weak scaling: every rank owns per_rank consecutive pairs of one seeded global set."""
    if len(global_pairs) < per_rank * world:
        raise ValueError("global pair set smaller than per_rank * world")
    return global_pairs[rank * per_rank:(rank + 1) * per_rank]


def init_raster_comm(engine, group=None):
    """Join every rank's engine to one RCCL communicator of libuampath (uam_comm_init): rank 0
    draws the unique id, the process group ships its 128 bytes (an object broadcast, so gloo
    and nccl groups both work), every rank joins.  Collective."""
    dist = _dist()
    obj = [engine.comm_unique_id() if dist.get_rank(group) == 0 else None]
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=group)
    engine.comm_init(obj[0], dist.get_world_size(group), dist.get_rank(group))


def broadcast_raster(raster, src=0, group=None, engine=None, rebuild=None):
    """Broadcast the record raster in place from global rank src; returns seconds taken
    (synchronised on the tensor's device before and after).

    raster: a CostRaster, whose rec is broadcast and whose derived copies -- the gather-skip
    bitmap (summary) and the packed copy K2h / K2g / K2s read (packed) -- were built from the
    receiver's OLD records, so they are rebuilt from the broadcast records with `rebuild`
    (default: `engine`) or, with no engine at hand, dropped (the evaluation then gathers rec);
    a RiskVolume, whose buffer is broadcast and whose packed copy (K4h) is rebuilt
    (`volume_pack`) or dropped the same way; or a bare tensor (rec of a CostRaster, a volume's
    buffer), broadcast as is -- its caller owns any derived copy.  With an engine whose communicator init_raster_comm set up, the
    bytes move by libuampath's RCCL broadcast (uam_bcast_raster, xGMI on the GPU node), whose
    ranks are the process group's ranks (src is converted); without one (CPU tensors: the gloo
    tests, or several ranks sharing one GPU in a rehearsal) by torch.distributed.broadcast."""
    import torch

    dist = _dist()
    volume = hasattr(raster, "buf") and hasattr(raster, "packed")
    rec = raster.buf if volume else getattr(raster, "rec", raster)
    dev = rec.device
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if engine is not None:
        root = dist.get_group_rank(group, src) if group is not None else src
        engine.bcast_raster(rec, root=root)
    else:
        dist.broadcast(rec, src=src, group=group)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    secs = time.perf_counter() - t0
    eng = rebuild if rebuild is not None else engine
    if volume:
        if raster.packed is not None:
            if eng is not None:
                eng.volume_pack(raster)
            else:
                raster.packed = None
    elif rec is not raster and (raster.summary is not None or raster.packed is not None):
        if eng is not None:
            eng.raster_summary(raster, raster.block, packed=raster.packed is not None)
        else:
            raster.summary = raster.packed = None
    return secs


def max_over_ranks(values, device=None):
    """Element-wise max of a list of floats over all ranks."""
    import torch

    dist = _dist()
    t = torch.tensor([float(v) for v in values], dtype=torch.float64,
                     device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def global_best(local_values, local_offset, take_sqrt=True):
    """Best candidate over all ranks with the reference's rule (strict '<' on fval =
    sqrt(cost), ties to the lowest global index, NaN never wins) -- identical to the single
    GPU answer.  local_values: 1-D CPU float64 tensor of this rank's per-path costs."""
    import torch

    dist = _dist()
    v = local_values.to(torch.float64)
    f = torch.sqrt(v) if take_sqrt else v
    ok = ~torch.isnan(f)
    if ok.any():
        fv = torch.where(ok, f, torch.full_like(f, float("inf")))
        i = int(torch.argmin(fv))           # torch.argmin returns the first minimum
        cand = torch.tensor([float(f[i]), float(local_offset + i)], dtype=torch.float64)
    else:
        cand = torch.tensor([float("nan"), float("inf")], dtype=torch.float64)
    world = dist.get_world_size()
    allc = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(allc, cand)
    best_v, best_i = float("nan"), -1
    for c in allc:
        cv, ci = float(c[0]), c[1]
        if cv != cv:
            continue
        if best_i < 0 or cv < best_v or (cv == best_v and ci < best_i):
            best_v, best_i = cv, int(ci)
    return best_v, best_i
