"""world_size-2 gloo tests (CPU) of the multi-GPU plumbing used by bench.py: weak pair
sharding, the one-time raster broadcast, max-over-ranks timing and the cross-rank best
candidate (bit-identical to the single-rank answer)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from uam_path_planning_amd import distributed as D
        from uam_path_planning_amd.synthetic import random_pairs

        res = {}
        per = 1000
        allp = random_pairs(per * world, seed=0)
        mine = D.weak_shard(allp, per, rank, world)
        res["shard_sum"] = float(mine.sum())
        res["shard_first"] = mine[0].tolist()
        # rank 0 owns the raster; others receive it
        rec = torch.zeros((32, 48, 4), dtype=torch.int32)
        if rank == 0:
            g = torch.Generator().manual_seed(123)
            rec = torch.randint(-2**31, 2**31 - 1, (32, 48, 4), dtype=torch.int32, generator=g)
        secs = D.broadcast_raster(rec, src=0)
        res["rec_checksum"] = int(rec.to(torch.int64).sum())
        res["bcast_s"] = secs

        # a CostRaster whose derived copies (skip bitmap, packed copy) were built from the
        # receiver's OLD records: after the broadcast they must not survive (distributed.py
        # broadcast_raster) -- dropped with no engine, rebuilt from the new records with one
        from uam_path_planning_amd.engine import CostRaster
        from uam_path_planning_amd.scenario import raster_geo

        def stale_raster(seed):
            g = torch.Generator().manual_seed(seed)
            r = torch.randint(-2**31, 2**31 - 1, (32, 48, 4), dtype=torch.int32, generator=g)
            return CostRaster(raster_geo(32), r, summary=torch.full((8,), 7 + rank),
                              block=8, packed=torch.full((16,), 9 + rank))

        cr = stale_raster(123 if rank == 0 else 999)
        D.broadcast_raster(cr, src=0)
        res["dropped"] = (cr.summary is None, cr.packed is None,
                          int(cr.rec.to(torch.int64).sum()))

        class _Rebuild:
            calls = []

            def raster_summary(self, raster, block, packed=False):
                # the stub "rebuilds" from the records it is handed: their checksum
                self.calls.append((block, packed))
                raster.summary = int(raster.rec.to(torch.int64).sum())
                raster.packed = raster.summary if packed else None

        cr = stale_raster(123 if rank == 0 else 999)
        rb = _Rebuild()
        D.broadcast_raster(cr, src=0, rebuild=rb)
        res["rebuilt"] = (rb.calls, cr.summary, cr.packed)

        # a RiskVolume's packed copy (K4h) is likewise stale after its buffer's broadcast
        from uam_path_planning_amd.engine import RiskVolume

        def stale_volume(seed):
            g = torch.Generator().manual_seed(seed)
            b = torch.randint(-2**31, 2**31 - 1, (4096,), dtype=torch.int32, generator=g)
            return RiskVolume(geo=None, buf=b, vox=None, cols=None,
                              packed=torch.full((16,), 5 + rank))

        vol = stale_volume(7 if rank == 0 else 8)
        D.broadcast_raster(vol, src=0)
        res["vol_dropped"] = (vol.packed is None, int(vol.buf.to(torch.int64).sum()))

        class _Repack:
            def volume_pack(self, v):
                v.packed = int(v.buf.to(torch.int64).sum())

        vol = stale_volume(7 if rank == 0 else 8)
        D.broadcast_raster(vol, src=0, rebuild=_Repack())
        res["vol_rebuilt"] = (vol.packed, int(vol.buf.to(torch.int64).sum()))
        res["max"] = D.max_over_ranks([float(rank), 10.0 - rank])

        # the RCCL communicator setup of uam_comm_init: rank 0 draws the id, every rank joins
        class _Eng:
            def comm_unique_id(self):
                assert rank == 0, "only rank 0 draws the unique id"
                return bytes(range(128))

            def comm_init(self, uid, nranks, r):
                self.joined = (uid == bytes(range(128)), nranks, r)

        e = _Eng()
        D.init_raster_comm(e)
        res["comm"] = e.joined
        # a cost vector per rank: global best must equal the single-process answer
        costs = torch.tensor(np.random.default_rng(rank + 5).uniform(1, 2, size=50))
        if rank == 1:
            costs[7] = 0.25          # global best lives on rank 1
            costs[9] = 0.25          # tie: lower global index (50 + 7) wins
        best = D.global_best(costs, local_offset=rank * 50)
        res["best"] = best
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    from uam_path_planning_amd.synthetic import random_pairs

    allp = random_pairs(2000, seed=0)
    assert out[0]["shard_first"] == allp[0].tolist()
    assert out[1]["shard_first"] == allp[1000].tolist()
    assert out[0]["shard_sum"] + out[1]["shard_sum"] == pytest.approx(float(allp.sum()))
    assert out[0]["rec_checksum"] == out[1]["rec_checksum"] != 0
    # stale derived copies: dropped without an engine, rebuilt from the broadcast records
    ck = out[0]["dropped"][2]
    assert out[0]["dropped"] == out[1]["dropped"] == (True, True, ck)
    assert out[0]["rebuilt"] == out[1]["rebuilt"] == ([(8, True)], ck, ck)
    vk = out[0]["vol_dropped"][1]
    assert out[0]["vol_dropped"] == out[1]["vol_dropped"] == (True, vk)
    assert out[0]["vol_rebuilt"] == out[1]["vol_rebuilt"] == (vk, vk)
    assert out[0]["max"] == out[1]["max"] == [1.0, 10.0]
    assert out[0]["comm"] == (True, 2, 0) and out[1]["comm"] == (True, 2, 1)
    assert out[0]["best"] == out[1]["best"] == (0.5, 57)


def test_shard_ranges_cover():
    from uam_path_planning_amd.distributed import shard_range

    for n in (0, 1, 7, 100, 12345):
        for world in (1, 2, 3, 8):
            got = [shard_range(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            assert max(h - lo for lo, h in got) - min(h - lo for lo, h in got) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_spatial_shard():
    """cfg4's strong-scaling shards by space: every pair in exactly one shard, sizes within 1,
    and each shard's midpoints compact (a Hilbert-order cut: a shard's bounding box is far
    smaller than the whole set's); NaN pairs sort last; 6-column (3-D) pairs use x/y."""
    import numpy as np

    from uam_path_planning_amd import distributed as udist
    from uam_path_planning_amd.synthetic import random_pairs

    pr = random_pairs(20000, seed=3)
    pr[5] = np.nan
    world = 8
    idx = [udist.spatial_shard(pr, r, world)[1] for r in range(world)]
    allidx = np.concatenate(idx)
    assert len(allidx) == len(pr) and len(np.unique(allidx)) == len(pr)
    assert max(map(len, idx)) - min(map(len, idx)) <= 1
    assert 5 in idx[-1]
    mid = 0.5 * (pr[:, :2] + pr[:, 2:4])
    whole = np.nanmax(mid, 0) - np.nanmin(mid, 0)
    for r in range(world - 1):
        m = mid[idx[r]]
        box = m.max(0) - m.min(0)
        assert (box[0] * box[1]) < 0.5 * whole[0] * whole[1]
    p6 = np.concatenate([pr[:, :2], np.zeros((len(pr), 1)), pr[:, 2:4], np.ones((len(pr), 1))], 1)
    np.testing.assert_array_equal(udist.spatial_shard(p6, 2, world)[1], idx[2])
    sh, ix = udist.spatial_shard(pr, 1, world)
    np.testing.assert_array_equal(sh, pr[ix])
