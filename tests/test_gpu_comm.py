"""The RCCL raster broadcast of the C-ABI (uam_comm_unique_id / uam_comm_init /
uam_bcast_raster / uam_bcast_raster_group) on one GPU: world size 1, so the broadcast must
leave the root's bytes intact; through distributed.init_raster_comm + broadcast_raster, the
path bench.py takes at N > 1 (one broadcast, no collective in the hot loop;
the sharded loop is main.py:160-193)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def eng():
    from uam_path_planning_amd.engine import Engine

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    return Engine(0)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_comm_world1_bcast(eng):
    uid = eng.comm_unique_id()
    assert len(uid) == 128
    eng.comm_init(uid, 1, 0)
    g = torch.Generator().manual_seed(5)
    host = torch.randint(-2**31, 2**31 - 1, (257, 300, 4), dtype=torch.int32, generator=g)
    rec = host.to("cuda")
    eng.bcast_raster(rec, root=0)
    torch.cuda.synchronize()
    assert torch.equal(rec.cpu(), host)
    with pytest.raises(ValueError):
        eng.bcast_raster(host)          # host tensors are refused


def test_init_raster_comm_and_broadcast(eng):
    import torch.distributed as dist

    from uam_path_planning_amd import distributed as udist
    from uam_path_planning_amd.scenario import canonical_spec, canonical_params, raster_geo
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map
    from uam_path_planning_amd.synthetic import synthetic_dem

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        udist.init_raster_comm(eng)
        spec = canonical_spec(nfz_polygons=4)
        eng.set_geometry(compile_map(build_region_map(spec)))
        eng.set_params(canonical_params(spec, N=20))
        r = eng.raster_build(raster_geo(512), synthetic_dem(512))
        before = r.rec.cpu().numpy().copy()
        secs = udist.broadcast_raster(r.rec, src=0, engine=eng)
        assert secs >= 0
        np.testing.assert_array_equal(r.rec.cpu().numpy(), before)
    finally:
        dist.destroy_process_group()


def test_bcast_raster_group_single_process(eng):
    from uam_path_planning_amd import _lib
    import ctypes

    lib = _lib.load()
    t = torch.arange(4096, dtype=torch.int32, device="cuda")
    ctxs = (ctypes.c_void_p * 1)(eng._ctx.value)
    bufs = (ctypes.c_void_p * 1)(t.data_ptr())
    _lib.check(lib.uam_bcast_raster_group(ctxs, bufs, 1, t.numel() * 4, 0, None),
               "uam_bcast_raster_group")
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(4096, dtype=torch.int32))
    # the group's communicator stays with the context
    eng.bcast_raster(t, root=0)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(4096, dtype=torch.int32))


def test_kernel_timing_events(eng):
    """uam_kernel_timing / uam_kernel_time (bench.py's kernel_ms): one event pair per launch of
    the dominant kernel on the launch stream, none while stopped, reset by each query."""
    import numpy as np

    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec()
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=40))
    ut = arc_table(40, displacements(5))
    raster = eng.raster_build(raster_geo(256), synthetic_dem(256))
    pairs = random_pairs(5000, seed=1)
    eng.kernel_timing(True)
    for _ in range(3):
        eng.eval_generated(pairs, ut, raster=raster)
    eng.eval_generated(pairs, ut)               # analytic (K3b) counts too
    ms, n = eng.kernel_time()
    assert n == 4 and np.isfinite(ms) and ms > 0.0
    assert eng.kernel_time() == (0.0, 0)        # the query resets
    eng.kernel_timing(False)
    eng.eval_generated(pairs, ut, raster=raster)
    assert eng.kernel_time() == (0.0, 0)
