"""CPU-only checks of the product's host side: the C-ABI library loads and exports every
symbol include/uampath.h declares (no compute without a GPU), the geometry compiler produces
the same tables as the oracle's independent compiler, the arc table, the safe text loader and
the reference's error behaviour."""
import ctypes
import os
import re

import numpy as np
import pytest

import golden_io as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from uam_path_planning_amd import _lib, build

    build.build_library()
    return _lib.load()


def test_header_symbols_exported(lib):
    from uam_path_planning_amd import _lib

    with open(os.path.join(ROOT, "include", "uampath.h")) as f:
        text = f.read()
    declared = set(re.findall(r"^\s*(?:int|int32_t|int64_t|void|const char\*)\s+(uam_\w+)\s*\(", text,
                              re.M))
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    assert lib.uam_abi_version() == _lib.ABI_VERSION == 2


def _vpk_sections(nx, ny, nz):
    """The packed volume's sections (uampath.hip VpkDims): header (codes, bounds, superblocks),
    bound scratch, then in 4 x 8-column blocks the 4-B risk layers, the 4-B column terrain and
    the 8-B risk/psi layers, the 16-B voxel layers in 4 x 2-column blocks and the 8-B
    {risk, terrain} layers in 4 x 4-column blocks, each 256-B aligned."""
    al = lambda v: (v + 255) // 256 * 256
    w16 = lambda v: -(-v // 16) * 16
    cw = (((nx + 7) // 8) * ((ny + 7) // 8) + 15) // 16
    bsh = 3
    while (-(-nx // (1 << bsh))) * (-(-ny // (1 << bsh))) > 16384:
        bsh += 1
    bnbx, bnby = -(-nx // (1 << bsh)), -(-ny // (1 << bsh))
    hdr = w16(cw * 4) + w16(bnbx * bnby * 2) + w16(-(-bnbx // 4) * -(-bnby // 4) * 8)
    layer = ((ny + 3) // 4) * ((nx + 7) // 8) * 32
    layer44 = ((ny + 3) // 4) * ((nx + 3) // 4) * 16   # q8: 4 x 4-column blocks
    layer42 = ((ny + 1) // 2) * ((nx + 3) // 4) * 8    # v16: 4 x 2-column blocks
    return [al(hdr), al(bnbx * bnby * 8), al(layer * nz * 4), al(layer * 4), al(layer * nz * 8),
            al(layer42 * nz * 16), al(layer44 * nz * 8)]


def test_volume_packed_bytes(lib):
    """uam_volume_packed_bytes (host only) against the packed volume's sections; an invalid
    description fails loudly."""
    from uam_path_planning_amd import _lib

    for nx, ny, nz in ((1024, 1024, 64), (300, 300, 7), (1, 1, 1), (1001, 77, 3)):
        vd = _lib.VolumeDesc(nx, ny, nz, 0.0, 20.0, 60.0 / nx, 60.0 / nx, 0.0, 10.0)
        n = ctypes.c_int64()
        assert lib.uam_volume_packed_bytes(ctypes.byref(vd), ctypes.byref(n)) == _lib.UAM_OK
        assert n.value == sum(_vpk_sections(nx, ny, nz)), (nx, ny, nz)
    vd = _lib.VolumeDesc(1024, 1024, 64, 0.0, 20.0, 60.0 / 1024, 60.0 / 1024, 0.0, 10.0)
    assert lib.uam_volume_packed_bytes(ctypes.byref(vd), ctypes.byref(n)) == _lib.UAM_OK
    # 1024^2 x 64: 1 GiB of 16-B voxels, 256 MiB of risk, 512 MiB of risk/psi, 512 MiB of
    # risk/terrain, 4 MiB of terrain, a 44 KiB header (4 KiB of codes, 32 KiB of 8-column bound
    # blocks, 8 KiB of superblocks)
    assert n.value == (1024 + 256 + 512 + 512 + 4) * 2**20 + 45056 + 131072
    assert lib.uam_volume_packed_bytes(ctypes.byref(vd), None) == _lib.UAM_E_INVALID
    bad = _lib.VolumeDesc(0, 1024, 64, 0.0, 20.0, 1.0, 1.0, 0.0, 10.0)
    assert lib.uam_volume_packed_bytes(ctypes.byref(bad), ctypes.byref(n)) == _lib.UAM_E_INVALID


def test_invalid_calls_fail_loudly(lib):
    from uam_path_planning_amd import _lib

    assert lib.uam_set_geometry(None, None) == _lib.UAM_E_INVALID
    assert b"NULL" in lib.uam_last_error()
    assert lib.uam_argmin(None, None, 1, 1, 0, None, None) == _lib.UAM_E_INVALID
    assert lib.uam_bcast_raster(None, None, 16, 0, None) == _lib.UAM_E_INVALID
    assert lib.uam_comm_init(None, None, 1, 0) == _lib.UAM_E_INVALID
    assert lib.uam_bcast_raster_group(None, None, 0, 16, 0, None) == _lib.UAM_E_INVALID
    assert lib.uam_raster_summary(None, None, None, 0, None, None) == _lib.UAM_E_INVALID
    rd = _lib.RasterDesc(4096, 4096, 0.0, 20.0, 60 / 4096, 60 / 4096, -9999.0, 0.0)
    b, nbx, nby = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    assert lib.uam_raster_summary_shape(ctypes.byref(rd), 0, ctypes.byref(b), ctypes.byref(nbx),
                                        ctypes.byref(nby)) == _lib.UAM_OK
    assert (b.value, nbx.value, nby.value) == (16, 256, 256)    # 65536-bit LDS bitmap
    assert lib.uam_raster_summary_shape(ctypes.byref(rd), 8, None, None, None) == \
        _lib.UAM_E_INVALID                                        # 262144 blocks: too many
    nbytes = ctypes.c_int64()
    assert lib.uam_raster_pack_shape(ctypes.byref(rd), 0, ctypes.byref(b),
                                     ctypes.byref(nbytes)) == _lib.UAM_OK
    # header: 2-bit codes of 65536 blocks (16 KiB), 128^2 bound blocks of 32^2 cells (u16,
    # 32 KiB), 32^2 superblocks (float2, 8 KiB); the bound scratch (float2 per bound block);
    # the 4-B phi and terrain planes, the 8-B {phi, psi | nfz} plane, the 16-B record plane and
    # the 8-B {phi, terrain} plane (4 x 4-cell blocks) of 4096^2 cells
    assert (b.value, nbytes.value) == (16, 16384 + 32768 + 8192 + 8 * 16384 +
                                       (4 + 4 + 8 + 16 + 8) * 4096 * 4096)
    # a raster that is no multiple of the blocks: every section padded to whole blocks
    rd2 = _lib.RasterDesc(1000, 700, 0.0, 20.0, 0.05, 0.05, -9999.0, 0.0)
    assert lib.uam_raster_pack_shape(ctypes.byref(rd2), 4, ctypes.byref(b),
                                     ctypes.byref(nbytes)) == _lib.UAM_OK
    words = (250 * 175 * 2 + 31) // 32                 # 4-cell code blocks
    nbb = 125 * 88                                     # 8-cell bound blocks (11000 <= 16384)
    hdr = -(-words * 4 // 16) * 16 + -(-nbb * 2 // 16) * 16 + 32 * 22 * 8
    a256 = lambda v: -(-v // 256) * 256
    planes = (2 * a256(175 * 125 * 32 * 4) + a256(175 * 250 * 16 * 8) +
              a256(175 * 500 * 8 * 16) + a256(175 * 250 * 16 * 8))  # (p8: 175 x 250 blocks)
    assert (b.value, nbytes.value) == (4, a256(hdr) + a256(nbb * 8) + planes)
    assert lib.uam_raster_pack(None, None, None, 0, None, None) == _lib.UAM_E_INVALID
    assert lib.uam_eval_generated(None, 1, None, None, None, 0, None, None, 0, None, 5, None,
                                  None) == _lib.UAM_E_INVALID
    assert lib.uam_eval_generated3d(None, None, None, None, None, 0, None, 5, None,
                                    None) == _lib.UAM_E_INVALID
    assert lib.uam_device_status(None) == _lib.UAM_E_INVALID
    assert lib.uam_synchronize(None, None) == _lib.UAM_E_INVALID


def test_status_mapping():
    """The wrapper's error convention: UAM_E_INVALID -> ValueError (the reference's argument
    errors), UAM_E_DEVICE -> DeviceCheckError (a device-side check of an earlier call failed;
    its outputs are poisoned), any other status -> UamError."""
    from uam_path_planning_amd import _lib

    _lib.check(_lib.UAM_OK, "ok")
    with pytest.raises(ValueError):
        _lib.check(_lib.UAM_E_INVALID, "x")
    with pytest.raises(_lib.DeviceCheckError, match="status -6"):
        _lib.check(_lib.UAM_E_DEVICE, "x")
    assert issubclass(_lib.DeviceCheckError, _lib.UamError)
    with pytest.raises(_lib.UamError):
        _lib.check(_lib.UAM_E_HIP, "x")
    assert _lib.OPTIONS["test_sort_fault"] == 22


def _specs():
    meta, _ = G.canonical()
    yield "canonical", meta["map"]
    for i, c in enumerate(G.random_cases()):
        yield f"random{i}", c["map"]
    from uam_path_planning_amd.scenario import canonical_spec
    yield "cfg3", canonical_spec(nfz_polygons=64)


@pytest.mark.parametrize("name,spec", list(_specs()))
def test_compiler_matches_oracle(oracle_mod, name, spec):
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map

    ours = compile_map(build_region_map(spec))
    ref = oracle_mod.compile_spec(spec)
    for k in ("ineq_kind", "ineq_par", "shape_first", "shape_count", "shape_center",
              "region_first"):
        np.testing.assert_array_equal(getattr(ours, k), getattr(ref, k), err_msg=k)
    assert ours.n_obstacles == ref.n_obstacles and ours.n_regions == ref.n_regions


def test_arc_table_matches_oracle(oracle_mod):
    from uam_path_planning_amd.arcs import arc_table

    ds = [-1.0, -0.95, -0.5, -1e-3, 0.0, 1e-3, 0.25, 0.5, 1.0]
    for N in (1, 4, 80, 254):
        np.testing.assert_array_equal(arc_table(N, ds), oracle_mod.arc_table(N, ds))


def test_reference_errors():
    from uam_path_planning_amd.arcs import check_displacement
    from uam_path_planning_amd.path_generation import RegionMap, ball, polygon

    errs = G.errors()
    for case, pts in (("polygon_two_points", [[0.0, 0.0], [1.0, 0.0]]),
                      ("polygon_collinear", [[0.0, 0.0], [1.0, 0.0], [2.0, 0.0], [1.0, 1.0]]),
                      ("polygon_nonconvex", [[0.0, 0.0], [4.0, 0.0], [1.0, 1.0], [0.0, 4.0]])):
        with pytest.raises(ValueError) as ei:
            polygon(*pts)
        assert str(ei.value) == errs[case]["message"]
    polygon([0.0, 0.0], [1.0, 0.0], [1.0, 1.0], [0.0, 1.0])
    with pytest.raises(ValueError) as ei:
        check_displacement(1.5)
    assert str(ei.value) == errs["arc_displacement_gt1"]["message"]
    m = RegionMap()
    m.new_region("A", "Red")
    with pytest.raises(ValueError) as ei:
        m.new_region("A", "Blue")
    assert str(ei.value) == errs["region_duplicate"]["message"]
    with pytest.raises(ValueError) as ei:
        m.add_shape_to_region("B", ball([0, 0], 1))
    assert str(ei.value) == errs["region_unknown"]["message"]
    # mixed int/float vertices: the reference's numpy casting error
    with pytest.raises(TypeError):
        polygon([0, 0], [1.5, 0.0], [1.0, 1.0])


def test_polygon_properties():
    from uam_path_planning_amd.path_generation import polygon

    sq = polygon([0.0, 0.0], [0.0, 2.0], [2.0, 2.0], [2.0, 0.0])
    assert sq.area == pytest.approx(4.0)
    np.testing.assert_allclose(np.asarray(sq.center).reshape(-1), [1.0, 1.0])
    assert len(sq) == 4
    for h in sq.inequalities:       # inside -> all h < 0 (host evaluation of the Function API)
        assert h([1.0, 1.0]) < 0


def test_safe_loader(tmp_path):
    from uam_path_planning_amd.path_generation.utils import get_var_from_file

    p = tmp_path / "area.txt"
    p.write_text("vertices = [polygon([0.0, 0.0], [1.0, 0.0], [1.0, 1.0]),\n"
                 "ball([2.0, 2.0], 1.5)\n]")
    shapes = get_var_from_file(str(p), "vertices")
    assert len(shapes) == 2 and len(shapes[0]) == 3 and len(shapes[1]) == 1
    p.write_text("import os\nvertices = [polygon([0, 0], [1, 0], [1, 1])]")
    with pytest.raises(ValueError):
        get_var_from_file(str(p), "vertices")
    p.write_text("vertices = [__import__('os').system('true')]")
    with pytest.raises(ValueError):
        get_var_from_file(str(p), "vertices")


def test_engine_refuses_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from uam_path_planning_amd.engine import Engine

    with pytest.raises(RuntimeError, match="no GPU"):
        Engine(0)


def test_synthetic_dem_statistics():
    from uam_path_planning_amd import synthetic as S

    dem = S.synthetic_dem(256)
    valid = dem != S.NODATA
    assert abs(valid.mean() - S.DEM_VALID) < 0.01
    v = dem[valid].astype(np.float64)
    assert v.min() >= S.DEM_MIN - 1e-3 and v.max() <= S.DEM_MAX + 1e-3
    assert abs(v.mean() - S.DEM_MEAN) < 15 and abs(v.std() - S.DEM_STD) < 15


def test_function_compose_host():
    """Function.compose (function.py:122-157): h(A x + b) on the host callables, the
    reference's shape errors, and the device spec dropped (map compilation rejects it)."""
    import numpy as np
    import pytest

    from uam_path_planning_amd.geometry import compile_shapes
    from uam_path_planning_amd.path_generation import ball

    obs = ball([1.0, 2.0], 1.0, 2.0)
    h = obs.inequalities[0]
    x = np.array([[3.0], [1.0]])
    ref = float(np.asarray(h(np.array([[3.0 * 2.0 + 0.5], [1.0 * 2.0 - 1.0]]))).reshape(-1)[0])
    h.compose(np.array([[2.0]]), np.array([[0.5], [-1.0]]))
    assert float(np.asarray(h(x)).reshape(-1)[0]) == ref
    assert h.spec is None
    with pytest.raises(ValueError):
        compile_shapes([obs], [])
    with pytest.raises(ValueError, match="translation vector"):
        ball([0.0, 0.0], 1.0).inequalities[0].compose(np.eye(2), np.zeros(2))
    with pytest.raises(ValueError, match="scaling matrix"):
        ball([0.0, 0.0], 1.0).inequalities[0].compose(np.eye(3))


def test_bench_roofline_bookkeeping():
    """bench.py's roofline fields are recomputable from the line alone: frac = (16 W + 16) B x
    paths / kernel_ms / 8 TB/s, traffic and its ratio from the PMC record."""
    import bench

    prof = {"l2_fabric_bytes_per_launch": 4.264e9, "l2_hit_rate": 0.14, "source": "x"}
    r = bench.gather_roofline(prof, 500_000, 82, 0.7105, "k")
    assert r["algorithmic_bytes_per_path"] == 1328
    assert r["algorithmic_bytes_per_launch"] == 1328 * 500_000
    assert abs(r["frac"] - 1328 * 500_000 / 0.7105e-3 / 1e9 / 8000.0) < 1e-4
    assert r["traffic"] == 4.264e9 and abs(r["traffic_over_algorithmic"] - 6.42) < 0.01
    assert "Infinity-Cache" in r["traffic_label"]
    a = bench.analytic_roofline({"f64_flop_per_launch": 1.3e10}, 500_000, 3.55, "k3b")
    assert a["unit"] == "TFLOP/s" and abs(a["achieved"] - 1.3e10 / 3.55e-3 / 1e12) < 1e-3
    assert bench.analytic_roofline({}, 1, 1.0, "k")["frac"] is None


DIV_CHECK_C = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
/* q0 = a RN(1/N); q = RN(q0 + RN(a - q0 N) RN(1/N)) against RN(a / N) for every 24-bit
   significand a in [2^23, 2^24) and N in [lo, hi] */
int main(int argc, char** argv) {
    const int lo = atoi(argv[1]), hi = atoi(argv[2]);
    long bad = 0;
#pragma omp parallel for schedule(dynamic) reduction(+ : bad)
    for (int n = lo; n <= hi; ++n) {
        const double dn = (double)n, y = 1.0 / dn;
        for (uint32_t m = 1u << 23; m < (1u << 24); ++m) {
            const double a = (double)m, q0 = a * y;
            if (fma(fma(-q0, dn, a), y, q0) != a / dn) ++bad;
        }
    }
    printf("%ld\n", bad);
    return 0;
}
"""


@pytest.mark.parametrize("lo,hi", [(1, 160), (4000, 4096)])
def test_k2g_phi_over_n_division(tmp_path, lo, hi):
    """k_g_eval forms Phi / N as q0 = a (1/N) plus one fma residual step (Markstein) instead of
    the IEEE division, which must give the same bits: Phi is a float, so a = m 2^e with a
    24-bit significand m, and in double every step scales exactly by 2^e (no under- or
    overflow for float magnitudes over N <= 4096), so checking all 2^23 significands per N
    covers every finite float.  Zero and infinity are handled apart in the kernel.  The full
    range 1..4096 was checked the same way (0 mismatches); the CPU suite runs two slices."""
    import shutil
    import subprocess

    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc not available")
    src = tmp_path / "div.c"
    src.write_text(DIV_CHECK_C)
    exe = tmp_path / "div"
    subprocess.run([cc, "-O2", "-fopenmp", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"],
                   check=True)
    out = subprocess.run([str(exe), str(lo), str(hi)], check=True, capture_output=True, text=True)
    assert int(out.stdout.strip()) == 0
