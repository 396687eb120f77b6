"""The evalio pipeline mirror form_amd.fmx.FORM (python/bindings.cpp:48-180) on the
GPU against the CPU oracle (VERDICT r2 "next round" 7): a stream driven through
set_params / set_lidar_params / set_imu_T_lidar / initialize / add_lidar, with the
returned features, pose() and map() (fmx_map_download) checked scan by scan, and the
reference config's ablations (config/25.10.03_full.yaml:9-17) run end to end."""
import types

import numpy as np
import pytest

from form_amd import synth

pytestmark = pytest.mark.gpu


def _lidar(geo):
    return types.SimpleNamespace(min_range=1.0, max_range=100.0, num_rows=geo.rows, num_columns=geo.cols)


def _oracle_est(oracle, p, entry):
    prm = oracle.default_params(p)
    if entry.get("disable_smoothing"):
        prm.disable_smoothing = 1
    if "point_feats_per_sector" in entry:
        prm.extraction.point_feats_per_sector = entry["point_feats_per_sector"]
    return oracle.Estimator(prm)


def _imu_T_lidar():
    T = np.eye(4)
    c, s = np.cos(0.3), np.sin(0.3)
    T[:3, :3] = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    T[:3, 3] = [0.1, -0.05, 0.2]
    return T


def _check_map(got, ref, w):
    """fmx map() == oracle map(): the same records per scan (world positions within
    1e-6: the poses agree to ~1e-8), grouped voxel by voxel, push_back order inside."""
    for name in ("planar", "point"):
        g, (rx, _, rs) = got[name], ref[name]
        assert len(g) == len(rx), name
        gs = g[:, 3].astype(np.uint64)
        assert np.array_equal(np.sort(gs), np.sort(rs))
        for s in np.unique(rs):
            a = g[gs == s, :3]
            b = rx[rs == s]
            a = a[np.lexsort(a.T[::-1])]
            b = b[np.lexsort(b.T[::-1])]
            assert np.abs(a - b).max() < 1e-6, (name, s)
        # grouping: each voxel's records contiguous, scans non-decreasing inside a voxel
        cells = np.floor(g[:, :3] / w).astype(np.int64)
        change = np.any(cells[1:] != cells[:-1], axis=1)
        assert change.sum() + 1 == len(np.unique(cells, axis=0)) if len(g) else True
        same = ~change
        assert np.all(gs[1:][same] >= gs[:-1][same])


@pytest.mark.parametrize("entry", [{"pipeline": "form"},
                                   {"pipeline": "form", "name": "form_single", "disable_smoothing": True}])
def test_form_pipeline_stream_matches_oracle(fmx_mod, oracle, entry):
    geo = synth.GEOMETRIES["c2"]
    p = synth.default_params(geo)
    world = synth.World()
    f = fmx_mod.FORM()
    f.set_params(entry)
    f.set_lidar_params(_lidar(geo))
    imu_T_lidar = _imu_T_lidar()
    f.set_imu_T_lidar(imu_T_lidar)
    f.initialize()
    assert bool(f.params.disable_smoothing) == bool(entry.get("disable_smoothing", False))
    oest = _oracle_est(oracle, p, entry)
    for k in range(10):
        s, _, _ = synth.make_scan("c2", k, world=world)
        xyz = s.numpy()[:, :3].astype(np.float64)
        feats = f.add_lidar(types.SimpleNamespace(points=xyz))
        To, _, _ = oest.register_scan(s.numpy())
        ex = oracle.extract(s.numpy(), p)
        pl_ref, pt_ref = oracle.features_from(s.numpy(), ex)
        assert np.array_equal(feats["planar"][:, :3], pl_ref[:, :3].astype(np.float64))
        assert np.array_equal(feats["point"][:, :3], pt_ref.astype(np.float64))
        assert np.all(feats["planar"][:, 3] == k) and np.all(feats["point"][:, 3] == k)
        To44 = np.eye(4)
        To44[:3] = To
        assert np.abs(f.pose() - To44 @ np.linalg.inv(imu_T_lidar)).max() < 1e-6, k
        if k in (0, 4, 9):
            _check_map(f.map(), oest.map(), f.params.min_dist_map)


def test_form_single_ablation_is_single_pose(fmx_mod, oracle):
    """disable_smoothing: true (config/25.10.03_full.yaml:15-17) registers like the
    oracle's single-pose mode, and not like its smoothing mode."""
    geo = synth.GEOMETRIES["tiny"]
    p = synth.default_params(geo)
    world = synth.World()
    f = fmx_mod.FORM()
    f.set_params({"pipeline": "form", "name": "form_single", "disable_smoothing": True})
    f.set_lidar_params(_lidar(geo))
    f.initialize()
    single = _oracle_est(oracle, p, {"disable_smoothing": True})
    smooth = _oracle_est(oracle, p, {})
    dsm = 0.0
    for k in range(12):
        s, _, _ = synth.make_scan("tiny", k, world=world)
        f.add_lidar(s.numpy()[:, :3])
        Ts, _, _ = single.register_scan(s.numpy())
        Tm, _, _ = smooth.register_scan(s.numpy())
        assert np.abs(f.pose()[:3] - Ts).max() < 1e-6, k
        dsm = max(dsm, float(np.abs(Ts - Tm).max()))
    assert dsm > 1e-5  # the two modes do differ on this stream


def test_form_planar_ablation(fmx_mod, oracle):
    """point_feats_per_sector: 0 (config/25.10.03_full.yaml:12-14): no point features
    (extraction.tpp:366-368), planar-only registration equal to the oracle's."""
    geo = synth.GEOMETRIES["small"]
    p = synth.default_params(geo)
    world = synth.World()
    f = fmx_mod.FORM()
    f.set_params({"pipeline": "form", "name": "form_planar", "point_feats_per_sector": 0})
    f.set_lidar_params(_lidar(geo))
    f.initialize()
    p0 = dict(p, point_feats_per_sector=0)
    oest = _oracle_est(oracle, p0, {"point_feats_per_sector": 0})
    for k in range(8):
        s, _, _ = synth.make_scan("small", k, world=world)
        feats = f.add_lidar(s.numpy()[:, :3])
        assert len(feats["point"]) == 0 and len(feats["planar"]) > 100
        To, _, _ = oest.register_scan(s.numpy())
        assert np.abs(f.pose()[:3] - To).max() < 1e-6, k
    assert len(f.map()["point"]) == 0


def test_map_download_edge_cases(fmx_mod):
    """fmx_map_download before any registered scan is a state error; a buffer smaller
    than the map is a size error; the size query needs no buffers."""
    import ctypes as C
    geo = synth.GEOMETRIES["tiny"]
    p = synth.default_params(geo)
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams(extraction=fmx_mod.KeypointExtractionParams(**p)))
    with pytest.raises(fmx_mod.FmxError) as e:
        ctx.map_download(0.1)
    assert e.value.status == 5  # FMX_E_STATE
    world = synth.World()
    for k in range(3):
        ctx.register_scan(synth.make_scan("tiny", k, world=world)[0].to("cuda:0"))
    L = fmx_mod.lib()
    npl, npt = C.c_uint32(0), C.c_uint32(0)
    assert L.fmx_map_download(ctx.h, C.c_double(0.1), None, None, C.byref(npl), None, None, C.byref(npt)) == 0
    assert npl.value > 0 and npt.value > 0
    small = np.zeros(6 * (npl.value - 1))
    cap, cap2 = C.c_uint32(npl.value - 1), C.c_uint32(npt.value)
    pt = np.zeros(3 * npt.value)
    st = L.fmx_map_download(ctx.h, C.c_double(0.1), small.ctypes.data_as(C.c_void_p), None, C.byref(cap),
                            pt.ctypes.data_as(C.c_void_p), None, C.byref(cap2))
    assert st == 2  # FMX_E_SIZE
    assert L.fmx_map_download(ctx.h, C.c_double(0.0), None, None, C.byref(npl), None, None, C.byref(npt)) == 1
    m = ctx.map_download(0.1)
    assert len(m["planar"][0]) == npl.value and len(m["point"][0]) == npt.value
    ctx.close()
