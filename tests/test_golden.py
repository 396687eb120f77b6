"""Committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture bit for bit (regression pin of the
oracle).  GPU: the HIP path through the C-ABI matches the fixtures — exact indices
and pair assignments, G within 1e-10 relative, poses within 1e-6.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def test_oracle_reproduces_extract(oracle):
    g = load("extract_tiny.npz")
    p = json.loads(str(g["params"]))
    ex = oracle.extract(g["scan"], p)
    for k in ("sel", "normal_ok", "normals", "point_idx", "planar_mask", "point_mask", "curvature"):
        assert np.array_equal(ex[k], g[k]), k


def _maps(oracle, g):
    w = float(g["voxel_width"])
    maps = [oracle.VoxelMap(w, 0), oracle.VoxelMap(w, 1)]
    for k in range(4):
        maps[0].add_scan(k, g["poses"][k], g[f"map_planar_{k}"])
        maps[1].add_scan(k, g["poses"][k], g[f"map_point_{k}"])
    return maps


def test_oracle_reproduces_match(oracle):
    g = load("match_tiny.npz")
    mp, mt = _maps(oracle, g)
    a = mp.match(g["q_planar"], g["pose_j"])
    b = mt.match(g["q_point"], g["pose_j"])
    for k in ("found", "scan", "d2", "pi", "ni"):
        assert np.array_equal(a[k], g["pl_" + k]), k
    for k in ("found", "scan", "d2", "pi"):
        assert np.array_equal(b[k], g["pt_" + k]), k


def test_oracle_reproduces_linearize(oracle):
    g = load("linearize_small.npz")
    args = [g[k] for k in ("n_plane", "plane_pi", "plane_ni", "plane_pj", "n_point", "point_pi", "point_pj",
                           "poses_i", "poses_j")]
    G, err = oracle.linearize(*args, float(g["sigma"]), False)
    assert np.array_equal(G, g["G"]) and np.array_equal(err, g["err"])
    G1, err1 = oracle.linearize(*args, float(g["sigma"]), True)
    assert np.array_equal(G1, g["G_single"]) and np.array_equal(err1, g["err_single"])


@pytest.mark.parametrize("name", ["stream_tiny.npz", "stream_tiny_smooth.npz"])
def test_oracle_reproduces_stream(oracle, name):
    g = load(name)
    p = json.loads(str(g["params"]))
    prm = oracle.default_params(p)
    prm.disable_smoothing = int(g["disable_smoothing"])
    prm.max_num_recent_scans, prm.max_num_keyscans = (int(v) for v in g["window"])
    est = oracle.Estimator(prm, 1)
    for k in range(len(g["scans"])):
        T, st, _ = est.register_scan(g["scans"][k])
        assert np.array_equal(T, g["poses"][k])
        assert np.array_equal(st, g["stats"][k])


# ------------------------------------------------------------------ GPU vs fixtures
def _ctx(fmx, p):
    return fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**p)))


@pytest.mark.gpu
def test_gpu_extract_golden(fmx_mod):
    g = load("extract_tiny.npz")
    p = json.loads(str(g["params"]))
    ctx = _ctx(fmx_mod, p)
    ctx.extract(g["scan"], 0)
    d = ctx.extract_download(with_mask=True)
    ok = g["normal_ok"]
    assert np.array_equal(d["planar_index"], g["sel"][ok])
    assert np.array_equal(d["point_index"], g["point_idx"])
    assert np.array_equal(d["planar_mask"], g["planar_mask"])
    assert np.abs(np.sum(d["planar"][:, 3:] * g["normals"][ok], 1)).min() >= 1 - 1e-6


@pytest.mark.gpu
def test_gpu_match_golden(fmx_mod):
    g = load("match_tiny.npz")
    ctx = _ctx(fmx_mod, json.loads(str(load("extract_tiny.npz")["params"])))
    for k in range(4):
        ctx.keypoints_add(k, g[f"map_planar_{k}"], g[f"map_point_{k}"])
    ctx.map_build(np.arange(4), g["poses"], float(g["voxel_width"]))
    ctx.set_queries(g["q_planar"], g["q_point"], 4)
    ctx.match(g["pose_j"], float(g["voxel_width"]))
    m = ctx.match_download()
    npl = len(g["q_planar"])
    md2 = float(g["voxel_width"]) ** 2
    for sl, pre in ((slice(0, npl), "pl_"), (slice(npl, None), "pt_")):
        acc = g[pre + "found"] & (g[pre + "d2"] < md2)
        assert np.array_equal(m["pair"][sl] >= 0, acc)
        assert np.array_equal(m["pair"][sl][acc].astype(np.uint64), g[pre + "scan"][acc])
        assert np.array_equal(m["pi"][sl][acc], g[pre + "pi"][acc])
    acc = g["pl_found"] & (g["pl_d2"] < md2)
    assert np.array_equal(m["ni"][acc], g["pl_ni"][acc])


@pytest.mark.gpu
def test_gpu_linearize_golden(fmx_mod):
    g = load("linearize_small.npz")
    ctx = _ctx(fmx_mod, json.loads(str(load("extract_tiny.npz")["params"])))
    ctx.corr_set(*[g[k] for k in ("n_plane", "plane_pi", "plane_ni", "plane_pj", "n_point", "point_pi", "point_pj")])
    for single, Gk, ek in ((False, "G", "err"), (True, "G_single", "err_single")):
        G, err = ctx.linearize(g["poses_i"], g["poses_j"], float(g["sigma"]), single)
        scale = np.abs(g[Gk]).max(axis=1, keepdims=True) + 1e-300
        assert np.all(np.abs(G - g[Gk]) <= 1e-10 * scale)
        assert np.allclose(err, g[ek], rtol=1e-10, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["stream_tiny.npz", "stream_tiny_smooth.npz"])
def test_gpu_stream_golden(fmx_mod, name):
    g = load(name)
    rec, key = (int(v) for v in g["window"])
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams(
        extraction=fmx_mod.KeypointExtractionParams(**json.loads(str(g["params"]))),
        disable_smoothing=bool(g["disable_smoothing"]), max_num_recent_scans=rec, max_num_keyscans=key))
    for k in range(len(g["scans"])):
        ctx.register_scan(g["scans"][k])
        assert np.abs(ctx.current_pose() - g["poses"][k]).max() < 1e-6
        st = ctx.last_stats()
        assert st["matched_planar"] == g["stats"][k][4] and st["matched_point"] == g["stats"][k][5]
