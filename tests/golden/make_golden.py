"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

  python tests/golden/make_golden.py

The reference ships no golden vectors and cannot be built here,
so these fixtures pin the oracle's own outputs on deterministic synthetic inputs:
a regression anchor for the oracle and a target for the GPU tests.  Every fixture is
data (inputs + expected outputs), no reference source.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_py as O  # noqa: E402
from form_amd import synth  # noqa: E402
from scenario import perturb, random_corr, stream_features  # noqa: E402


def main():
    world = synth.World()
    # 1. extraction on a 16x256 scan
    scan, T, geo = synth.make_scan("tiny", 3, world=world)
    p = synth.default_params(geo)
    ex = O.extract(scan.numpy(), p)
    np.savez_compressed(os.path.join(HERE, "extract_tiny.npz"), scan=scan.numpy(), params=json.dumps(p),
                        sel=ex["sel"], normal_ok=ex["normal_ok"], normals=ex["normals"],
                        point_idx=ex["point_idx"], planar_mask=ex["planar_mask"], point_mask=ex["point_mask"],
                        curvature=ex["curvature"])
    # 2. voxel map + match: 4 map scans, 1 query scan (features from the oracle)
    feats = stream_features(O, "tiny", 5, world)
    w = 0.8
    maps = [O.VoxelMap(w, 0), O.VoxelMap(w, 1)]
    for k in range(4):
        maps[0].add_scan(k, feats[k]["pose"], feats[k]["planar"])
        maps[1].add_scan(k, feats[k]["pose"], feats[k]["point"])
    q = feats[4]
    Tj = perturb(q["pose"], np.random.default_rng(4), 0.005, 0.03)
    mp = maps[0].match(q["planar"], Tj)
    mt = maps[1].match(q["point"], Tj)
    arrs = {}
    for k in range(4):
        arrs[f"map_planar_{k}"] = feats[k]["planar"]
        arrs[f"map_point_{k}"] = feats[k]["point"]
    np.savez_compressed(os.path.join(HERE, "match_tiny.npz"), poses=np.stack([feats[k]["pose"] for k in range(4)]),
                        q_planar=q["planar"], q_point=q["point"], pose_j=Tj, voxel_width=w,
                        pl_found=mp["found"], pl_scan=mp["scan"], pl_d2=mp["d2"], pl_pi=mp["pi"], pl_ni=mp["ni"],
                        pt_found=mt["found"], pt_scan=mt["scan"], pt_d2=mt["d2"], pt_pi=mt["pi"], **arrs)
    # 3. linearization of random pair-major correspondence sets
    rng = np.random.default_rng(99)
    np_, ppi, pni, ppj, nt, tpi, tpj, Pi, Pj = random_corr(rng, 6, max_rows=400)
    G, err = O.linearize(np_, ppi, pni, ppj, nt, tpi, tpj, Pi, Pj, 0.1, False)
    G1, err1 = O.linearize(np_, ppi, pni, ppj, nt, tpi, tpj, Pi, Pj, 0.1, True)
    np.savez_compressed(os.path.join(HERE, "linearize_small.npz"), n_plane=np_, plane_pi=ppi, plane_ni=pni,
                        plane_pj=ppj, n_point=nt, point_pi=tpi, point_pj=tpj, poses_i=Pi, poses_j=Pj, sigma=0.1,
                        G=G, err=err, G_single=G1, err_single=err1)
    # 4. register_scan on a 6-scan 16x256 stream (single-pose ablation mode) and on a
    #    16-scan stream in the default smoothing mode (marginalization from scan 11 on)
    #    (a small window — 4 recent scans, 3 keyscans — so keyscans get marginalized)
    for name, n, single, win in (("stream_tiny.npz", 6, 1, (10, 50)), ("stream_tiny_smooth.npz", 16, 0, (4, 3))):
        prm = O.default_params(p)
        prm.disable_smoothing = single
        prm.max_num_recent_scans, prm.max_num_keyscans = win
        est = O.Estimator(prm, 1)
        scans, poses, stats = [], [], []
        for k in range(n):
            s, _, _ = synth.make_scan("tiny", k, world=world)
            Tp, st, _ = est.register_scan(s.numpy())
            scans.append(s.numpy())
            poses.append(Tp)
            stats.append(st)
        np.savez_compressed(os.path.join(HERE, name), scans=np.stack(scans), poses=np.stack(poses),
                            stats=np.stack(stats), params=json.dumps(p), disable_smoothing=single,
                            window=np.array(win))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
