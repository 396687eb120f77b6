"""ctypes binding of liboracle.so (the CPU oracle).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by form_amd/.  Parity vs reference outputs: unpinned (see
form_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class ExtractParams(C.Structure):
    _fields_ = [
        ("neighbor_points", C.c_uint32), ("num_sectors", C.c_uint32),
        ("planar_threshold", C.c_double), ("planar_feats_per_sector", C.c_uint32),
        ("point_feats_per_sector", C.c_uint32), ("radius", C.c_double),
        ("min_points", C.c_uint32), ("min_norm_squared", C.c_double),
        ("max_norm_squared", C.c_double), ("num_columns", C.c_int32), ("num_rows", C.c_int32),
    ]


class Params(C.Structure):
    _fields_ = [
        ("extraction", ExtractParams), ("max_dist_matching", C.c_double),
        ("new_pose_threshold", C.c_double), ("max_num_rematches", C.c_uint32),
        ("planar_constraint_sigma", C.c_double), ("disable_smoothing", C.c_int32),
        ("max_num_keyscans", C.c_int64), ("max_steps_unused_keyscan", C.c_int64),
        ("max_num_recent_scans", C.c_uint32), ("keyscan_match_ratio", C.c_double),
        ("min_dist_map", C.c_double),
    ]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _LIB = C.CDLL(path)
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def extract_params(d: dict) -> ExtractParams:
    p = ExtractParams()
    for k, _ in ExtractParams._fields_:
        setattr(p, k, d[k])
    return p


def default_params(extract: dict | None = None) -> Params:
    p = Params()
    lib().orc_default_params(C.byref(p))
    if extract:
        p.extraction = extract_params(extract)
    return p


def extract(scan: np.ndarray, params: dict, nthreads: int = 0) -> dict:
    """FeatureExtractor::extract restated; returns indices, normals and masks."""
    scan = np.ascontiguousarray(scan, dtype=np.float32)
    R, Cc = params["num_rows"], params["num_columns"]
    n = scan.shape[0]
    cap = R * params["num_sectors"] * (params["planar_feats_per_sector"] + 1)
    sel = np.zeros(cap, np.uint32)
    ok = np.zeros(cap, np.uint8)
    nrm = np.zeros((cap, 3), np.float32)
    pidx = np.zeros(max(n, 1), np.uint32)
    pm = np.zeros(n, np.uint8)
    vm = np.zeros(n, np.uint8)
    curv = np.zeros(n, np.float32)
    nsel = C.c_uint32(0)
    npt = C.c_uint32(0)
    ep = extract_params(params)
    rc = lib().orc_extract(C.byref(ep), _p(scan), C.c_size_t(n), C.c_int(nthreads), _p(sel),
                           C.byref(nsel), _p(ok), _p(nrm), _p(pidx), C.byref(npt), _p(pm), _p(vm),
                           _p(curv))
    if rc != 0:
        raise RuntimeError(f"Provided scan does not match the expected size {R * Cc} != {n}")
    ns, nq = nsel.value, npt.value
    return dict(sel=sel[:ns].copy(), normal_ok=ok[:ns].astype(bool), normals=nrm[:ns].copy(),
                point_idx=pidx[:nq].copy(), planar_mask=pm.astype(bool), point_mask=vm.astype(bool),
                curvature=curv)


def features_from(scan: np.ndarray, ex: dict):
    """(planar (F,6) float32 xyz+nxyz, point (F,3) float32) as extract() would return."""
    s = ex["sel"][ex["normal_ok"]]
    planar = np.concatenate([scan[s, :3], ex["normals"][ex["normal_ok"]]], 1).astype(np.float32)
    point = scan[ex["point_idx"], :3].astype(np.float32)
    return np.ascontiguousarray(planar), np.ascontiguousarray(point)


class VoxelMap:
    def __init__(self, voxel_width: float, kind: int):
        L = lib()
        L.orc_map_new.restype = C.c_void_p
        self.kind = kind
        self.h = C.c_void_p(L.orc_map_new(C.c_double(voxel_width), C.c_int(kind)))

    def __del__(self):
        try:
            lib().orc_map_free(self.h)
        except Exception:
            pass

    def add_scan(self, scan_id: int, pose34: np.ndarray, feats: np.ndarray):
        feats = np.ascontiguousarray(feats, np.float32)
        pose = np.ascontiguousarray(pose34, np.float64).reshape(12)
        lib().orc_map_add_scan(self.h, C.c_uint64(scan_id), _p(pose), _p(feats),
                               C.c_uint32(feats.shape[0]))

    def num_voxels(self) -> int:
        lib().orc_map_num_voxels.restype = C.c_uint64
        return int(lib().orc_map_num_voxels(self.h))

    def match(self, queries: np.ndarray, pose_j34: np.ndarray, nthreads: int = 0) -> dict:
        q = np.ascontiguousarray(queries, np.float32)
        nq = q.shape[0]
        found = np.zeros(nq, np.uint8)
        scan = np.zeros(nq, np.uint64)
        d2 = np.zeros(nq, np.float64)
        pi = np.zeros((nq, 3), np.float64)
        ni = np.zeros((nq, 3), np.float64)
        pose = np.ascontiguousarray(pose_j34, np.float64).reshape(12)
        lib().orc_map_match(self.h, _p(q), C.c_uint32(nq), _p(pose), C.c_int(nthreads), _p(found),
                            _p(scan), _p(d2), _p(pi), _p(ni))
        return dict(found=found.astype(bool), scan=scan, d2=d2, pi=pi, ni=ni)


def linearize(np_, plane_pi, plane_ni, plane_pj, nt, point_pi, point_pj, poses_i, poses_j,
              sigma=0.1, single=False):
    np_ = np.ascontiguousarray(np_, np.uint32)
    nt = np.ascontiguousarray(nt, np.uint32)
    K = np_.shape[0]
    G = np.zeros((K, 28 if single else 91), np.float64)
    err = np.zeros(K, np.float64)
    a = [np.ascontiguousarray(x, np.float64) for x in (plane_pi, plane_ni, plane_pj, point_pi,
                                                        point_pj, poses_i, poses_j)]
    lib().orc_linearize(C.c_uint32(K), _p(np_), _p(a[0]), _p(a[1]), _p(a[2]), _p(nt), _p(a[3]),
                        _p(a[4]), _p(a[5]), _p(a[6]), C.c_double(sigma), C.c_int(int(single)),
                        _p(G), _p(err))
    return G, err


def factor_rows(plane_pi, plane_ni, plane_pj, point_pi, point_pj, pose_i, pose_j):
    a = [np.ascontiguousarray(x, np.float64).reshape(-1, 3) for x in (plane_pi, plane_ni, plane_pj,
                                                                       point_pi, point_pj)]
    np_, nt = a[0].shape[0], a[3].shape[0]
    rows = np_ + 3 * nt
    r = np.zeros(rows)
    J = np.zeros((rows, 12))
    pi_ = np.ascontiguousarray(pose_i, np.float64).reshape(12)
    pj_ = np.ascontiguousarray(pose_j, np.float64).reshape(12)
    lib().orc_factor_rows(C.c_uint32(np_), _p(a[0]), _p(a[1]), _p(a[2]), C.c_uint32(nt), _p(a[3]),
                          _p(a[4]), _p(pi_), _p(pj_), _p(r), _p(J))
    return r, J


def expmap(xi):
    out = np.zeros(12)
    lib().orc_pose_expmap(_p(np.ascontiguousarray(xi, np.float64)), _p(out))
    return out.reshape(3, 4)


def logmap(T):
    xi = np.zeros(6)
    lib().orc_pose_logmap(_p(np.ascontiguousarray(T, np.float64).reshape(12)), _p(xi))
    return xi


def compose(a, b):
    out = np.zeros(12)
    lib().orc_pose_compose(_p(np.ascontiguousarray(a, np.float64).reshape(12)),
                           _p(np.ascontiguousarray(b, np.float64).reshape(12)), _p(out))
    return out.reshape(3, 4)


class Estimator:
    """register_scan restatement (single-pose mode)."""

    def __init__(self, params: Params, nthreads: int = 0):
        lib().orc_estimator_new.restype = C.c_void_p
        self.h = C.c_void_p(lib().orc_estimator_new(C.byref(params), C.c_int(nthreads)))
        lib().orc_estimator_map.restype = C.c_uint32

    def __del__(self):
        try:
            lib().orc_estimator_free(self.h)
        except Exception:
            pass

    def register_scan(self, scan: np.ndarray):
        scan = np.ascontiguousarray(scan, np.float32)
        pose = np.zeros(12)
        stats = np.zeros(6, np.uint32)
        tms = np.zeros(4)
        rc = lib().orc_register_scan(self.h, _p(scan), C.c_size_t(scan.shape[0]), _p(pose),
                                     _p(stats), _p(tms))
        if rc != 0:
            raise RuntimeError("scan size mismatch")
        return pose.reshape(3, 4), stats, tms

    def map(self):
        """FORM::map() restated (bindings.cpp:96-119): {"planar": (xyz (M,3), normals
        (M,3), scans (M,)), "point": (xyz, None, scans)} in push_back order."""
        out = {}
        for kind, name in ((0, "planar"), (1, "point")):
            n = lib().orc_estimator_map(self.h, C.c_int(kind), None, None, None)
            xyz = np.zeros((n, 3))
            nrm = np.zeros((n, 3)) if kind == 0 else None
            sc = np.zeros(n, np.uint64)
            lib().orc_estimator_map(self.h, C.c_int(kind), _p(xyz), _p(nrm), _p(sc))
            out[name] = (xyz, nrm, sc)
        return out
