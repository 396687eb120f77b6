"""ctypes host layer over libfmx.so (include/fmx/fmx.h).

Mirrors the reference's Python-facing surface for this path:
  * ``KeypointExtractionParams`` / ``extract_keypoints`` — form._core
    (python/bindings.cpp:194-240): returns (planar_points, normals, point_points).
  * ``Estimator`` — form::Estimator (form/form.hpp:40-84): ``register_scan(scan)``
    returns the (planar, point) features, ``current_lidar_estimate()`` the pose.
  * ``Context`` — the stage-level seams (extract / map_build / match /
    linearize / error / insert) used by the parity tests.

There is no CPU fallback: if libfmx.so is missing or no HIP device is visible the
import or the constructor raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, fields

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FMX_LIB", os.path.join(_HERE, "libfmx.so"))  # FMX_LIB: A/B of two builds
_LIB = None

FMX_OK = 0
_STATUS = {1: "FMX_E_INVAL", 2: "FMX_E_SIZE", 3: "FMX_E_OOM", 4: "FMX_E_HIP", 5: "FMX_E_STATE",
           6: "FMX_E_RANGE", 7: "FMX_E_RCCL"}


class FmxError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{_STATUS.get(status, status)}: {msg}")
        self.status = status


class _ExtractParams(C.Structure):
    _fields_ = [
        ("neighbor_points", C.c_uint32), ("num_sectors", C.c_uint32),
        ("planar_threshold", C.c_double), ("planar_feats_per_sector", C.c_uint32),
        ("point_feats_per_sector", C.c_uint32), ("radius", C.c_double),
        ("min_points", C.c_uint32), ("min_norm_squared", C.c_double),
        ("max_norm_squared", C.c_double), ("num_columns", C.c_int32), ("num_rows", C.c_int32),
    ]


class _Params(C.Structure):
    _fields_ = [
        ("extraction", _ExtractParams), ("max_dist_matching", C.c_double),
        ("new_pose_threshold", C.c_double), ("max_num_rematches", C.c_uint32),
        ("planar_constraint_sigma", C.c_double), ("disable_smoothing", C.c_int32),
        ("max_num_keyscans", C.c_int64), ("max_steps_unused_keyscan", C.c_int64),
        ("max_num_recent_scans", C.c_uint32), ("keyscan_match_ratio", C.c_double),
        ("min_dist_map", C.c_double), ("keypoint_pool_capacity", C.c_uint64),
        ("max_pairs", C.c_uint32), ("voxel_subdivision", C.c_uint32),
    ]


class _Counts(C.Structure):
    _fields_ = [("planar", C.c_uint32), ("point", C.c_uint32), ("planar_selected", C.c_uint32)]


def lib():
    """Load libfmx.so (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C form_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        L.fmx_last_error.restype = C.c_char_p
        L.fmx_profile_name.restype = C.c_char_p
        _LIB = L
    return _LIB


EXPORTED = [
    "fmx_abi_version", "fmx_default_params", "fmx_create", "fmx_destroy", "fmx_last_error",
    "fmx_extract", "fmx_extract_download", "fmx_set_queries", "fmx_set_queries_device", "fmx_keypoints_add",
    "fmx_keypoints_add_device",
    "fmx_keypoints_remove", "fmx_map_build", "fmx_match", "fmx_match_download", "fmx_map_insert",
    "fmx_corr_set", "fmx_linearize", "fmx_error", "fmx_linearize_matched", "fmx_register_scan", "fmx_next_scan",
    "fmx_current_pose",
    "fmx_last_stats", "fmx_match_work", "fmx_profile_enable", "fmx_profile_reset", "fmx_profile_count",
    "fmx_profile_name", "fmx_profile_read", "fmx_sync", "fmx_comm_unique_id", "fmx_comm_init",
    "fmx_map_download", "fmx_register_points", "fmx_scan_buffer", "fmx_match_cert", "fmx_profile_match_work",
    "fmx_corr_generation", "fmx_moments", "fmx_moments_contract",
]


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _ready(*tensors):
    """Device tensors handed to a context's stream: wait for the torch stream that
    produced them (fmx copies them on its own stream, unordered with torch's)."""
    import torch
    for t in tensors:
        if t is not None and t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()
            return


@dataclass
class KeypointExtractionParams:
    """form::FeatureExtractor::Params (extraction.hpp:59-88); same names as the
    nanobind class KeypointExtractionParams (bindings.cpp:194-211)."""
    neighbor_points: int = 5
    num_sectors: int = 6
    planar_threshold: float = 1.0
    planar_feats_per_sector: int = 50
    point_feats_per_sector: int = 3
    radius: float = 1.0
    min_points: int = 5
    min_norm_squared: float = 1.0
    max_norm_squared: float = 100.0 * 100.0
    num_columns: int = 1024
    num_rows: int = 64

    def as_dict(self):
        return {f.name: getattr(self, f.name) for f in fields(self)}


@dataclass
class EstimatorParams:
    """form::Estimator::Params (form.hpp:42-56), flattened like the evalio YAML keys
    (bindings.cpp:66-88)."""
    extraction: KeypointExtractionParams = None
    max_dist_matching: float = 0.8
    new_pose_threshold: float = 1e-4
    max_num_rematches: int = 30
    planar_constraint_sigma: float = 0.1
    disable_smoothing: bool = False  # constraints.hpp:56 (True: single-pose ablation)
    max_num_keyscans: int = 50
    max_steps_unused_keyscan: int = 10
    max_num_recent_scans: int = 10
    keyscan_match_ratio: float = 0.1
    min_dist_map: float = 0.1
    keypoint_pool_capacity: int = 4 << 20
    max_pairs: int = 1024
    voxel_subdivision: int = 1

    def __post_init__(self):
        if self.extraction is None:
            self.extraction = KeypointExtractionParams()

    def to_c(self) -> _Params:
        p = _Params()
        lib().fmx_default_params(C.byref(p))
        for k, v in self.extraction.as_dict().items():
            setattr(p.extraction, k, v)
        for f in fields(self):
            if f.name != "extraction":
                setattr(p, f.name, int(getattr(self, f.name)) if isinstance(getattr(self, f.name), bool)
                        else getattr(self, f.name))
        return p


class Context:
    """One fmx context (one HIP device + stream).  Thin, stage-level API."""

    def __init__(self, params: EstimatorParams | None = None, device: int = 0):
        self.params = params or EstimatorParams()
        self._L = lib()
        h = C.c_void_p()
        st = self._L.fmx_create(C.byref(self.params.to_c()), C.c_int(device), C.byref(h))
        if st != FMX_OK:
            raise FmxError(st, "fmx_create failed (is a HIP device visible?)")
        self.h = h
        self.K = 0
        self.n_planar = 0
        self.n_point = 0

    def close(self):
        if getattr(self, "h", None):
            self._L.fmx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st: int):
        if st != FMX_OK:
            raise FmxError(st, self._L.fmx_last_error(self.h).decode())

    # ---------------------------------------------------------------- stage 1
    def extract(self, scan, scan_idx: int = 0):
        """scan: (N, 4) float32 numpy array (host) or torch tensor (host or device)."""
        on_dev, ptr, n, keep = _scan_ptr(scan)
        c = _Counts()
        self._chk(self._L.fmx_extract(self.h, ptr, C.c_size_t(n), C.c_uint64(scan_idx),
                                      C.c_int(on_dev), C.byref(c)))
        del keep
        self.n_planar, self.n_point = c.planar, c.point
        return c.planar, c.point, c.planar_selected

    def extract_download(self, with_mask: bool = False):
        npl, npt = self.n_planar, self.n_point
        planar = np.zeros((npl, 6), np.float32)
        pidx = np.zeros(npl, np.uint32)
        point = np.zeros((npt, 3), np.float32)
        tidx = np.zeros(npt, np.uint32)
        e = self.params.extraction
        mask = np.zeros(e.num_rows * e.num_columns, np.uint8) if with_mask else None
        self._chk(self._L.fmx_extract_download(self.h, _p(planar), _p(pidx), _p(point), _p(tidx), _p(mask)))
        out = dict(planar=planar, planar_index=pidx, point=point, point_index=tidx)
        if with_mask:
            out["planar_mask"] = mask.astype(bool)
        return out

    def set_queries(self, planar: np.ndarray, point: np.ndarray, scan_idx: int = 0):
        planar = np.ascontiguousarray(planar, np.float32).reshape(-1, 6)
        point = np.ascontiguousarray(point, np.float32).reshape(-1, 3)
        self._chk(self._L.fmx_set_queries(self.h, C.c_uint64(scan_idx), _p(planar), C.c_uint32(len(planar)),
                                          _p(point), C.c_uint32(len(point))))
        self.n_planar, self.n_point = len(planar), len(point)

    def set_queries_device(self, planar_pos4, planar_nrm4, point_pos4=None, scan_idx: int = 0):
        """Device-resident queries: (N,4) float32 CUDA tensors."""
        npt = 0 if point_pos4 is None else point_pos4.shape[0]
        pp = C.c_void_p(point_pos4.data_ptr()) if npt else None
        _ready(planar_pos4, planar_nrm4, point_pos4)
        self._chk(self._L.fmx_set_queries_device(self.h, C.c_uint64(scan_idx), C.c_void_p(planar_pos4.data_ptr()),
                                                 C.c_void_p(planar_nrm4.data_ptr()), C.c_uint32(planar_pos4.shape[0]),
                                                 pp, C.c_uint32(npt)))
        self.n_planar, self.n_point = planar_pos4.shape[0], npt

    # ---------------------------------------------------------------- stage 2
    def keypoints_add_device(self, scan_idx: int, planar_pos4, planar_nrm4, point_pos4=None):
        npt = 0 if point_pos4 is None else point_pos4.shape[0]
        pp = C.c_void_p(point_pos4.data_ptr()) if npt else None
        _ready(planar_pos4, planar_nrm4, point_pos4)
        self._chk(self._L.fmx_keypoints_add_device(self.h, C.c_uint64(scan_idx), C.c_void_p(planar_pos4.data_ptr()),
                                                   C.c_void_p(planar_nrm4.data_ptr()), C.c_uint32(planar_pos4.shape[0]),
                                                   pp, C.c_uint32(npt)))

    def keypoints_add(self, scan_idx: int, planar: np.ndarray, point: np.ndarray):
        planar = np.ascontiguousarray(planar, np.float32).reshape(-1, 6)
        point = np.ascontiguousarray(point, np.float32).reshape(-1, 3)
        self._chk(self._L.fmx_keypoints_add(self.h, C.c_uint64(scan_idx), _p(planar), C.c_uint32(len(planar)),
                                            _p(point), C.c_uint32(len(point))))

    def keypoints_remove(self, scan_idx: int):
        self._chk(self._L.fmx_keypoints_remove(self.h, C.c_uint64(scan_idx)))

    def map_build(self, scans, poses34, voxel_width: float):
        scans = np.ascontiguousarray(scans, np.uint64)
        poses = np.ascontiguousarray(poses34, np.float64).reshape(-1, 12)
        self._chk(self._L.fmx_map_build(self.h, _p(scans), _p(poses), C.c_uint32(len(scans)),
                                        C.c_double(voxel_width)))
        self.K = len(scans)

    def match(self, pose_j34, max_dist: float, counts: bool = True):
        """fmx_match; counts=False returns None without waiting for the kernel."""
        pose = np.ascontiguousarray(pose_j34, np.float64).reshape(12)
        if not counts:
            self._chk(self._L.fmx_match(self.h, _p(pose), C.c_double(max_dist), None, None))
            return None
        cpl = np.zeros(max(self.K, 1), np.uint32)
        cpt = np.zeros(max(self.K, 1), np.uint32)
        self._chk(self._L.fmx_match(self.h, _p(pose), C.c_double(max_dist), _p(cpl), _p(cpt)))
        return cpl[:self.K], cpt[:self.K]

    def match_download(self):
        nq = self.n_planar + self.n_point
        pair = np.zeros(nq, np.int32)
        d2 = np.zeros(nq, np.float64)
        pi = np.zeros((nq, 3), np.float64)
        ni = np.zeros((self.n_planar, 3), np.float64)
        self._chk(self._L.fmx_match_download(self.h, _p(pair), _p(d2), _p(pi), _p(ni)))
        return dict(pair=pair, d2=d2, pi=pi, ni=ni)

    def map_insert(self, min_dist_map: float | None = None):
        n = np.zeros(2, np.uint32)
        md = self.params.min_dist_map if min_dist_map is None else min_dist_map
        self._chk(self._L.fmx_map_insert(self.h, C.c_double(md), _p(n)))
        return int(n[0]), int(n[1])

    # ---------------------------------------------------------------- stage 3
    def corr_set(self, n_plane, plane_pi, plane_ni, plane_pj, n_point, point_pi, point_pj):
        n_plane = np.ascontiguousarray(n_plane, np.uint32)
        n_point = np.ascontiguousarray(n_point, np.uint32)
        arrs = [np.ascontiguousarray(a, np.float64).reshape(-1, 3) for a in
                (plane_pi, plane_ni, plane_pj, point_pi, point_pj)]
        self._chk(self._L.fmx_corr_set(self.h, C.c_uint32(len(n_plane)), _p(n_plane), _p(arrs[0]), _p(arrs[1]),
                                       _p(arrs[2]), _p(n_point), _p(arrs[3]), _p(arrs[4])))
        self.K = len(n_plane)

    def linearize(self, poses_i, poses_j, sigma: float = 0.1, single: bool = False):
        pi_ = np.ascontiguousarray(poses_i, np.float64).reshape(-1, 12)
        pj_ = np.ascontiguousarray(poses_j, np.float64).reshape(-1, 12)
        G = np.zeros((max(self.K, 1), 28 if single else 91))
        err = np.zeros(max(self.K, 1))
        self._chk(self._L.fmx_linearize(self.h, _p(pi_), _p(pj_), C.c_double(sigma), C.c_int(int(single)),
                                        _p(G), _p(err)))
        return G[:self.K], err[:self.K]

    def error(self, poses_i, poses_j, sigma: float = 0.1):
        pi_ = np.ascontiguousarray(poses_i, np.float64).reshape(-1, 12)
        pj_ = np.ascontiguousarray(poses_j, np.float64).reshape(-1, 12)
        err = np.zeros(max(self.K, 1))
        self._chk(self._L.fmx_error(self.h, _p(pi_), _p(pj_), C.c_double(sigma), _p(err)))
        return err[:self.K]

    def linearize_matched(self, pose_j34, sigma: float = 0.1):
        """Single-pose 7x7 system (28 packed) summed over every accepted match of the
        last match at pose_j, and its error."""
        pose = np.ascontiguousarray(pose_j34, np.float64).reshape(12)
        out = np.zeros(29)
        self._chk(self._L.fmx_linearize_matched(self.h, _p(pose), C.c_double(sigma), _p(out)))
        return out[:28].copy(), float(out[28])

    def register_points(self, pose_init34, max_dist: float, sigma: float = 0.1, max_iters: int = 30,
                        threshold: float = 1e-4):
        """fmx_register_points: Gauss-Newton ICP of the query set against the built map
        (match + summed 7x7 + solve per iteration, all in libfmx).  Returns (pose 3x4,
        iterations)."""
        T0 = np.ascontiguousarray(pose_init34, np.float64).reshape(12)
        T = np.zeros(12)
        it = C.c_uint32(0)
        self._chk(self._L.fmx_register_points(self.h, _p(T0), C.c_double(max_dist), C.c_double(sigma),
                                              C.c_uint32(max_iters), C.c_double(threshold), _p(T), C.byref(it)))
        return T.reshape(3, 4), int(it.value)

    # ---------------------------------------------------------------- multi-GPU
    def comm_init(self, unique_id: bytes, nranks: int, rank: int):
        """Attach an RCCL communicator (see comm_unique_id): linearization sums are then
        all-reduced over the ranks on the device, on this context's stream."""
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._chk(self._L.fmx_comm_init(self.h, buf, C.c_int(nranks), C.c_int(rank)))

    # ---------------------------------------------------------------- estimator
    def register_scan(self, scan):
        on_dev, ptr, n, keep = _scan_ptr(scan)
        c = _Counts()
        self._chk(self._L.fmx_register_scan(self.h, ptr, C.c_size_t(n), C.c_int(on_dev), C.byref(c)))
        del keep
        self.n_planar, self.n_point = c.planar, c.point
        return c.planar, c.point

    def scan_buffer(self, n: int | None = None) -> np.ndarray:
        """fmx_scan_buffer: a context-owned page-locked (n, 4) float32 buffer (default:
        rows * cols points) to assemble a scan in; registered or announced as a host scan
        it is DMA'd without a staging copy.  Buffers rotate over three: the array
        returned here aliases the one returned by the third next call."""
        e = self.params.extraction
        n = n or e.num_rows * e.num_columns
        p = C.c_void_p()
        self._chk(self._L.fmx_scan_buffer(self.h, C.c_size_t(n), C.byref(p)))
        a = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), shape=(n, 4))
        # the memory belongs to the context: the array keeps the Context alive (a view
        # whose base holds it).  It is invalid after close() and after a later
        # scan_buffer call that asks for more points than this buffer holds.
        return np.asarray(_CtxBuffer(a, self))

    def next_scan(self, scan):
        """fmx_next_scan: announce the scan that follows the one the next register_scan
        receives — a contiguous (N, 4) float32 CUDA tensor, or a host array / tensor (its
        staging copy then starts at once, in the background) — left unchanged until its
        own register_scan; that call extracts it while registering.  None withdraws."""
        if scan is None:
            self._chk(self._L.fmx_next_scan(self.h, None, C.c_size_t(0), C.c_int(0)))
            return
        on_dev, ptr, n, keep = _scan_ptr(scan)
        # a converted copy would not be the memory later registered
        same = (keep is scan) if not isinstance(scan, np.ndarray) else (
            keep.__array_interface__["data"][0] == scan.__array_interface__["data"][0])
        if not same:
            raise ValueError("next_scan needs a contiguous (N, 4) float32 array or tensor")
        self._chk(self._L.fmx_next_scan(self.h, ptr, C.c_size_t(n), C.c_int(on_dev)))
        # the tensor must outlive the extraction queued for it
        self._pf_keep = (getattr(self, "_pf_keep", (None, None))[1], scan)

    def current_pose(self) -> np.ndarray:
        T = np.zeros(12)
        self._chk(self._L.fmx_current_pose(self.h, _p(T)))
        return T.reshape(3, 4)

    def map_download(self, voxel_width: float):
        """fmx_map_download: FORM::map()'s to_voxel_map of both feature types at the
        current estimates (bindings.cpp:96-119), voxel by voxel.  Returns {"planar":
        (xyz (M,3), normals (M,3), scans (M,)), "point": (xyz, None, scans)}."""
        npl, npt = C.c_uint32(0), C.c_uint32(0)
        self._chk(self._L.fmx_map_download(self.h, C.c_double(voxel_width), None, None, C.byref(npl), None, None,
                                           C.byref(npt)))
        pl = np.zeros((npl.value, 6))
        spl = np.zeros(npl.value, np.uint64)
        pt = np.zeros((npt.value, 3))
        spt = np.zeros(npt.value, np.uint64)
        self._chk(self._L.fmx_map_download(self.h, C.c_double(voxel_width), _p(pl), _p(spl), C.byref(npl), _p(pt),
                                           _p(spt), C.byref(npt)))
        return {"planar": (pl[:npl.value, :3].copy(), pl[:npl.value, 3:].copy(), spl[:npl.value]),
                "point": (pt[:npt.value], None, spt[:npt.value])}

    def last_stats(self) -> dict:
        keys = ["icp_iters", "lm_iters", "matched_planar", "matched_point", "map_planar", "map_point",
                "linearizations", "map_scans", "host_waits", "spec_matches", "spec_hits", "spec_map",
                "pipelined", "window_poses"]
        s = np.zeros(len(keys), np.uint64)
        self._chk(self._L.fmx_last_stats(self.h, _p(s), C.c_int(len(keys))))
        return {k: int(v) for k, v in zip(keys, s)}

    def match_work(self) -> dict:
        w = np.zeros(3)
        self._chk(self._L.fmx_match_work(self.h, _p(w)))
        return dict(queries=float(w[0]), probes=float(w[1]), candidates=float(w[2]))

    # ---------------------------------------------------------------- profiling
    def moments(self, ref_i, ref_j) -> np.ndarray:
        """fmx_moments: the (K, 272) pair moments of the context's correspondences at
        reference poses ref_i[k], ref_j[k] (K x 3 x 4); evaluate them at any poses with
        moments_contract (no device round trip)."""
        ri = np.ascontiguousarray(ref_i, np.float64).reshape(-1, 12)
        rj = np.ascontiguousarray(ref_j, np.float64).reshape(-1, 12)
        out = np.zeros((max(self.K, 1), 272))
        self._chk(self._L.fmx_moments(self.h, _p(ri), _p(rj), _p(out)))
        return out[:self.K]

    def match_cert(self, per_query: bool = False):
        """fmx_match_cert: the warm certificate of the last match — (certified, warm)
        query counts, and with per_query a uint8 array (planar then point queries, 1 =
        settled by the certificate without a search)."""
        cnt = np.zeros(2, np.uint64)
        flags = np.zeros(self.n_planar + self.n_point if per_query else 0, np.uint8)
        self._chk(self._L.fmx_match_cert(self.h, _p(cnt), _p(flags) if per_query else None))
        out = dict(certified=int(cnt[0]), warm=int(cnt[1]))
        if per_query:
            out["flags"] = flags
        return out

    def profile_match_work(self) -> dict:
        """fmx_profile_match_work: the profiled match launches' work since the last
        reset, split into cold (first match on a map / query set) and warm launches."""
        w = np.zeros(12)
        self._chk(self._L.fmx_profile_match_work(self.h, _p(w)))
        return {k: dict(launches=w[6 * i], queries=w[6 * i + 1], probes=w[6 * i + 2], candidates=w[6 * i + 3],
                        certified=w[6 * i + 4], warm=w[6 * i + 5])
                for i, k in enumerate(("cold", "warm"))}

    def corr_generation(self) -> int:
        g = C.c_uint64()
        self._chk(self._L.fmx_corr_generation(self.h, C.byref(g)))
        return int(g.value)

    def profile(self, on: bool = True):
        self._chk(self._L.fmx_profile_enable(self.h, C.c_int(int(on))))

    def profile_reset(self):
        self._chk(self._L.fmx_profile_reset(self.h))

    def profile_read(self) -> dict:
        n = self._L.fmx_profile_count()
        ms = np.zeros(n)
        la = np.zeros(n, np.uint64)
        by = np.zeros(n)
        self._chk(self._L.fmx_profile_read(self.h, _p(ms), _p(la), _p(by), C.c_int(n)))
        return {self._L.fmx_profile_name(k).decode(): dict(ms=float(ms[k]), launches=int(la[k]), bytes=float(by[k]))
                for k in range(n)}

    def sync(self):
        self._chk(self._L.fmx_sync(self.h))


class _CtxBuffer:
    """Buffer protocol over a context-owned pinned array that also holds the context."""

    def __init__(self, arr, ctx):
        self._arr = arr
        self._ctx = ctx
        self.__array_interface__ = arr.__array_interface__


def _scan_ptr(scan):
    """(on_device, pointer, n_points, keepalive) for a numpy array or torch tensor."""
    try:
        import torch
        if isinstance(scan, torch.Tensor):
            if scan.dtype != torch.float32 or scan.dim() != 2 or scan.shape[1] != 4:
                raise ValueError("scan tensor must be (N, 4) float32")
            t = scan.contiguous()
            return (1 if t.is_cuda else 0), C.c_void_p(t.data_ptr()), t.shape[0], t
    except ImportError:
        pass
    a = np.ascontiguousarray(scan, np.float32)
    if a.ndim != 2 or a.shape[1] != 4:
        raise ValueError("scan must be (N, 4) float32 (PointXYZf layout)")
    return 0, _p(a), a.shape[0], a


def moments_contract(mom, ref_i, ref_j, poses_i, poses_j, sigma: float):
    """fmx_moments_contract (host only): packed 13 x 13 G (K, 91) and errors (K,) of K
    pairs at poses (poses_i[k], poses_j[k]) from their moments taken at (ref_i, ref_j)."""
    m = np.ascontiguousarray(mom, np.float64).reshape(-1, 272)
    K = m.shape[0]
    a = [np.ascontiguousarray(x, np.float64).reshape(K, 12) for x in (ref_i, ref_j, poses_i, poses_j)]
    G = np.zeros((max(K, 1), 91))
    err = np.zeros(max(K, 1))
    st = lib().fmx_moments_contract(C.c_uint32(K), _p(m), _p(a[0]), _p(a[1]), _p(a[2]), _p(a[3]),
                                    C.c_double(sigma), _p(G), _p(err))
    if st != FMX_OK:
        raise FmxError(st, "fmx_moments_contract failed")
    return G[:K], err[:K]


def comm_unique_id() -> bytes:
    """fmx_comm_unique_id: the 128-byte RCCL id one rank creates and shares."""
    buf = (C.c_uint8 * 128)()
    st = lib().fmx_comm_unique_id(buf)
    if st != FMX_OK:
        raise FmxError(st, "fmx_comm_unique_id failed (RCCL missing?)")
    return bytes(buf)


class Estimator:
    """form::Estimator (form/form.hpp:40-84) backed by the MI355X path."""

    def __init__(self, params: EstimatorParams | None = None, device: int = 0):
        self.ctx = Context(params, device)

    def register_scan(self, scan):
        """Returns (planar (F,6) xyz+normal, point (F,3)) like register_scan's tuple."""
        self.ctx.register_scan(scan)
        d = self.ctx.extract_download()
        return d["planar"], d["point"]

    def current_lidar_estimate(self) -> np.ndarray:
        return self.ctx.current_pose()


def extract_keypoints(points, params: KeypointExtractionParams, lidar_params=None):
    """form._core.extract_keypoints (bindings.cpp:214-240): (planar_points, normals,
    point_points).  lidar_params is accepted and ignored, as in the reference."""
    pts = np.asarray(points, np.float64).reshape(-1, 3)
    scan = np.zeros((len(pts), 4), np.float32)
    scan[:, :3] = pts.astype(np.float32)
    ctx = Context(EstimatorParams(extraction=params))
    try:
        ctx.extract(scan, 0)
        d = ctx.extract_download()
    finally:
        ctx.close()
    planar = d["planar"].astype(np.float64)
    return planar[:, :3].copy(), planar[:, 3:].copy(), d["point"].astype(np.float64)


# ---------------------------------------------------------------------------- evalio
# The evalio pipeline surface of form._core.FORM (python/bindings.cpp:48-180), backed by
# fmx.  evalio itself is not needed: lidar parameters, measurements and poses are
# duck-typed (attributes / numpy arrays), and results are numpy arrays.

# EVALIO_SETUP_PARAMS (bindings.cpp:66-88): YAML key -> (type, default, where it lands).
# Note the reference's key `max_dist_map` sets KeypointMapParams::min_dist_map (:85),
# and `num_threads` sizes the reference's TBB pool (no role on the GPU path).
PIPELINE_PARAMS = {
    "neighbor_points": (int, 5, "extraction.neighbor_points"),
    "num_sectors": (int, 6, "extraction.num_sectors"),
    "planar_threshold": (float, 1.0, "extraction.planar_threshold"),
    "planar_feats_per_sector": (int, 50, "extraction.planar_feats_per_sector"),
    "point_feats_per_sector": (int, 3, "extraction.point_feats_per_sector"),
    "radius": (float, 1.0, "extraction.radius"),
    "min_points": (int, 5, "extraction.min_points"),
    "max_dist_matching": (float, 0.8, "max_dist_matching"),
    "new_pose_threshold": (float, 1e-4, "new_pose_threshold"),
    "max_num_rematches": (int, 30, "max_num_rematches"),
    "disable_smoothing": (bool, False, "disable_smoothing"),
    "max_num_keyscans": (int, 50, "max_num_keyscans"),
    "max_num_recent_scans": (int, 10, "max_num_recent_scans"),
    "max_steps_unused_keyscan": (int, 10, "max_steps_unused_keyscan"),
    "keyscan_match_ratio": (float, 0.1, "keyscan_match_ratio"),
    "max_dist_map": (float, 0.1, "min_dist_map"),
    "num_threads": (int, 0, None),
}
# keys of an evalio config's pipeline entry that are not pipeline parameters
CONFIG_KEYS = ("pipeline", "name")


def _pose44(T) -> np.ndarray:
    T = np.asarray(T, np.float64)
    if T.shape == (4, 4):
        return T.copy()
    out = np.eye(4)
    out[:3, :] = T.reshape(3, 4)
    return out


def _points_xyz(mm) -> np.ndarray:
    """A LidarMeasurement's points as (N, 3): an (N, >=3) array, a measurement with a
    `points` attribute, or a sequence of objects with x, y, z (evalio.Point)."""
    pts = getattr(mm, "points", mm)
    try:
        a = np.asarray(pts, np.float64)
        if a.ndim == 2 and a.shape[1] >= 3:
            return a[:, :3]
    except (TypeError, ValueError):
        pass
    return np.array([[p.x, p.y, p.z] for p in pts], np.float64).reshape(-1, 3)


class FORM:
    """form._core.FORM (bindings.cpp:48-180) on the MI355X path.

    Same call sequence as evalio drives the reference: ``set_params`` (YAML keys),
    ``set_lidar_params``, ``set_imu_T_lidar``, ``initialize``, then ``add_lidar`` per
    scan, ``pose()`` and ``map()``.  ``add_lidar`` returns {"planar", "point"} as
    (F, 4) arrays of (x, y, z, scan) in the scan's frame — the reference's evalio
    Points carry the scan index in `col` as a uint16 (bindings.cpp:31-41, so it wraps
    modulo 65536); ``map()`` the same in the
    world frame, voxel by voxel (bindings.cpp:96-119)."""

    def __init__(self, device: int = 0):
        self.params = EstimatorParams()
        self.num_threads = 0
        self.device = device
        self.lidar_T_imu = np.eye(4)
        self._est = None
        self._scan = -1
        self._pose = np.eye(4)

    @staticmethod
    def name() -> str:
        return "form"

    @staticmethod
    def url() -> str:
        return "https://github.com/rpl-cmu/form"

    @staticmethod
    def default_params() -> dict:
        return {k: d for k, (_, d, _) in PIPELINE_PARAMS.items()}

    def set_params(self, params: dict) -> dict:
        """Apply YAML parameter overrides (EVALIO_SETUP_PARAMS keys, bindings.cpp:66-88);
        an evalio config entry's own keys (pipeline, name) are skipped.  Unknown keys
        raise KeyError.  Returns the full parameter dict now in effect."""
        for k, v in params.items():
            if k in CONFIG_KEYS:
                continue
            if k not in PIPELINE_PARAMS:
                raise KeyError(f"unknown FORM parameter {k!r}")
            typ, _, dest = PIPELINE_PARAMS[k]
            v = typ(v)
            if dest is None:
                self.num_threads = v
            elif dest.startswith("extraction."):
                setattr(self.params.extraction, dest.split(".", 1)[1], v)
            else:
                setattr(self.params, dest, v)
        return self.get_params()

    def get_params(self) -> dict:
        out = {}
        for k, (_, _, dest) in PIPELINE_PARAMS.items():
            if dest is None:
                out[k] = self.num_threads
            elif dest.startswith("extraction."):
                out[k] = getattr(self.params.extraction, dest.split(".", 1)[1])
            else:
                out[k] = getattr(self.params, dest)
        return out

    def set_imu_params(self, params) -> None:  # bindings.cpp:123 (unused)
        pass

    def set_lidar_params(self, params) -> None:
        """bindings.cpp:126-132: range limits (squared) and the organized geometry."""
        e = self.params.extraction
        e.min_norm_squared = float(params.min_range) * float(params.min_range)
        e.max_norm_squared = float(params.max_range) * float(params.max_range)
        e.num_columns = int(params.num_columns)
        e.num_rows = int(params.num_rows)

    def set_imu_T_lidar(self, T) -> None:
        """bindings.cpp:135-137: lidar_T_imu = (imu_T_lidar)^-1."""
        self.lidar_T_imu = np.linalg.inv(_pose44(T))

    def initialize(self) -> None:
        """bindings.cpp:141: a fresh estimator with the current parameters."""
        if self._est is not None:
            self._est.close()
        self._est = Context(self.params, self.device)
        self._scan = -1
        self._pose = np.eye(4)

    def add_imu(self, mm) -> None:  # bindings.cpp:144 (unused)
        pass

    def add_lidar(self, mm) -> dict:
        """bindings.cpp:147-179: register the scan, update the pose
        (current_lidar_estimate * lidar_T_imu) and return its features."""
        if self._est is None:
            raise RuntimeError("FORM.add_lidar before initialize()")
        xyz = _points_xyz(mm)
        # point_to_form: PointXYZf(x, y, z) (bindings.cpp:43-45), assembled straight into
        # a pinned fmx_scan_buffer: the registration then DMAs it with no staging copy
        scan = self._est.scan_buffer(len(xyz))
        scan[:, :3] = xyz
        scan[:, 3] = 0.0
        self._est.register_scan(scan)
        self._scan += 1
        self._pose = _pose44(self._est.current_pose()) @ self.lidar_T_imu
        d = self._est.extract_download()
        # point_to_evalio stores the scan id as static_cast<uint16_t>(scan) in the
        # point's col (bindings.cpp:31-41): it wraps past 65535 scans
        sid = self._scan % 65536
        planar = np.zeros((len(d["planar"]), 4))
        planar[:, :3] = d["planar"][:, :3]
        planar[:, 3] = sid
        point = np.zeros((len(d["point"]), 4))
        point[:, :3] = d["point"]
        point[:, 3] = sid
        return {"planar": planar, "point": point}

    def pose(self) -> np.ndarray:
        """bindings.cpp:93: the latest pose (4 x 4)."""
        return self._pose.copy()

    def map(self) -> dict:
        """bindings.cpp:96-119: the window's keypoints in the world frame, to_voxel_map
        at voxel width min_dist_map, as (M, 4) arrays of (x, y, z, scan)."""
        if self._est is None or self._scan < 0:
            return {"planar": np.zeros((0, 4)), "point": np.zeros((0, 4))}
        m = self._est.map_download(self.params.min_dist_map)
        out = {}
        for name, (xyz, _, sc) in m.items():
            a = np.zeros((len(xyz), 4))
            a[:, :3] = xyz
            a[:, 3] = sc % 65536  # uint16 col, as add_lidar (map_download keeps the raw id)
            out[name] = a
        return out
