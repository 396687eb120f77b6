"""The C-ABI library loads and exports every entry point include/fmx/fmx.h declares;
without a HIP device fmx_create fails with a status (no crash, no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "fmx", "fmx.h")).read()
    return sorted(set(re.findall(r"\b(fmx_[a-z_]+)\s*\(", hdr)))


def test_header_symbols_exported():
    from form_amd import fmx
    L = fmx.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(fmx.EXPORTED) == syms


def test_abi_version_and_defaults():
    from form_amd import fmx
    L = fmx.lib()
    assert L.fmx_abi_version() == 1
    p = fmx._Params()
    L.fmx_default_params(C.byref(p))
    # FORM defaults (extraction.hpp:59-88, matcher.hpp:32-41, constraints.hpp:60, map.hpp:97-100)
    assert p.extraction.neighbor_points == 5 and p.extraction.num_sectors == 6
    assert p.extraction.planar_feats_per_sector == 50 and p.extraction.point_feats_per_sector == 3
    assert p.max_dist_matching == 0.8 and p.max_num_rematches == 30 and p.new_pose_threshold == 1e-4
    assert p.planar_constraint_sigma == 0.1 and p.min_dist_map == 0.1
    assert p.max_num_recent_scans == 10 and p.max_num_keyscans == 50


def test_struct_layout_matches_oracle():
    import oracle_py
    from form_amd import fmx
    assert C.sizeof(fmx._ExtractParams) == C.sizeof(oracle_py.ExtractParams)
    for (a, _), (b, _) in zip(fmx._ExtractParams._fields_, oracle_py.ExtractParams._fields_):
        assert a == b


def test_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from form_amd import fmx
    with pytest.raises(fmx.FmxError):
        fmx.Context()


def test_null_context_is_rejected():
    from form_amd import fmx
    L = fmx.lib()
    assert L.fmx_sync(None) == 1  # FMX_E_INVAL
    assert L.fmx_last_error(None) == b"null context"


def test_ate_rmse_alignment():
    """ATE helper (form_amd.metrics): relative to the first pose, so a constant frame
    offset costs nothing and a translation error shows up exactly."""
    from form_amd import metrics, synth
    gt = [synth.trajectory_pose(k) for k in range(10)]
    off = np.eye(3, 4)
    off[:, 3] = [5.0, -2.0, 1.0]
    shifted = [metrics._mul(off, G) for G in gt]  # same trajectory, other world frame
    assert metrics.ate_rmse(shifted, gt) < 1e-12
    est = [metrics._mul(metrics._inv(gt[0]), G) for G in gt]  # estimator frame: identity at scan 0
    assert metrics.ate_rmse(est, gt) < 1e-12
    bad = [E.copy() for E in est]
    for E in bad[1:]:
        E[0, 3] += 0.01
    assert abs(metrics.ate_rmse(bad, gt) - 0.01 * np.sqrt(9 / 10)) < 1e-12
