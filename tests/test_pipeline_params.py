"""The evalio pipeline parameters of form._core.FORM (python/bindings.cpp:66-88) map
onto fmx_params exactly as the reference's EVALIO_SETUP_PARAMS does, including the
YAML key `max_dist_map` -> KeypointMapParams::min_dist_map (:85) and
`disable_smoothing` -> ConstraintManager::Params (:79); and the lidar geometry comes
from set_lidar_params (:126-132).  Host only: no device needed."""
import types

import pytest

# the FORM pipeline entries of the reference's config/25.10.03_full.yaml:9-17
FULL_YAML_FORM_ENTRIES = [
    {"pipeline": "form"},
    {"pipeline": "form", "name": "form_planar", "point_feats_per_sector": 0},
    {"pipeline": "form", "name": "form_single", "disable_smoothing": True},
]


def test_defaults_equal_reference_table():
    from form_amd import fmx
    d = fmx.FORM.default_params()
    assert d == {"neighbor_points": 5, "num_sectors": 6, "planar_threshold": 1.0, "planar_feats_per_sector": 50,
                 "point_feats_per_sector": 3, "radius": 1.0, "min_points": 5, "max_dist_matching": 0.8,
                 "new_pose_threshold": 1e-4, "max_num_rematches": 30, "disable_smoothing": False,
                 "max_num_keyscans": 50, "max_num_recent_scans": 10, "max_steps_unused_keyscan": 10,
                 "keyscan_match_ratio": 0.1, "max_dist_map": 0.1, "num_threads": 0}
    f = fmx.FORM()
    assert f.get_params() == d
    assert fmx.FORM.name() == "form"


def test_full_yaml_ablations_reach_the_c_params():
    from form_amd import fmx
    got = []
    for entry in FULL_YAML_FORM_ENTRIES:
        f = fmx.FORM()
        f.set_params(entry)
        got.append(f.params.to_c())
    base, planar, single = got
    assert base.disable_smoothing == 0 and base.extraction.point_feats_per_sector == 3
    assert planar.extraction.point_feats_per_sector == 0 and planar.disable_smoothing == 0
    assert single.disable_smoothing == 1  # the ablation runs the single-pose LM
    assert single.extraction.point_feats_per_sector == 3


def test_max_dist_map_lands_in_min_dist_map():
    from form_amd import fmx
    f = fmx.FORM()
    f.set_params({"max_dist_map": 0.25, "max_dist_matching": 1.1, "neighbor_points": 4, "num_threads": 7,
                  "keyscan_match_ratio": 0.2, "max_num_recent_scans": 6})
    c = f.params.to_c()
    assert c.min_dist_map == 0.25 and c.max_dist_matching == 1.1 and c.extraction.neighbor_points == 4
    assert c.keyscan_match_ratio == 0.2 and c.max_num_recent_scans == 6
    assert f.get_params()["max_dist_map"] == 0.25 and f.num_threads == 7
    with pytest.raises(KeyError):
        f.set_params({"min_dist_map": 0.3})  # not a pipeline key in the reference


def test_set_lidar_params_sets_geometry():
    from form_amd import fmx
    f = fmx.FORM()
    f.set_lidar_params(types.SimpleNamespace(min_range=0.5, max_range=120.0, num_rows=128, num_columns=2048))
    c = f.params.to_c()
    assert c.extraction.min_norm_squared == 0.25 and c.extraction.max_norm_squared == 14400.0
    assert c.extraction.num_rows == 128 and c.extraction.num_columns == 2048
