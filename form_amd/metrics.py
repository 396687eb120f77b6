"""Trajectory metrics for the synthetic stream (the ATE stand-in).

The reference's ATE on newer_college_2020 needs evalio, a built form._core and a
dataset download, none available offline.  Its stand-in here: absolute trajectory
error of the GPU path and of the CPU oracle path against the synthetic ground truth
(synth.trajectory_pose) over the same scans, and their difference.
"""
from __future__ import annotations

import numpy as np


def _inv(T: np.ndarray) -> np.ndarray:
    R, t = T[:, :3], T[:, 3]
    out = np.zeros((3, 4))
    out[:, :3] = R.T
    out[:, 3] = -R.T @ t
    return out


def _mul(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    out = np.zeros((3, 4))
    out[:, :3] = A[:, :3] @ B[:, :3]
    out[:, 3] = A[:, :3] @ B[:, 3] + A[:, 3]
    return out


def ate_rmse(est, gt) -> float:
    """RMSE of translation after expressing both trajectories relative to their first
    pose (the estimator starts at identity at scan 0, evalio's alignment-free ATE)."""
    est = [np.asarray(T, np.float64).reshape(3, 4) for T in est]
    gt = [np.asarray(T, np.float64).reshape(3, 4) for T in gt]
    if len(est) != len(gt) or not est:
        raise ValueError("trajectories must be non-empty and of equal length")
    e0, g0 = _inv(est[0]), _inv(gt[0])
    d = [(_mul(e0, E)[:, 3] - _mul(g0, G)[:, 3]) for E, G in zip(est, gt)]
    return float(np.sqrt(np.mean(np.sum(np.square(d), axis=1))))
