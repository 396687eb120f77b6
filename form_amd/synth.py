"""Deterministic synthetic organized LiDAR scans (SURVEY.md §8(d) "Synthetic inputs").

The reference ships no data and newer_college needs a network download, so every
test and benchmark input is ray-cast here: a sensor 1.8 m above the floor of an
80 x 60 x 10 m room holding 40 yaw-rotated boxes and 20 vertical cylinders.  Rows
are spread uniformly in elevation, columns over 360 deg of azimuth; range noise
N(0, sigma) and random dropouts (zero points, which the extractor's range check
rejects) are added.  Points come out in the sensor frame as an organized R x C
float32 array with a zero pad (the PointXYZf layout, form/utils.hpp:38-46).

Plain torch, so the same code runs on the CPU (tests) and on the GPU (bench.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

SEED = 0x464F524D  # "FORM"


@dataclass
class ScanGeometry:
    rows: int = 128
    cols: int = 2048
    elev_deg: float = 22.5  # rows uniformly over [-elev, +elev]
    noise: float = 0.01
    dropout: float = 0.02
    max_range: float = 100.0


GEOMETRIES = {
    "c2": ScanGeometry(64, 1024, 16.6, 0.01, 0.02),    # OS1-64
    "c3": ScanGeometry(64, 2048, 16.6, 0.01, 0.08),    # HDL-64E stand-in, organized
    "c4": ScanGeometry(128, 2048, 22.5, 0.01, 0.02),   # OS2-128
    "tiny": ScanGeometry(16, 256, 15.0, 0.01, 0.02),
    "small": ScanGeometry(32, 512, 16.6, 0.01, 0.02),
    "wide": ScanGeometry(8, 4096, 15.0, 0.01, 0.02),  # > 2048 columns: the split normals path
}


class World:
    """Room + boxes + cylinders; fixed by the seed."""

    def __init__(self, seed: int = SEED, n_boxes: int = 40, n_cyl: int = 20):
        g = np.random.default_rng(seed)
        self.room = np.array([[-40.0, 40.0], [-30.0, 30.0], [0.0, 10.0]])
        cx = g.uniform(-36, 36, n_boxes)
        cy = g.uniform(-26, 26, n_boxes)
        # keep a corridor along y ~ 0 free for the trajectory
        cy = np.where(np.abs(cy) < 4.0, cy + np.sign(cy + 1e-9) * 5.0, cy)
        self.box_c = np.stack([cx, cy, np.zeros(n_boxes)], 1)
        self.box_h = np.stack([g.uniform(0.4, 3.0, n_boxes), g.uniform(0.4, 3.0, n_boxes),
                               g.uniform(0.5, 4.0, n_boxes)], 1)  # half extents (z full height/2)
        self.box_c[:, 2] = self.box_h[:, 2]
        self.box_yaw = g.uniform(-math.pi, math.pi, n_boxes)
        ccx = g.uniform(-36, 36, n_cyl)
        ccy = g.uniform(-26, 26, n_cyl)
        ccy = np.where(np.abs(ccy) < 4.0, ccy + np.sign(ccy + 1e-9) * 5.0, ccy)
        self.cyl = np.stack([ccx, ccy, g.uniform(0.15, 1.0, n_cyl), g.uniform(2.0, 6.0, n_cyl)], 1)


def trajectory_pose(k: int, rate_hz: float = 10.0, speed: float = 1.5, yaw_rate: float = 0.1,
                    start=(-15.0, 0.0, 1.8)) -> np.ndarray:
    """World pose (3x4 row-major) of scan k: 1.5 m/s forward, 0.1 rad/s yaw, 10 Hz,
    with a small deterministic roll/pitch wobble so every DoF is excited."""
    t = k / rate_hz
    yaw = yaw_rate * t
    if abs(yaw_rate) > 1e-12:
        x = start[0] + speed / yaw_rate * math.sin(yaw)
        y = start[1] + speed / yaw_rate * (1.0 - math.cos(yaw))
    else:
        x, y = start[0] + speed * t, start[1]
    z = start[2] + 0.05 * math.sin(0.7 * t)
    roll = 0.02 * math.sin(1.3 * t)
    pitch = 0.015 * math.sin(0.9 * t + 0.3)
    cr, sr, cp, sp, cy, sy = (math.cos(roll), math.sin(roll), math.cos(pitch), math.sin(pitch),
                              math.cos(yaw), math.sin(yaw))
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1.0]])
    Ry = np.array([[cp, 0, sp], [0, 1.0, 0], [-sp, 0, cp]])
    Rx = np.array([[1.0, 0, 0], [0, cr, -sr], [0, sr, cr]])
    T = np.zeros((3, 4))
    T[:, :3] = Rz @ Ry @ Rx
    T[:, 3] = (x, y, z)
    return T


def _ray_dirs(geo: ScanGeometry, device, dtype=torch.float64) -> torch.Tensor:
    el = torch.linspace(math.radians(geo.elev_deg), -math.radians(geo.elev_deg), geo.rows,
                        device=device, dtype=dtype)
    az = torch.arange(geo.cols, device=device, dtype=dtype) * (2 * math.pi / geo.cols)
    E, A = torch.meshgrid(el, az, indexing="ij")
    d = torch.stack([torch.cos(E) * torch.cos(A), torch.cos(E) * torch.sin(A), torch.sin(E)], -1)
    return d.reshape(-1, 3)


def raycast(world: World, pose34: np.ndarray, geo: ScanGeometry, seed: int, device="cpu") -> torch.Tensor:
    """Organized scan in the sensor frame: (rows*cols, 4) float32, pad 0, zeros for drops."""
    dev = torch.device(device)
    d_s = _ray_dirs(geo, dev)
    R = torch.as_tensor(pose34[:, :3], device=dev, dtype=torch.float64)
    o = torch.as_tensor(pose34[:, 3], device=dev, dtype=torch.float64)
    d = d_s @ R.T  # world directions
    n = d.shape[0]
    best = torch.full((n,), float("inf"), device=dev, dtype=torch.float64)
    inv = 1.0 / torch.where(d.abs() < 1e-12, torch.full_like(d, 1e-12), d)

    # room interior: exit distance along each axis
    room = torch.as_tensor(world.room, device=dev, dtype=torch.float64)
    t_lo = (room[:, 0] - o) * inv
    t_hi = (room[:, 1] - o) * inv
    t_exit = torch.maximum(t_lo, t_hi).min(dim=1).values
    best = torch.minimum(best, t_exit)

    # yaw-rotated boxes (slab test in box frame)
    bc = torch.as_tensor(world.box_c, device=dev, dtype=torch.float64)
    bh = torch.as_tensor(world.box_h, device=dev, dtype=torch.float64)
    yaw = torch.as_tensor(world.box_yaw, device=dev, dtype=torch.float64)
    c, s = torch.cos(yaw), torch.sin(yaw)
    for b in range(bc.shape[0]):
        ob = o - bc[b]
        # rotate into the box frame (R_box^T)
        obx = c[b] * ob[0] + s[b] * ob[1]
        oby = -s[b] * ob[0] + c[b] * ob[1]
        dbx = c[b] * d[:, 0] + s[b] * d[:, 1]
        dby = -s[b] * d[:, 0] + c[b] * d[:, 1]
        dbz = d[:, 2]
        tmin = torch.full((n,), -float("inf"), device=dev, dtype=torch.float64)
        tmax = torch.full((n,), float("inf"), device=dev, dtype=torch.float64)
        for oo, dd, h in ((obx, dbx, bh[b, 0]), (oby, dby, bh[b, 1]), (ob[2], dbz, bh[b, 2])):
            dd = torch.where(dd.abs() < 1e-12, torch.full_like(dd, 1e-12), dd)
            t1 = (-h - oo) / dd
            t2 = (h - oo) / dd
            tmin = torch.maximum(tmin, torch.minimum(t1, t2))
            tmax = torch.minimum(tmax, torch.maximum(t1, t2))
        hit = (tmax >= tmin) & (tmin > 1e-6)
        best = torch.where(hit & (tmin < best), tmin, best)

    # vertical cylinders (side surface only)
    cyl = torch.as_tensor(world.cyl, device=dev, dtype=torch.float64)
    for k in range(cyl.shape[0]):
        cx, cy, r, h = cyl[k]
        ox, oy = o[0] - cx, o[1] - cy
        a = d[:, 0] ** 2 + d[:, 1] ** 2
        bq = 2 * (ox * d[:, 0] + oy * d[:, 1])
        cq = ox * ox + oy * oy - r * r
        disc = bq * bq - 4 * a * cq
        ok = disc > 0
        sq = torch.sqrt(torch.clamp(disc, min=0))
        t = (-bq - sq) / (2 * a.clamp(min=1e-12))
        z = o[2] + t * d[:, 2]
        hit = ok & (t > 1e-6) & (z >= 0) & (z <= h)
        best = torch.where(hit & (t < best), t, best)

    g = torch.Generator(device="cpu").manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
    noise = torch.randn(n, generator=g, dtype=torch.float64).to(dev) * geo.noise
    drop = torch.rand(n, generator=g, dtype=torch.float64).to(dev) < geo.dropout
    rng = best + noise
    valid = torch.isfinite(best) & (rng < geo.max_range) & ~drop
    pts = d_s * rng[:, None]
    pts = torch.where(valid[:, None], pts, torch.zeros_like(pts))
    out = torch.zeros((n, 4), device=dev, dtype=torch.float32)
    out[:, :3] = pts.to(torch.float32)
    return out


def make_scan(config: str = "tiny", k: int = 0, seed: int = SEED, device="cpu", world: World | None = None):
    """(scan (N,4) float32, pose34, geometry) for scan index k of the stream."""
    geo = GEOMETRIES[config]
    w = world or World(seed)
    T = trajectory_pose(k)
    return raycast(w, T, geo, seed + 7919 * (k + 1), device), T, geo


def default_params(geo: ScanGeometry) -> dict:
    """FORM defaults (extraction.hpp:59-88, matcher.hpp:32-41, ...) for a geometry."""
    return dict(
        neighbor_points=5, num_sectors=6, planar_threshold=1.0, planar_feats_per_sector=50,
        point_feats_per_sector=3, radius=1.0, min_points=5, min_norm_squared=1.0,
        max_norm_squared=100.0 * 100.0, num_columns=geo.cols, num_rows=geo.rows,
    )
