"""bench.py — scan-to-submap registration throughput on MI355X (driver contract).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2|c3]
  (N > 1: launched by torch.distributed.run, one rank per GPU)

A step = Estimator::register_scan of one synthetic organized scan (form/form.cpp:40-114):
feature extraction, voxel-map build of the window keyscans, the ICP loop (match + LM
whose linearizations and error evaluations run on the GPU) and map insertion.  Scans
are ray-cast on the GPU before the timed region (inputs resident in HBM).  Multi-GPU:
real scans do not shard, so every rank registers its own independent
stream ("replicas only", weak scaling); value = all ranks' scans / max-over-ranks time.

Prints ONE JSON line (rank 0) with the contract fields plus `roofline` (dominant
kernel, HIP-event timed inside the timed region) and `cpu_baseline` (the C++ oracle
on the host cores, bounded sample of the same stream).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from form_amd import fmx, metrics, synth  # noqa: E402

METRIC = "scans/sec + Mpts/sec scan-to-submap ICP (128-beam); ATE delta vs reference"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c4", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--c5-side", type=int, default=7071, help="C5 terrain grid side (7071^2 = 50M voxels)")
    ap.add_argument("--c5-queries", type=int, default=2097152, help="C5 query points (2M)")
    ap.add_argument("--cpu-sample-s", type=float, default=15.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--profile-steps", type=int, default=None,
                    help="extra steps, after the timed ones, with per-kernel HIP-event timing (roofline); "
                         "default = --steps.  The timed region itself runs without event overhead.")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default="smooth", choices=["smooth", "single"],
                    help="ConstraintManager mode: smooth = the reference default (window smoother), "
                         "single = the disable_smoothing ablation (single-pose LM)")
    ap.add_argument("--no-ablation", action="store_true", help="skip the other mode's secondary measurement")
    ap.add_argument("--no-pin", action="store_true",
                    help="leave the registering thread unpinned (default: bound to the CPU it runs on for the "
                         "GPU measurements, released before the CPU baseline)")
    ap.add_argument("--subdiv", type=int, default=None, help="override voxel_subdivision (device map cells per voxel edge)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py output); default "
                         "profiles/traffic_latest.json (c4) or profiles/traffic_<workload>.json")
    return ap.parse_args()


def dist_setup(n):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world, local):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world, local):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def pmc_traffic(a, name):
    """HBM bytes per launch of kernel class `name` from the committed PMC summary of this
    workload (tools/gpu_pmc.sh, tools/gpu_c5pmc.sh), or None."""
    path = a.traffic_json or os.path.join(
        ROOT, "profiles", "traffic_latest.json" if a.workload == "c4" else f"traffic_{a.workload}.json")
    try:
        with open(path) as f:
            tj = json.load(f)
        if tj.get("workload") == a.workload and name in tj.get("kernels", {}):
            return tj["kernels"][name]["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    return None


def pin_thread(world, local):
    """Bind the calling (registering) thread to one CPU; returns the previous affinity.
    register_scan is a host-GPU latency chain (~15 host<->GPU round trips per scan): a
    thread migrating between cores mid-chain measured up to 12 % slower on some boxes
    (tools/step_times.py), never faster unpinned.  One rank: the CPU it runs on.  Several
    ranks: distinct CPUs from each GPU's NUMA-local list (sysfs local_cpulist)."""
    old = os.sched_getaffinity(0)
    cpu = None
    if world > 1:
        try:
            pr = torch.cuda.get_device_properties(local)
            bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
            cpus = []
            for part in open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus += list(range(int(lo), int(hi or lo) + 1))
            cands = [c for c in cpus if c in old]
            cpu = cands[(4 * local) % len(cands)] if cands else None
        except (OSError, ValueError, AttributeError):
            cpu = None
        if cpu is None:
            return None
    else:
        with open("/proc/thread-self/stat") as f:
            cpu = int(f.read().rsplit(")", 1)[1].split()[36])
    os.sched_setaffinity(0, {cpu})
    return old


def cpu_baseline(scans_host, params, budget_s, single):
    """Oracle register_scan on the host cores over the first scans of the same stream."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O  # CPU baseline only (test infrastructure)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    prm = O.default_params(params)
    prm.disable_smoothing = int(single)
    est = O.Estimator(prm, threads)
    times = []
    t_all = time.perf_counter()
    poses = []
    for s in scans_host:
        t0 = time.perf_counter()
        T, _, _ = est.register_scan(s)
        times.append(time.perf_counter() - t0)
        poses.append(T)
        if time.perf_counter() - t_all > budget_s:
            break
    # steady state: skip the first (empty-map) scan when there is more than one
    steady = times[1:] if len(times) > 2 else times
    per = float(np.median(steady))
    return dict(value=1.0 / per, unit="scans/s", cores=threads, kind="port",
                sample=f"oracle register_scan ({'single-pose' if single else 'smoothing'} mode; C++ restatement, "
                       f"std::thread at the reference's TBB sites: normals, match queries, factor linearization) "
                       f"over the first {len(times)} scans of the same synthetic stream; median of "
                       f"{len(steady)} steady-state scans = {per * 1e3:.1f} ms/scan",
                ms_per_scan=per * 1e3), poses


def ate_block(scans_host, oracle_poses, params, k0, device, single):
    """ATE of the GPU path and of the CPU oracle path over the same scans against the
    synthetic ground truth (the newer_college ATE is unavailable
    offline).  Untimed; a fresh context replays the sample."""
    n = len(oracle_poses)
    ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**params),
                                          disable_smoothing=single), device=device)
    gpu = []
    for s in scans_host[:n]:
        ctx.register_scan(s)
        gpu.append(ctx.current_pose())
    gt = [synth.trajectory_pose(k0 + k) for k in range(n)]
    a_gpu, a_cpu = metrics.ate_rmse(gpu, gt), metrics.ate_rmse(oracle_poses, gt)
    return {"gpu_m": round(a_gpu, 6), "cpu_port_m": round(a_cpu, 6), "delta_m": round(a_gpu - a_cpu, 9),
            "max_pose_diff_m": round(float(max(np.abs(np.asarray(g)[:, 3] - np.asarray(o)[:, 3]).max()
                                               for g, o in zip(gpu, oracle_poses))), 9),
            "scans": n, "truth": "synthetic trajectory (synth.trajectory_pose)"}


def run_c5(a, rank, world, local):
    """C5: 2M query points vs a 50M-voxel terrain submap, queries
    sharded over ranks, map replicated.  A step = one ICP iteration of the full 2M
    point set: match the shard, reduce it to the 7x7 normal equations (single pose),
    all_reduce (RCCL over xGMI when N > 1), identical Gauss-Newton update on every
    rank.  Strong scaling: the total work per step is fixed."""
    from form_amd import shard
    dev = f"cuda:{local}"
    w = 0.8
    pos4, nrm4 = shard.terrain_map(a.c5_side, w, synth.SEED, dev)
    Ttrue = shard.compose(np.hstack([np.eye(3), np.array([[0.03], [-0.04], [0.0]])]),
                          shard.expmap(np.array([0.0, 0.0, np.radians(0.5), 0.0, 0.0, 0.0])))
    q4, n4 = shard.make_queries(pos4, nrm4, a.c5_queries, Ttrue, 0.05, synth.SEED + 1)
    b, e = shard.shard_bounds(a.c5_queries, rank, world)
    n_map = pos4.shape[0]
    prm = fmx.EstimatorParams(keypoint_pool_capacity=n_map + 1024, voxel_subdivision=a.subdiv or 1)  # one record per voxel
    ctx = fmx.Context(prm, device=local)
    ctx.keypoints_add_device(0, pos4, nrm4)
    I34 = np.hstack([np.eye(3), np.zeros((3, 1))])
    ctx.map_build([0], I34[None], w)
    qs, ns = q4[b:e].contiguous(), n4[b:e].contiguous()
    ctx.set_queries_device(qs, ns)
    del pos4, nrm4
    torch.cuda.synchronize()
    T = I34.copy()

    def step(T):
        ctx.match(T, w)
        G, _ = ctx.linearize(I34[None], T[None], 0.1, True)
        Gs = shard.allreduce_sum(G[0], device=dev)
        return shard.compose(T, shard.expmap(shard.gauss_newton_step(Gs)))

    for _ in range(a.warmup):
        T = step(T)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        T = step(T)
    torch.cuda.synchronize()
    barrier(world)
    t_local = time.perf_counter() - t0
    ctx.profile(True)
    ctx.profile_reset()
    psteps = a.steps if a.profile_steps is None else a.profile_steps
    for _ in range(psteps):
        T = step(T)
    ctx.sync()
    prof = ctx.profile_read()
    work = ctx.match_work()
    t_max = max_over_ranks(t_local, world, local)
    if rank != 0:
        return None
    value = a.steps / t_max
    name, d = max(prof.items(), key=lambda kv: kv[1]["ms"])
    avg_ms = d["ms"] / max(d["launches"], 1)
    bytes_per = d["bytes"] / max(d["launches"], 1)
    achieved = bytes_per / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    err = float(np.abs(T - Ttrue).max())
    return {
        "metric": METRIC, "value": round(value, 3), "unit": "scans/s (2M-point scans)", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(t_max / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "fp32 points / fp64 map, residuals and normal equations",
        "data": "synthetic (jittered terrain grid, seed 0x464F524D)",
        "config": {"workload": f"c5: {a.c5_queries} queries vs {n_map}-voxel submap, queries sharded, "
                               "7x7 normal equations all-reduced", "points_per_scan": a.c5_queries,
                   "parallelism": f"query shards x{world} + all_reduce"},
        "mpts_per_s": round(value * a.c5_queries / 1e6, 3),
        "roofline": dict(bound="hbm", kernel=name, achieved=round(achieved, 3), peak=HBM_PEAK_GBS, unit="GB/s",
                         frac=round(achieved / HBM_PEAK_GBS, 6), traffic=pmc_traffic(a, name),
                         avg_launch_us=round(avg_ms * 1e3, 3), alg_bytes_per_launch=bytes_per),
        "kernels_ms_per_step": {k: round(v["ms"] / max(psteps, 1), 4) for k, v in prof.items()},
        "pose_error_vs_truth": err,
        "match_work_per_query": {k: round(v / max(work["queries"], 1), 3) for k, v in work.items() if k != "queries"},
    }


def main():
    a = parse()
    rank, world, local = dist_setup(a.gpus)
    if a.workload == "c5":
        torch.cuda.set_device(local)
        out = run_c5(a, rank, world, local)
        if out is not None:
            print(json.dumps(out))
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    dev = f"cuda:{local}"
    torch.cuda.set_device(local)
    geo = synth.GEOMETRIES[a.workload]
    params = synth.default_params(geo)
    n_pts = geo.rows * geo.cols
    # independent stream per rank (replicas): different trajectory phase
    world_obj = synth.World()
    k0 = 1000 * rank
    psteps = a.steps if a.profile_steps is None else a.profile_steps
    total = a.warmup + a.steps + psteps
    scans = [synth.raycast(world_obj, synth.trajectory_pose(k0 + k), geo, synth.SEED + 7919 * (k0 + k + 1), dev)
             for k in range(total)]
    torch.cuda.synchronize()
    single = a.mode == "single"

    def new_ctx(single_pose):
        return fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**params),
                                               voxel_subdivision=a.subdiv or 0, disable_smoothing=single_pose),
                           device=local)

    prev_aff = None if a.no_pin else pin_thread(world, local)
    ablation = None
    if not a.no_ablation:  # the other mode over the same scans (secondary, untimed by the driver)
        actx = new_ctx(not single)
        for k in range(a.warmup):
            actx.register_scan(scans[k])
        actx.sync()
        ta = time.perf_counter()
        for k in range(a.warmup, a.warmup + a.steps):
            actx.register_scan(scans[k])
        actx.sync()
        ta = time.perf_counter() - ta
        ablation = {"mode": "single-pose (disable_smoothing)" if not single else "smoothing (default)",
                    "scans_per_s": round(a.steps / ta, 3), "ms_per_step": round(ta / a.steps * 1e3, 3)}
        actx.close()
        del actx
    ctx = new_ctx(single)
    for k in range(a.warmup):
        ctx.register_scan(scans[k])
    ctx.sync()
    stats = []
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.warmup, a.warmup + a.steps):
        ctx.register_scan(scans[k])
        stats.append(ctx.last_stats())
    ctx.sync()
    torch.cuda.synchronize()
    barrier(world)
    t_local = time.perf_counter() - t0
    # roofline pass: same stream continued, per-kernel HIP events on the context stream
    ctx.profile(True)
    ctx.profile_reset()
    for k in range(a.warmup + a.steps, total):
        ctx.register_scan(scans[k])
    ctx.sync()
    prof = ctx.profile_read()
    work = ctx.match_work()
    ctx.profile(False)
    t_max = max_over_ranks(t_local, world, local)
    scans_total = sum_over_ranks(float(a.steps), world, local)
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    value = scans_total / t_max
    ms_per_step = t_max / a.steps * 1e3
    # dominant kernel by device time in the timed region
    dom = max(prof.items(), key=lambda kv: kv[1]["ms"])
    name, d = dom
    avg_ms = d["ms"] / max(d["launches"], 1)
    bytes_per = d["bytes"] / max(d["launches"], 1)
    achieved = bytes_per / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = pmc_traffic(a, name)
    roof = dict(bound="hbm", kernel=name, achieved=round(achieved, 3), peak=HBM_PEAK_GBS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBS, 6), traffic=traffic, avg_launch_us=round(avg_ms * 1e3, 3),
                alg_bytes_per_launch=bytes_per)
    st_mean = {k: float(np.mean([s[k] for s in stats])) for k in stats[0]}
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "scans/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32 points / fp64 map, residuals and normal equations",
        "data": "synthetic (ray-cast organized scans, seed 0x464F524D; no datasets offline)",
        "config": {"workload": f"{a.workload}: {geo.rows}x{geo.cols} organized scan stream ({n_pts} pts/scan), "
                               f"register_scan, {'single-pose ablation (disable_smoothing)' if single else 'smoothing mode (ConstraintManager default)'}",
                   "points_per_scan": n_pts, "parallelism": f"replicas x{world}"},
        "mpts_per_s": round(value * n_pts / 1e6, 3),
        "roofline": roof,
        "kernels_ms_per_step": {k: round(v["ms"] / max(psteps, 1), 4) for k, v in prof.items()},
        "profile_steps": psteps,
        "counters": st_mean,
        "match_work_per_query": {k: round(v / max(work["queries"], 1), 3) for k, v in work.items() if k != "queries"},
    }
    if ablation is not None:
        out["ablation"] = ablation
    if prev_aff is not None:
        os.sched_setaffinity(0, prev_aff)  # the CPU baseline's threads use every host core
    if not a.no_cpu_baseline and world == 1:
        host = [s.cpu().numpy() for s in scans[: min(total, 60)]]
        out["cpu_baseline"], opos = cpu_baseline(host, params, a.cpu_sample_s, single)
        out["ate"] = ate_block(host, opos, params, k0, local, single)
    print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
