"""bench.py's multi-GPU contract on the host (VERDICT r2 "next round" 2a): --gpus N
never reports a run on fewer ranks than asked for."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=300)


def test_more_gpus_than_devices_fails_loudly():
    import torch
    n = torch.cuda.device_count() + 1
    r = _run(["--gpus", str(n), "--steps", "1"])
    assert r.returncode != 0
    assert r.stdout.strip() == ""  # no JSON line
    assert f"--gpus {n}" in r.stderr


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "1", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_box_fails():
    """On the 1-GPU box a --gpus 2 run exits non-zero before touching the GPU."""
    import torch
    if torch.cuda.device_count() != 1:
        pytest.skip("needs exactly one visible GPU")
    r = _run(["--gpus", "2", "--steps", "1"])
    assert r.returncode != 0 and r.stdout.strip() == ""


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_rehearsed_two_rank_orchestration(fmx_mod):
    """The --gpus N path end to end on the 1-GPU box (--rehearse-ranks, test only):
    spawn_ranks -> torch.distributed.run -> 2 ranks on cuda:0, gloo for the control
    collectives -> C4 replicas and the sharded C5 registrations through max_over_ranks,
    the C5 exchange as a host all-reduce.  Rank 0 prints one parsable rehearsal record
    (never a driver line), and the 2-rank C5 pose equals a 1-rank registration of the
    whole query set to 1e-9 (summation order only)."""
    import json

    import numpy as np

    from form_amd import shard, synth
    side, nq, w = 1501, 200000, 0.8
    r = _run(["--gpus", "2", "--rehearse-ranks", "--steps", "3", "--warmup", "1", "--prefill", "4",
              "--c5-side", str(side), "--c5-queries", str(nq), "--c5-steps", "2", "--c5-warmup", "0",
              "--no-cpu-baseline", "--streams", "", "--no-ablation", "--sub-workloads", "", "--no-host-input",
              "--no-pin"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["rehearsal"] is True and rec["value"] is None and rec["ranks"] == 2
    assert rec["c4_scans_per_s_all_ranks"] > 0
    I34 = np.hstack([np.eye(3), np.zeros((3, 1))])
    pos4, nrm4 = shard.terrain_map(side, w, synth.SEED, "cuda:0")
    q4, n4 = shard.make_queries(pos4, nrm4, nq, shard.c5_offset(), 0.03, synth.SEED + 1)
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams(keypoint_pool_capacity=pos4.shape[0] + 1024))
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], w)
    ctx.set_queries_device(q4, n4)
    T1, it1 = ctx.register_points(I34, w, 0.1, 30, 1e-4)
    ctx.close()
    T2 = np.array(rec["sharded_c5"]["pose"]).reshape(3, 4)
    assert rec["sharded_c5"]["icp_iters_per_registration"] == it1
    assert np.abs(T2 - T1).max() < 1e-9, np.abs(T2 - T1).max()
