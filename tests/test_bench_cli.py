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
