"""Host staging of pageable scans (form_amd/csrc/stage.hpp), CPU only: helper threads and
the caller copying the chunks of several requests together, plain and packed
(float4 -> xyz), reuse after retire, helpers restarted — once plain and once under
ThreadSanitizer (tests/cpp/test_stage.cpp, built by __graft_entry__.build())."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["test_stage", "test_stage_tsan"])
def test_stage_helpers(name):
    path = os.path.join(ROOT, "tests", "cpp", name)
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: run __graft_entry__.build() (make -C tests/cpp)")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([path], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "stage ok" in r.stdout, r.stdout + r.stderr[-3000:]


def test_stage_helpers_respect_a_restricted_mask():
    """The same run restricted to two CPUs (taskset-like affinity before the library
    loads, and FMX_STAGE_CPUS narrowing it to one): the helper-CPU check holds."""
    path = os.path.join(ROOT, "tests", "cpp", "test_stage")
    cpus = sorted(os.sched_getaffinity(0))[:2]
    for env_extra in ({}, {"FMX_STAGE_CPUS": str(cpus[0])}):
        env = dict(os.environ, **env_extra)
        r = subprocess.run([path], capture_output=True, text=True, timeout=300, env=env,
                           preexec_fn=lambda: os.sched_setaffinity(0, set(cpus)))
        assert r.returncode == 0 and "stage ok" in r.stdout, r.stdout + r.stderr[-3000:]


def test_smoother_host():
    """The window smoother's host LM (form_amd/csrc/smoother.cpp: dense LM with priors, a
    linear container factor and callback-linearized pair factors, plain and split form;
    Schur marginal; Cholesky up to D = 108) — tests/cpp/test_smoother.cpp, also run under
    ASan + UBSan by tools/asan_check.sh."""
    path = os.path.join(ROOT, "tests", "cpp", "test_smoother")
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: run __graft_entry__.build() (make -C tests/cpp)")
    r = subprocess.run([path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "smoother ok" in r.stdout, r.stdout + r.stderr[-3000:]
