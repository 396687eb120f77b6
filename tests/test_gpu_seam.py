"""The GTSAM seam as compiled C++ (include/fmx/fmx_seam.hpp): tests/cpp/test_seam, a
plain g++ -Wall -Werror program and the first non-ctypes caller of the C-ABI, unpacks
fmx_linearize's packed [A b]^T [A b] into GTSAM's HessianFactor blocks (G11, G12, g1,
G22, g2, f; gtsam.hpp:67-86) and the single-pose 7 x 7 (gtsam.hpp:144-170), and checks
them against the oracle's G and against [A b]^T [A b] formed from the oracle's raw rows
(1e-10), the error as f / 2, and FmxBatch's one launch per set of poses."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_seam")


def _binary():
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} missing: run __graft_entry__.build() (make -C tests/cpp)")
    return BIN


@pytest.mark.gpu
def test_seam_cpp_caller(fmx_mod):
    r = subprocess.run([_binary()], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "seam ok" in r.stdout


def test_seam_cpp_caller_links_without_device():
    """CPU side: the program links against libfmx.so and liboracle.so and, with no HIP
    device, fails fmx_create cleanly (status, no crash)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible (the gpu test covers this)")
    r = subprocess.run([_binary()], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "fmx_create failed" in r.stderr, (r.returncode, r.stderr)
