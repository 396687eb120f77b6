"""The opt-in product switch of libfmx under the GPU suite (VERDICT r5 "next round" 3).

FMX_MOMENTS=1 makes register_scan's LMs linearize from pair moments (window.hip
k_win_moments once per ICP iteration + host contractions, moments.cpp; the final LM
from the stored pairs' moments) instead of relinearizing every trial on the device.
The switch is read once per process, so each run is a fresh interpreter: a C2 stream
(64 x 1024, smoothing mode, sequential and pipelined) through register_scan against the
oracle Estimator (form/form.cpp:40-114), every pose within 1e-6 — the same bar as the
default path (tests/test_gpu_configs.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r'''
import sys
import torch  # first, as in every GPU process here: libfmx then binds torch's HIP runtime
root = sys.argv[1]
for p in (root, root + "/oracle", root + "/tests"):
    sys.path.insert(0, p)
import oracle_py
from form_amd import fmx
oracle_py.lib()
fmx.lib()
from test_gpu_configs import _stream
maxd, stats = _stream(fmx, oracle_py, sys.argv[2], int(sys.argv[3]), pipelined=True)
print("MAXD", maxd["sequential"], maxd["pipelined"])
print("MAPSCANS", stats["sequential"]["map_scans"], "PIPELINED", stats["pipelined"]["pipelined"])
'''


def _run(env_extra, config, n):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-u", "-c", _SCRIPT, ROOT, config, str(n)], env=env, capture_output=True,
                       text=True, timeout=600)
    print(r.stdout, r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    out = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines() if ln[:1].isupper()}
    return out


@pytest.mark.timeout(700)
def test_register_stream_c2_moments_mode():
    """24 C2 scans with FMX_MOMENTS=1 (ICP-loop LMs and the final LM from pair moments):
    poses within 1e-6 of the oracle's, sequential and pipelined, with the window full."""
    out = _run({"FMX_MOMENTS": "1"}, "c2", 24)
    seq, pipe = float(out["MAXD"][0]), float(out["MAXD"][1])
    assert seq < 1e-6 and pipe < 1e-6, out
    assert int(out["MAPSCANS"][0]) >= 10 and int(out["MAPSCANS"][2]) == 1, out
