"""Several contexts on one GPU, each driven from its own host thread (bench.py's
concurrent_streams, a serving setup): every stream registers exactly as it does alone
(bit for bit), so contexts share no mutable state (include/fmx/fmx.h: one context per
host thread)."""
import threading

import numpy as np
import pytest
import torch

from form_amd import synth

pytestmark = pytest.mark.gpu


def _stream(fmx_mod, scans, p, pipelined):
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams(extraction=fmx_mod.KeypointExtractionParams(**p)))
    out = []
    for k in range(len(scans)):
        if pipelined and k + 1 < len(scans):
            ctx.next_scan(scans[k + 1])
        ctx.register_scan(scans[k])
        out.append(ctx.current_pose())
    ctx.close()
    return np.stack(out)


@pytest.mark.parametrize("config,n,threads", [("small", 24, 4), ("c4", 12, 3)])
def test_concurrent_contexts_equal_sequential(fmx_mod, config, n, threads):
    geo = synth.GEOMETRIES[config]
    p = synth.default_params(geo)
    world = synth.World()
    scans = [synth.make_scan(config, k, world=world)[0].to("cuda:0") for k in range(n)]
    torch.cuda.synchronize()
    ref = _stream(fmx_mod, scans, p, True)
    got = [None] * threads
    errs = []

    def run(i):
        try:
            got[i] = _stream(fmx_mod, scans, p, i % 2 == 0)  # pipelined and sequential side by side
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for i in range(threads):
        assert np.array_equal(got[i], ref), (i, np.abs(got[i] - ref).max())
