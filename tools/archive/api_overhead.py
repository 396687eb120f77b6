"""Host cost of fmx API calls from Python (ctypes + guard + hipSetDevice), on the GPU box."""
import time

import torch

from form_amd import fmx

ctx = fmx.Context(fmx.EstimatorParams())
e = ctx.params.extraction
t = torch.zeros(e.num_rows * e.num_columns, 4, device="cuda:0")
N = 2000
for name, fn in (("last_stats", lambda: ctx.last_stats()), ("next_scan", lambda: ctx.next_scan(t)),
                 ("next_scan(None)", lambda: ctx.next_scan(None)), ("sync", lambda: ctx.sync())):
    for _ in range(100):
        fn()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    print(f"{name:16s} {(time.perf_counter() - t0) / N * 1e6:8.2f} us/call")
ctx.close()
