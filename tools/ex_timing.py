import sys; sys.path.insert(0, '.')
import torch
from form_amd import synth, fmx
scan, T, geo = synth.make_scan("c4", 3, device="cuda:0")
p = synth.default_params(geo)
ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**p)))
for i in range(3):
    ctx.extract(scan, 3); ctx.sync()
print(ctx.extract(scan, 3))
