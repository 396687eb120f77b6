import sys; sys.path.insert(0, '.')
import torch
from form_amd import synth, fmx
geo = synth.GEOMETRIES["c4"]
p = synth.default_params(geo)
ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**p)))
w = synth.World()
ctx.profile(True)
for k in range(12):
    s = synth.raycast(w, synth.trajectory_pose(k), geo, synth.SEED + 7919 * (k + 1), "cuda:0")
    ctx.register_scan(s)
    torch.cuda.synchronize()
