"""In-kernel phase stamps of the extraction kernels (build with -DFMX_EXTRACT_TIMING=1,
run with FMX_LIB pointing at it): a few C4 extractions, the kernels print per-row
phase durations in 10-ns ticks."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
from form_amd import fmx, synth

scan, T, geo = synth.make_scan("c4", 0)
p = synth.default_params(geo)
ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**p)))
s = scan.to("cuda:0")
for k in range(4):
    ctx.extract(s, k)
torch.cuda.synchronize()
