"""Profiling aid (not part of the product): 40 serial frames (graph mode) for a kernel trace of the
mapping stage."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
from lvo_amd_loader import lvo
frames = lvo.synth.sequence("hdl64", 40)
d = [torch.from_numpy(f).to("cuda:0") for f in frames]
ctx = lvo.Context(lvo.abi.default_params(64), device=0)
for k, f in enumerate(d):
    ctx.process_scan(device_ptr=f.data_ptr(), n=len(frames[k]))
torch.cuda.synchronize()
print("done")
