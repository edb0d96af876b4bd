"""Profiling aid (not part of the product): serial mapping stage wall time with the rebuild / stack lanes
concurrent (default) or serialised (ALOAM_EXP=8), to see whether the two lanes actually overlap."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
from lvo_amd_loader import lvo
frames = lvo.synth.sequence("hdl64", 50)
d = [torch.from_numpy(f).to("cuda:0") for f in frames]
torch.cuda.synchronize()
ctx = lvo.Context(lvo.abi.default_params(64), device=0)
T = []
for k, f in enumerate(d):
    ctx.scan_registration(len(frames[k]), device_ptr=f.data_ptr())
    od = ctx.odometry()
    t0 = time.perf_counter()
    ctx.mapping()
    T.append(time.perf_counter() - t0)
print("ALOAM_EXP", os.environ.get("ALOAM_EXP", "0"), "map ms median %.4f min %.4f" % (np.median(T[10:]) * 1e3, np.min(T[10:]) * 1e3), flush=True)
