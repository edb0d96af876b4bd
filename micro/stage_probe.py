"""Profiling aid (not part of the product): wall time of each stage call in graph mode (serial, one
context), the per-frame mapping breakdown with parts isolated by the ALOAM_EXP knob off, and the
pipelined throughput for comparison."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
from lvo_amd_loader import lvo

frames = lvo.synth.sequence("hdl64", 60)
dev = torch.device("cuda", 0)
d = [torch.from_numpy(f).to(dev) for f in frames]
torch.cuda.synchronize()
def run(label, **over):
  p = lvo.abi.default_params(64)
  for k_, v_ in over.items():
    setattr(p, k_, v_)
  ctx = lvo.Context(p, device=0)
  T = []
  for k, f in enumerate(d):
    t0 = time.perf_counter()
    ctx.scan_registration(len(frames[k]), device_ptr=f.data_ptr())
    t1 = time.perf_counter()
    od = ctx.odometry()
    t2 = time.perf_counter()
    mp = ctx.mapping() if od["publish_to_mapping"] else None
    t3 = time.perf_counter()
    if k >= 10:
        T.append((t1 - t0, t2 - t1, t3 - t2))
  T = np.array(T) * 1e3
  print(label, "stage wall ms (scanreg, odom, map): median", np.median(T, 0).round(4), "min", T.min(0).round(4), flush=True)
  ctx.close()

run("default")
run("odom_rounds=0 map_rounds=0", odom_rounds=0, map_rounds=0)
run("odom_rounds=1 map_rounds=1", odom_rounds=1, map_rounds=1)
run("max_solver_iterations=1", max_solver_iterations=1)
