"""Profiling aid (not part of the product): pipelined throughput with stages shortened through the
round-count parameters, to separate stage time from cross-stage contention."""
import os, sys, time
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
from lvo_amd_loader import lvo

frames = lvo.synth.sequence("hdl64", 130)
dev = torch.device("cuda", 0)
d = [torch.from_numpy(f).to(dev) for f in frames]
torch.cuda.synchronize()


def pipe_rate(label, **over):
    p = lvo.abi.default_params(64)
    for k, v in over.items():
        setattr(p, k, v)
    pl = lvo.Pipeline(p, device=0)
    for k in range(10):
        pl.push(device_ptr=d[k].data_ptr(), n=len(frames[k]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(10, 130):
        pl.push(device_ptr=d[k].data_ptr(), n=len(frames[k]))
    pl.flush()
    dt = time.perf_counter() - t0
    pl.close()
    print(f"{label:40s} pipeline {120 / dt:8.1f} scans/s  {dt / 120 * 1e3:.3f} ms/scan", flush=True)


def serial(label, **over):
    p = lvo.abi.default_params(64)
    for k, v in over.items():
        setattr(p, k, v)
    ctx = lvo.Context(p, device=0)
    T = []
    for k in range(60):
        t0 = time.perf_counter()
        ctx.scan_registration(len(frames[k]), device_ptr=d[k].data_ptr())
        od = ctx.odometry()
        t1 = time.perf_counter()
        ctx.mapping()
        t2 = time.perf_counter()
        if k >= 10:
            T.append((t1 - t0, t2 - t1))
    ctx.close()
    T = np.median(np.array(T), 0) * 1e3
    print(f"{label:40s} serial front {T[0]:.3f} ms  map {T[1]:.3f} ms", flush=True)


for lab, kw in [("default", {}), ("map_rounds=0", dict(map_rounds=0)), ("odom_rounds=0", dict(odom_rounds=0)),
                ("both 0", dict(map_rounds=0, odom_rounds=0))]:
    serial(lab, **kw)
    pipe_rate(lab, **kw)
