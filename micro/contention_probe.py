"""Profiling aid (not part of the product): is the pipeline's per-stage stretch host-side (two threads
of one process launching into one HIP runtime) or device-side? Each worker runs 60 serial frames on a
context restricted to its own half of the CUs: alone, as two threads of one process, and as two
processes."""
import ctypes as C
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def run(half, out, key, barrier=None):
    import torch
    from lvo_amd_loader import lvo
    frames = lvo.synth.sequence("hdl64", 70, start=1000 * half)
    d = [torch.from_numpy(f).to("cuda:0") for f in frames]
    torch.cuda.synchronize()
    ctx = lvo.Context(lvo.abi.default_params(64), device=0)
    mask = (C.c_uint * 8)(*([0xFFFFFFFF] * 4 + [0] * 4 if half == 0 else [0] * 4 + [0xFFFFFFFF] * 4))
    assert lvo.lib().aloam_set_cu_mask(ctx.h, mask, 8) == 0
    for k in range(10):
        ctx.process_scan(device_ptr=d[k].data_ptr(), n=len(frames[k]))
    if barrier is not None:
        barrier.wait()
    t0 = time.perf_counter()
    for k in range(10, 70):
        ctx.process_scan(device_ptr=d[k].data_ptr(), n=len(frames[k]))
    out[key] = (time.perf_counter() - t0) / 60 * 1e3
    ctx.close()


def proc_main(half, q, barrier):
    out = {}
    run(half, out, half, barrier)
    q.put(out[half])


if __name__ == "__main__":
    out = {}
    run(0, out, "alone")
    print(f"alone (CUs 0-127):        {out['alone']:.3f} ms/scan", flush=True)
    b = threading.Barrier(2)
    ts = [threading.Thread(target=run, args=(h, out, f"thr{h}", b)) for h in (0, 1)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    print(f"two threads, one process: {out['thr0']:.3f} / {out['thr1']:.3f} ms/scan", flush=True)
    import multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    pb = ctxm.Barrier(2)
    ps = [ctxm.Process(target=proc_main, args=(h, q, pb)) for h in (0, 1)]
    [p.start() for p in ps]
    r = [q.get(timeout=300) for _ in ps]
    [p.join() for p in ps]
    print(f"two processes:            {r[0]:.3f} / {r[1]:.3f} ms/scan", flush=True)
