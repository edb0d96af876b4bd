"""C4 search A/B in one process: the bench's C4 workload (128-line sweep vs the 2.09M-point map), the index
built once, then each variant's search (env knobs read per call) timed over N launches with HIP events
(Context timing), outputs compared bit for bit with the first variant's.

usage: python micro/c4_exp.py [launches] [VAR=VAL,VAR=VAL ...] ...   (each argument after the count = one variant)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402
from lvo_amd_loader import lvo  # noqa: E402

n_launch = int(sys.argv[1]) if len(sys.argv) > 1 else 20
variants = sys.argv[2:] or ["ALOAM_KNN_P2=0", "ALOAM_KNN_P2=1"]
synth = lvo.synth
m = synth.dense_map(4, 0.0, 0.0, step=0.107)
R, o = synth.pose("l128", 0)
s = synth.scan("l128", 0)
q = s.copy()
q[:, :3] = (s[:, :3].astype(np.float64) @ R.T + o).astype(np.float32)
dm, dq = torch.from_numpy(m).cuda(), torch.from_numpy(q).cuda()
ctx = lvo.Context(lvo.abi.default_params(128))
ctx.set_profiling(True)
bt = []
for _ in range(3):
    ctx.knn_build(dm.data_ptr(), len(m), 1.0)
    bt.append(ctx.timing()["knn_build_ms"] * 1e3)
print(f"map {len(m)} queries {len(q)} build us {bt}", flush=True)
ref = None
for v in variants:
    env = dict(kv.split("=", 1) for kv in v.split(",") if kv)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    rebuild = any(k_ in env for k_ in ("ALOAM_KNN_FINE", "ALOAM_GRID_RADIX"))
    if rebuild:                                      # build parameters: rebuild, report the build time
        bts = []
        for _ in range(3):
            ctx.knn_build(dm.data_ptr(), len(m), 1.0)
            bts.append(ctx.timing()["knn_build_ms"] * 1e3)
        print(f"  build with {v}: {[round(b_, 1) for b_ in bts]} us", flush=True)
    idx = torch.full((len(q), 5), -7, dtype=torch.int32, device="cuda")
    d2 = torch.full((len(q), 5), -7.0, dtype=torch.float32, device="cuda")
    us, by = [], []
    for it in range(n_launch + 2):
        ctx.knn_query(dq.data_ptr(), len(q), 5, idx.data_ptr(), d2.data_ptr())
        t = ctx.timing()
        if it >= 2:
            us.append(t["knn_ms"] * 1e3)
            by.append(t["knn_streamed_bytes"])
    out = (idx.cpu().numpy(), d2.cpu().numpy().view(np.uint32))
    same = None if ref is None else bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
    if ref is None:
        ref = out
    b = float(np.mean(by))
    print(f"{v:40s} {ctx.knn_kernel():28s} mean {np.mean(us):8.2f} us  median {np.median(us):8.2f}  min {np.min(us):8.2f}"
          f"  frac {b / (np.mean(us) * 1e-6) / 16.8e12:.4f}  same_as_first {same}", flush=True)
    for k_, v_ in old.items():
        if v_ is None:
            os.environ.pop(k_, None)
        else:
            os.environ[k_] = v_
    if "ALOAM_KNN_FINE" in env:
        ctx.knn_build(dm.data_ptr(), len(m), 1.0)
ctx.close()
