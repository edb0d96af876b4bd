"""Profiling probe (not a test): C4 mapping-search workload — 128-line sweep (~233k queries) against a
~2M-point dense local map, radius-1 5-NN through aloam_knn_device."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo, synth  # noqa: E402

step = float(os.environ.get("C4_STEP", "0.107"))
m = synth.dense_map(4, 0.0, 0.0, step=step)
R, o = synth.pose("l128", 0)
s = synth.scan("l128", 0)
q = s.copy()
q[:, :3] = (s[:, :3].astype(np.float64) @ R.T + o).astype(np.float32)
dm, dq = torch.from_numpy(m).cuda(), torch.from_numpy(q).cuda()
idx = torch.empty((len(q), 5), dtype=torch.int32, device="cuda")
d2 = torch.empty((len(q), 5), dtype=torch.float32, device="cuda")
ctx = lvo.Context(lvo.abi.default_params(128))
ctx.set_profiling(True)
ts = []
for it in range(12):
    ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr(), len(q), 5, 1.0, idx.data_ptr(), d2.data_ptr())
    t = ctx.timing()
    ts.append((t["knn_ms"], t["knn_bytes"]))
ms = np.median([a for a, _ in ts[2:]])
b = ts[-1][1]
found = (idx[:, 4] >= 0).float().mean().item()
print(f"GS={os.environ.get('ALOAM_KNN_GS', '8')} map={len(m)} q={len(q)} kernel {ms*1000:.1f} us, alg bytes {b/1e9:.3f} GB "
      f"-> {b/(ms*1e-3)/1e9:.0f} GB/s ({b/(ms*1e-3)/8e12*100:.1f}% of 8 TB/s); cand/q {(b/len(q)-56)/16:.0f}; 5 found {found:.3f}")
if os.environ.get("C4_CHECK"):
    import oracle_binding as ob
    rng = np.random.default_rng(0)
    sel = rng.choice(len(q), 2000, replace=False)
    t = time.time()
    oi, od = ob.knn(m, q[sel], 5, 1.0)
    gi = idx.cpu().numpy()[sel]
    bad = np.where((gi != oi).any(axis=1))[0]
    print(f"oracle check ({time.time()-t:.1f}s): {len(bad)} / {len(sel)} queries differ; oracle 5-found {(oi[:, 4] >= 0).mean():.3f}")
    if len(bad):
        b = bad[0]
        print("gpu", gi[b], "oracle", oi[b], "d2 gpu", d2.cpu().numpy()[sel][b], "oracle", od[b])
