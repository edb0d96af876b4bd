"""Diagnostic: test_knn_build_once_query_many's exact sequence in one context, mismatches printed."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402
import oracle_binding as ob  # noqa: E402
from lvo_amd_loader import lvo  # noqa: E402
synth = lvo.synth
m = synth.dense_map(4, 0.0, 0.0, step=0.25)
R, o = synth.pose("l128", 0)
s = synth.scan("l128", 0)
q = s.copy()
q[:, :3] = (s[:, :3].astype(np.float64) @ R.T + o).astype(np.float32)
for variant in sys.argv[1:] or ["", "ALOAM_GRID_RADIX=0"]:
    for kv in filter(None, variant.split(",")):
        a, b = kv.split("=")
        os.environ[a] = b
    dm, dq = torch.from_numpy(m).cuda(), torch.from_numpy(q).cuda()
    ctx = lvo.Context(lvo.abi.default_params(128))

    def run(fn, k, n_q):
        idx = torch.full((n_q, k), -7, dtype=torch.int32, device="cuda")
        d2 = torch.full((n_q, k), -7.0, dtype=torch.float32, device="cuda")
        fn(idx, d2)
        return idx.cpu().numpy(), d2.cpu().numpy()
    steps = []
    if "nodev" not in variant:
        run(lambda i, d: ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr(), len(q), 5, 1.0, i.data_ptr(), d.data_ptr()), 5, len(q))
        run(lambda i, d: ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr() + 16 * 1000, 5000, 3, 1.0, i.data_ptr(), d.data_ptr()), 3, 5000)
        ctx.knn_build(dm.data_ptr(), len(m), 1.0)
        dm.fill_(1e6)
        run(lambda i, d: ctx.knn_query(dq.data_ptr(), len(q), 5, i.data_ptr(), d.data_ptr()), 5, len(q))
    m2 = m[::2].copy()
    m2[:, 0] += 0.05
    dm2 = torch.from_numpy(m2).cuda()
    ctx.knn_build(dm2.data_ptr(), len(m2), 1.0)
    gi, gd = run(lambda i, d: ctx.knn_query(dq.data_ptr(), len(q), 5, i.data_ptr(), d.data_ptr()), 5, len(q))
    sel = np.random.default_rng(3).choice(len(q), 2000, replace=False)
    oi, od = ob.knn(m2, q[sel], 5, 1.0)
    bad_i = np.argwhere(gi[sel] != oi)
    ok = oi >= 0
    bad_d = np.argwhere(ok & (gd[sel].view(np.uint32) != od.view(np.uint32)))
    print(variant or "default", ctx.knn_kernel(), "idx mismatches", len(bad_i), "d2 mismatches", len(bad_d), flush=True)
    for r, c in list(bad_d[:6]) + list(bad_i[:4]):
        j = sel[r]
        pi = gi[j, c]
        print("   q", j, "slot", c, "gpu idx", pi, "oracle idx", oi[r, c], "gpu d2", gd[j, c], "oracle d2", od[r, c],
              "m2[idx]", m2[pi, :3] if 0 <= pi < len(m2) else None, "m[idx]", m[pi, :3] if 0 <= pi < len(m) else None, "q", q[j, :3], flush=True)
    ctx.close()
    for kv in filter(None, variant.split(",")):
        os.environ.pop(kv.split("=")[0], None)
