"""Diagnostic: the build-once test scenario, mismatches vs the oracle printed (GPU box)."""
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
dq = torch.from_numpy(q).cuda()
for variant in sys.argv[1:] or ["", "ALOAM_GRID_RADIX=0", "ALOAM_KNN_KEYS=0"]:
    for kv in filter(None, variant.split(",")):
        a, b = kv.split("=")
        os.environ[a] = b
    for mm, name in ((m, "m"), (m[::2].copy(), "m2")):
        if name == "m2":
            mm[:, 0] += 0.05
        ctx = lvo.Context(lvo.abi.default_params(128))
        dm = torch.from_numpy(mm).cuda()
        idx = torch.full((len(q), 5), -7, dtype=torch.int32, device="cuda")
        d2 = torch.full((len(q), 5), -7.0, dtype=torch.float32, device="cuda")
        ctx.knn_device(dm.data_ptr(), len(mm), dq.data_ptr(), len(q), 5, 1.0, idx.data_ptr(), d2.data_ptr())
        gi, gd = idx.cpu().numpy(), d2.cpu().numpy()
        sel = np.random.default_rng(3).choice(len(q), 2000, replace=False)
        oi, od = ob.knn(mm, q[sel], 5, 1.0)
        bad_i = np.argwhere(gi[sel] != oi)
        ok = oi >= 0
        bad_d = np.argwhere(ok & (gd[sel].view(np.uint32) != od.view(np.uint32)))
        print(variant or "default", name, len(mm), ctx.knn_kernel(), "idx mismatches", len(bad_i), "d2 mismatches", len(bad_d), flush=True)
        for r, c in bad_d[:5]:
            j = sel[r]
            pi = gi[j, c]
            p = mm[pi, :3].astype(np.float32)
            qq = q[j, :3]
            dd = np.float32(np.float32((p[0] - qq[0]) ** 2 + (p[1] - qq[1]) ** 2) + (p[2] - qq[2]) ** 2)
            print("   q", j, "slot", c, "idx", pi, "gpu", gd[j, c], "oracle", od[r, c], "host recompute", dd, flush=True)
        ctx.close()
    for kv in filter(None, variant.split(",")):
        os.environ.pop(kv.split("=")[0], None)
