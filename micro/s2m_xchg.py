"""C4 registration through aloam_s2m_register_group at W = 2, 4, 8 contexts sharing one GPU, with the
exchange the process was started with: host-ordered peer copies (default) or the device exchange
(ALOAM_S2M_PEER=1, one persistent Solve per rank). Wall time per registration; every rank's pose is
checked bit-identical to the single-context registration. Usage: python micro/s2m_xchg.py LABEL"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lvo_amd_loader import lvo  # noqa: E402

dev = torch.device("cuda", 0)
cm, sm, cq, sq, x0, _ = lvo.synth.c4_registration()
dm, dcq, dsq = (torch.from_numpy(a).to(dev) for a in (cm, cq, sq))


def ctx():
    p = lvo.abi.default_params(128)
    p.max_scan_points, p.max_map_points = 1024, 1024
    c = lvo.Context(p)
    c.s2m_set_map(dm.data_ptr(), dm.data_ptr(), len(cm), len(sm))
    c.s2m_set_queries(dcq.data_ptr(), dsq.data_ptr(), len(cq), len(sq))
    return c


c1 = ctx()
ref = c1.s2m_register(x0)
out = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "peer": os.environ.get("ALOAM_S2M_PEER", "0")}
for world in (2, 4, 8):
    ctxs = [ctx() for _ in range(world)]
    for _ in range(2):
        res = lvo.s2m_register_group(ctxs, x0)
    assert all(np.array_equal(r["x"].view(np.uint64), ref["x"].view(np.uint64)) for r in res)
    n = 10
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        lvo.s2m_register_group(ctxs, x0)
    torch.cuda.synchronize()
    out[f"W{world}_ms"] = round((time.perf_counter() - t) / n * 1e3, 3)
    print(world, out[f"W{world}_ms"], "ms per registration", flush=True)
    for c in ctxs:
        c.close()
print(json.dumps(out))
