"""Device exchange in group mode (ALOAM_S2M_PEER=1): W ranks on one GPU, one call, results vs the
single-context registration; prints the counters on a timeout (ALOAM_S2M_PEER_DEBUG)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
from lvo_amd_loader import lvo  # noqa: E402
import test_s2m as T  # noqa: E402

wl = T.small_workload()
x0 = wl[4]
cm, sm, cq, sq, _, _ = wl
p = lvo.abi.default_params(128)
p.max_scan_points, p.max_map_points = max(len(cq) + len(sq), 1024), 1024


def ctx():
    c = lvo.Context(p)
    c.s2m_set_map(cm, sm)
    c.s2m_set_queries(cq, sq)
    return c


g = ctx().s2m_register(x0)
for world in [int(w) for w in sys.argv[1:]] or [2]:
    ctxs = [ctx() for _ in range(world)]
    for call in range(3):
        t0 = time.time()
        try:
            res = lvo.s2m_register_group(ctxs, x0)
            same = all(np.array_equal(g["x"].view(np.uint64), r["x"].view(np.uint64)) for r in res)
            print("world", world, "call", call, "ok" if same else "DIFF", f"{(time.time() - t0) * 1e3:.1f} ms", flush=True)
        except lvo.ALOAMError as e:
            print("world", world, "call", call, "error", e, f"{(time.time() - t0) * 1e3:.1f} ms", flush=True)
    del ctxs
