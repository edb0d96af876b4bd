"""C4 registration at a rank's share (W = 1, 2, 4, 8 in-process contexts on one GPU, aloam_s2m_register_group):
wall time per group registration with the association's split 5-NN / fit kernels forced for every slot count
(ALOAM_S2M_BATCH_MIN=1) against the default threshold (65536: a rank's share below it runs the fused latency
kernel). Same results either way (tests/test_s2m.py::test_s2m_assoc_paths_bit_identical)."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
from lvo_amd_loader import lvo

dev = torch.device("cuda", 0)
cm, sm, cq, sq, x0, _ = lvo.synth.c4_registration()
dm, dcq, dsq = (torch.from_numpy(a).to(dev) for a in (cm, cq, sq))
out = {}
for world in (1, 2, 4, 8):
    ctxs = []
    for _ in range(world):
        p = lvo.abi.default_params(64)
        p.max_scan_points, p.max_map_points = 1024, 1024
        c = lvo.Context(p)
        c.s2m_set_map(dm.data_ptr(), dm.data_ptr(), len(cm), len(sm))
        c.s2m_set_queries(dcq.data_ptr(), dsq.data_ptr(), len(cq), len(sq))
        ctxs.append(c)
    for bm in ("65536", "1"):
        os.environ["ALOAM_S2M_BATCH_MIN"] = bm
        run = (lambda: ctxs[0].s2m_register(x0)) if world == 1 else (lambda: lvo.s2m_register_group(ctxs, x0))
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = 8
        for _ in range(n):
            r = run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / n * 1e3
        out[f"W{world}_bm{bm}"] = round(ms, 3)
        print(world, bm, round(ms, 3), "ms per registration", flush=True)
    for c in ctxs:
        c.close()
print(json.dumps(out))
