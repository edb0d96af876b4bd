"""Phase stamps of one mapping registration round's association (k_map_assoc, profiling build
-DALOAM_WSTAMP_MAP=<round>): a serial context runs N HDL-64 frames; after each frame the stamp table holds,
per wave of that round's launch, the wall clock (100 MHz) at 0 start, 1 pose loaded, 2 query + cache test,
6 grid searches done (round 0: all; later rounds: the queries that left their cache, a wave each),
3 cached-list k-NN done, 7 fit done (only waves that fitted), 4 factors written, 5 end. Profiling aid only.

usage: ALOAM_LIB_PATH=micro/_var_ast3/libaloam_hip.so python micro/assoc_stamps.py [frames]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import abi, lvo, synth  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 60
L = lvo.lib()
L.aloam_dbg_wstamps.argtypes = [C.c_void_p]
ctx = lvo.Context(abi.default_params(64))
tab = np.zeros((8192, 8), np.uint64)
spans, ph = [], {k: [] for k in ("pose", "query", "search", "list", "fit", "post", "end")}
nsearch, nfit, nw = [], [], []
for k in range(frames):
    ctx.process_scan(synth.scan("hdl64", k))
    L.aloam_dbg_wstamps(tab.ctypes.data)
    t = tab.astype(np.int64)
    live = t[:, 0] > 0
    if not live.any() or k < frames // 2:
        continue
    live &= t[:, 0] > t[live, 0].max() - 100000
    w = t[live]
    # a slot counts only if this launch wrote it: not before the wave's start stamp and within the launch's
    # window (slots a wave skips keep an earlier frame's value, which the round-4 version mixed in)
    t0 = w[:, 0:1]
    cur = (w >= t0) & (w <= w[:, 0].max() + 100000)
    spans.append((np.where(cur[:, 5], w[:, 5], 0).max() - w[:, 0].min()) / 100.0)
    act = cur[:, 4]
    nw.append(int(act.sum()))

    def d(a, b):
        ok = act & cur[:, a] & cur[:, b] & (w[:, b] >= w[:, a])
        return (w[ok, b] - w[ok, a]) / 100.0

    v = d(0, 1)
    ph["pose"].append(v.max() if len(v) else 0)
    for name, a, b in (("query", 1, 2), ("search", 2, 6), ("list", 6, 3), ("post", 3, 4), ("end", 4, 5)):
        v = d(a, b)
        ph[name].append((v.mean(), v.max()) if len(v) else (0, 0))
    v = d(3, 7)
    v = v[v > 0]                                  # waves that fitted
    nfit.append(len(v))
    ph["fit"].append((v.mean(), v.max()) if len(v) else (0, 0))
    nsearch.append(int((d(2, 6) > 1.0).sum()))
print(f"frames {frames // 2}..{frames - 1}: launch span mean {np.mean(spans):.1f} us max {np.max(spans):.1f}; active waves {np.mean(nw):.0f}, "
      f"waves with a grid search > 1 us {np.mean(nsearch):.1f}, waves fitting {np.mean(nfit):.0f}")
for name in ("query", "search", "list", "fit", "post", "end"):
    v = np.array(ph[name])
    print(f"  {name:7s} mean over waves {v[:, 0].mean():6.2f} us   slowest wave {v[:, 1].mean():6.2f} us (max {v[:, 1].max():.2f})")
