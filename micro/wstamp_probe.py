"""Profiling probe (not a test): per-wave phase stamps of the last launch of one kernel, from a library
built with -DALOAM_WSTAMP_MAP (k_map_assoc) or -DALOAM_WSTAMP_ODOM (k_odom_search):
  micro/build_flags.sh libaloam_ws_map "-DALOAM_WSTAMP_MAP"; python micro/wstamp_probe.py map
Serial frames (no pipeline), so the last launch ran alone on the GPU. Prints, over the waves that ran
a query, percentiles of each phase (us) and of the start / end offsets from the first wave's start."""
import ctypes as C
import os
import sys

import numpy as np

which = sys.argv[1] if len(sys.argv) > 1 else "map"
os.environ["ALOAM_LIB_PATH"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"libaloam_ws_{which}.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

ctx = lvo.Context(lvo.abi.default_params(64))
for k in range(8):
    ctx.process_scan(lvo.synth.scan("hdl64", k), mapping=(which == "map"))
ts = np.zeros(8192 * 8, np.uint64)
lvo.lib().aloam_dbg_wstamps(ts.ctypes.data_as(C.c_void_p))
t = ts.reshape(8192, 8).astype(np.float64)
live = (t[:, 0] > 0) & (t[:, 3] > 0)
t0 = t[t[:, 0] > 0, 0].min()
names = {"map": ["entry", "params", "query", "knn", "fit", "exit"], "odom": ["entry", "counts", "query", "nn", "window", "exit"]}[which]
print(f"waves with stamps {int((t[:, 0] > 0).sum())}, with a query {int(live.sum())}")
L = t[live]
def pc(v):
    return " ".join(f"{np.percentile(v, q) / 100:7.2f}" for q in (0, 50, 90, 99, 100))
print("phase              p0      p50     p90     p99     max   (us)")
for k in range(1, 6):
    if (L[:, k] > 0).all() and (L[:, k - 1] > 0).all():
        print(f"{names[k - 1]:>7}->{names[k]:<7} {pc(L[:, k] - L[:, k - 1])}")
if which == "map":
    F = L[(L[:, 6] > 0) & (L[:, 7] > 0)]
    print(f"fit: knn->pts     {pc(F[:, 6] - F[:, 3])}")
    print(f"fit: pts->solved  {pc(F[:, 7] - F[:, 6])}")
print(f"start offset     {pc(L[:, 0] - t0)}")
print(f"end offset       {pc(L[:, 5] - t0)}")
