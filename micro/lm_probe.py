"""Profiling probe (not a test): block-0 phase stamps of the last LM launch (build micro/libaloam_lmt.so
with -DALOAM_LM_TIMING). Runs odometry-only frames so the last launch is an odometry Solve."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["ALOAM_LIB_PATH"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libaloam_lmt.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

ctx = lvo.Context(lvo.abi.default_params(64))
for k in range(6):
    ctx.process_scan(lvo.synth.scan("hdl64", k), mapping=(sys.argv[1:] == ["map"]))
ts = np.zeros(48, np.uint64)
lvo.lib().aloam_dbg_lm_ts(ts.ctypes.data_as(C.c_void_p))
t = ts[:40].reshape(8, 5).astype(np.float64)
e0, e1 = float(ts[40]), float(ts[41])
print("stamps (us from kernel entry): pass: accumulated, block-reduced, gathered, reduced, tail-done")
for p in range(5):
    print(p, " ".join(f"{(t[p, k] - e0) / 100:7.2f}" for k in (4, 0, 1, 2, 3)))
print("exit", (e1 - e0) / 100)

ns = np.zeros(4, np.uint64)
lvo.lib().aloam_dbg_ns_ts(ns.ctypes.data_as(C.c_void_p))
n = ns.astype(np.float64)
print("last next_step: chol %.2f us, step->plus7 %.2f us, plus7+norm %.2f us" % ((n[1] - n[0]) / 100, (n[2] - n[1]) / 100, (n[3] - n[2]) / 100))
