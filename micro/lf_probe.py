"""Profiling probe (not a test): k_line_features phase timing (build micro/libaloam_lf.so with -DALOAM_LF_TIMING)."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["ALOAM_LIB_PATH"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get("LF_LIB", "libaloam_lf.so"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

ctx = lvo.Context(lvo.abi.default_params(64))
pts = lvo.synth.scan("hdl64", 7)
for _ in range(3):
    ctx.scan_registration(pts)
ts = np.zeros((64, 8), np.uint64)
lvo.lib().aloam_dbg_lf_ts(ts.ctypes.data_as(C.c_void_p))
d = np.diff(ts[:51].astype(np.float64), axis=1) / 100.0   # 100 MHz -> us
names = ["sort", "greedy", "lessflat", "vox-keys", "bitonic", "runs", "centroid"]
for i, n in enumerate(names):
    print(f"{n:9s} mean {d[:, i].mean():7.2f} us  max {d[:, i].max():7.2f}")
print("total per block: mean %.1f max %.1f us; block start spread %.1f us" % (
    (ts[:51, 7] - ts[:51, 0]).astype(float).mean() / 100, (ts[:51, 7] - ts[:51, 0]).astype(float).max() / 100,
    (ts[:51, 0].max() - ts[:51, 0].min()) / 100.0))

ts2 = np.zeros((64, 16), np.uint64)
lvo.lib().aloam_dbg_lf_ts2(ts2.ctypes.data_as(C.c_void_p))
g0 = ts[:51, 1].astype(np.float64)
seg = np.diff(np.concatenate([g0[:, None], ts2[:51, :13].astype(np.float64)], axis=1), axis=1) / 100.0
print("greedy per segment (corner, flat) us:", " ".join(f"{seg[:, i].mean():.1f}" for i in range(12)), "| tail", f"{seg[:, 12].mean():.1f}")

cnt = np.zeros((64, 12), np.int32)
if hasattr(lvo.lib(), "aloam_dbg_lf_cnt"):
    lvo.lib().aloam_dbg_lf_cnt(cnt.ctypes.data_as(C.c_void_p))
    print("corner chunks per segment:", cnt[:51, 0::2].mean(0), " pick-loop trips:", cnt[:51, 1::2].mean(0))
import hashlib
h = hashlib.sha1()
for a in ctx.features():
    h.update(np.ascontiguousarray(a).tobytes())
print("features sha1", h.hexdigest()[:16])
ts3 = np.zeros((64, 8), np.uint64)
if hasattr(lvo.lib(), "aloam_dbg_lf_ts3"):
    lvo.lib().aloam_dbg_lf_ts3(ts3.ctypes.data_as(C.c_void_p))
    t0 = ts[:51, 0].astype(np.float64)
    names3 = ["gapbits", "keys", "bitonic", "S+ties", "tie-redo"]
    prev = t0
    for i, n in enumerate(names3):
        cur = ts3[:51, i].astype(np.float64)
        if i == 4:
            has = cur > ts3[:51, 3]
            print(f"  {n:9s} lines with ties {has.sum()}  mean {((cur - ts3[:51, 3]) * has).sum() / max(has.sum(), 1) / 100:.2f} us")
            break
        print(f"  {n:9s} mean {(cur - prev).mean() / 100:7.2f} us")
        prev = cur
