"""Per-line phase times of k_line_features (micro/_var_lft build, ALOAM_LF_TIMING): LF_TS stamps 0-7."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from lvo_amd_loader import lvo
L = C.CDLL(lvo.LIB_PATH)
ctx = lvo.Context(lvo.abi.default_params(64), device=0)
frames = lvo.synth.sequence("hdl64", 3, start=0)
acc = np.zeros((64, 7)); n = 0
for it in range(6):
    ctx.scan_registration(frames[it % 3])
    ts = np.zeros((64, 8), np.uint64)
    L.aloam_dbg_lf_ts(ts.ctypes.data_as(C.c_void_p))
    if it >= 1:
        acc += np.diff(ts.astype(np.int64), axis=1) / 100.0; n += 1
acc /= n
names = ["setup", "greedy", "cand", "bbox+keys", "sort", "heads", "centroids"]
print("us per phase, mean / max over lines:", ", ".join(f"{nm} {acc[:, i].mean():.1f}/{acc[:, i].max():.1f}" for i, nm in enumerate(names)))
f = ctx.features()
print("less_flat", len(f["less_flat"]))
