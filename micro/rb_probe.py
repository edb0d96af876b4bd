"""Profiling probe (not a test): k_rb_cubevox phase stamps per cube of the last launch (lib built with
-DALOAM_WSTAMP_RB: micro/build_flags.sh libaloam_rb "-DALOAM_WSTAMP_RB"). The last launch is the surf lane."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["ALOAM_LIB_PATH"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libaloam_rb.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

os.environ["ALOAM_NO_GRAPHS"] = "1"
ctx = lvo.Context(lvo.abi.default_params(64))
for f in lvo.synth.sequence("hdl64", int(sys.argv[1]) if len(sys.argv) > 1 else 60, start=0):
    ctx.process_scan(f)
ts = np.zeros(8192 * 8, np.uint64)
lvo.lib().aloam_dbg_wstamps(ts.ctypes.data_as(C.c_void_p))
info = np.zeros((256, 4), np.int32)
lvo.lib().aloam_dbg_rb_info(info.ctypes.data_as(C.c_void_p))
t = ts.reshape(8192, 8)[:256].astype(np.float64)
print("cube     n   n_old unsorted | bbox   keys+chk sortnew  merge  centroids  total (us)  [cent: loads+scan heads walk]")
for b in range(256):
    if t[b, 0] == 0 or t[b, 5] == 0:
        continue
    d = lambda i, j: (t[b, j] - t[b, i]) / 100 if t[b, i] > 0 and t[b, j] > 0 else float("nan")
    print(("C" if b < 128 else "S") + f"{info[b,0]:5d} {info[b,1]:6d} {info[b,2]:6d} {info[b,3]:3d} | {d(0,1):6.2f} {d(1,2):7.2f} {d(2,3):7.2f} {d(3,4):7.2f} {d(4,5):9.2f} {d(0,5):7.2f}   {d(4,7):6.2f} {d(7,6):6.2f} {d(6,5):6.2f}")
