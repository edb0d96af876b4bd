"""Profiling probe (not a test): per-cube map sizes after N frames of the bench's C3 sequence."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 60
ctx = lvo.Context(lvo.abi.default_params(64))
for k, f in enumerate(lvo.synth.sequence("hdl64", N, start=0)):
    ctx.process_scan(f)
    if k + 1 in (5, 20, N):
        for w, name in ((0, "corner"), (1, "surf")):
            cnt = np.zeros(21 * 21 * 11, np.int32)
            val = np.zeros(21 * 21 * 11, np.int32)
            lvo.lib().aloam_dbg_cube_counts(C.c_void_p(ctx.h), w, cnt.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p))
            v = cnt[val > 0]
            print(f"frame {k + 1} {name}: total {cnt.sum()}, nonempty cubes {(cnt > 0).sum()}, valid cubes {int((val > 0).sum())}, "
                  f"valid sizes max {v.max() if len(v) else 0} p90 {np.percentile(v[v > 0], 90) if (v > 0).any() else 0:.0f} "
                  f"sum {v.sum()}, nonvalid nonempty {int(((cnt > 0) & (val == 0)).sum())}")
