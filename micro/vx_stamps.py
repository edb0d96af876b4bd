"""Phase stamps of the stack VoxelGrid launch k_vox_pcl (profiling build -DALOAM_PS_TIMING): a serial context runs
N HDL-64 frames; after each frame the stamps (100 MHz) of its last k_vox_pcl launch (the mapping stacks: job 0 the
less-sharp cloud at 0.4 m, sorted in LDS; job 1 the less-flat cloud at 0.8 m, split in global memory) give per job:
bbox, keys, sort (job 0) / split (job 1), and the split's levels (job 1). Profiling aid only.

usage: ALOAM_LIB_PATH=micro/_var_vxts/libaloam_hip.so python micro/vx_stamps.py [frames]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import abi, lvo, synth  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 40
L = lvo.lib()
L.aloam_dbg_vx_ts.argtypes = [C.c_void_p]
L.aloam_dbg_ps_ts.argtypes = [C.c_void_p, C.c_void_p]
ctx = lvo.Context(abi.default_params(64))
vx = np.zeros((2, 8), np.uint64)
ps = np.zeros((64, 6), np.uint64)
nseg = np.zeros(64, np.int32)
rows = []
ph = []   # per split level: count + scan, k, swaps + cuts, children (us)
for k in range(frames):
    ctx.process_scan(synth.scan("hdl64", k))
    L.aloam_dbg_vx_ts(vx.ctypes.data)
    L.aloam_dbg_ps_ts(ps.ctypes.data, nseg.ctypes.data)
    if k < 5:
        continue
    t = vx.astype(np.int64)
    d = lambda j, a, b: (t[j, b] - t[j, a]) / 100.0 if t[j, b] >= t[j, a] > 0 else float("nan")
    lv = []
    p = ps.astype(np.int64)
    for l in range(60):
        if p[l, 0] >= t[1, 2] and p[l, 4] >= p[l, 0]:
            lv.append(((p[l, 4] - p[l, 0]) / 100.0, int(nseg[l])))
            ph.append(np.diff(p[l, :5]) / 100.0)
    rows.append((int(t[0, 7]), d(0, 0, 1), d(0, 1, 2), d(0, 2, 3), d(0, 3, 4), int(t[1, 7]), d(1, 0, 1), d(1, 1, 2), d(1, 2, 3), lv))
for r in rows[-8:]:
    print(f"corner n {r[0]}: bbox {r[1]:.1f} keys {r[2]:.1f} sort {r[3]:.1f} reduce {r[4]:.1f} us | surf n {r[5]}: bbox {r[6]:.1f} "
          f"keys {r[7]:.1f} split {r[8]:.1f} us, levels {[(round(a, 1), b) for a, b in r[9]]}")
a = np.array([r[:9] for r in rows], float)
print("means:", {k: round(float(np.nanmean(a[:, i])), 1) for i, k in enumerate(("n_c", "bbox_c", "keys_c", "sort_c", "reduce_c", "n_s", "bbox_s", "keys_s", "split_s"))})
if ph:
    print("split level phases (mean us): count+scan %.1f, k %.1f, swaps+cuts %.1f, children %.1f" % tuple(np.mean(ph, axis=0)))
