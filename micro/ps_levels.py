"""Per-level phase times of the PCL-order sort (micro/_var_pst build, ALOAM_PS_TIMING) on one cloud."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from lvo_amd_loader import lvo
L = C.CDLL(lvo.LIB_PATH)
ctx = lvo.Context(lvo.abi.default_params(64), device=0)
pts = lvo.synth.scan("hdl64", 3)
for n in [int(a) for a in sys.argv[1:]] or [2000]:
    for _ in range(3):
        ctx.voxel_grid(pts[:n], 0.8)
    w = np.zeros((16, 8), np.uint64)
    L.aloam_dbg_ps_w(w.ctypes.data_as(C.c_void_p))
    ctx.voxel_grid(pts[:n], 0.8)
    L.aloam_dbg_ps_w(w.ctypes.data_as(C.c_void_p))
    print(f"n={n}: per wave (cycles): wait / partition (#, elems) / leaf (#)")
    for i in range(16):
        r = [int(x) for x in w[i]]
        print(f"  w{i:2d}: wait {r[0]:8d}  part {r[1]:8d} ({r[2]:4d}, {r[3]:6d})  leaf {r[4]:7d} ({r[5]:4d})"
              f"  cyc/part {r[1] / max(r[2], 1):7.0f}  cyc/leaf {r[4] / max(r[5], 1):6.0f}")
    ts = np.zeros((64, 6), np.uint64); ns = np.zeros(64, np.int32)
    L.aloam_dbg_ps_ts(ts.ctypes.data_as(C.c_void_p), ns.ctypes.data_as(C.c_void_p))
    print(f"n={n}: wave phase {(int(ts[60, 1]) - int(ts[60, 0])) / 100.0:.2f} us, {ns[60]} segments queued")
    for l in range(60):
        if ts[l, 0] == 0: break
        if ns[l] == 0:
            print(f"  level {l}: done"); break
        d = [(int(ts[l, k + 1]) - int(ts[l, k])) / 100.0 for k in range(4)]
        nxt = (int(ts[l + 1, 0]) - int(ts[l, 4])) / 100.0 if l + 1 < 64 and ts[l + 1, 0] else float('nan')
        print(f"  level {l:2d} nseg {ns[l]:5d}: median {d[0]:6.2f}  stops {d[1]:6.2f}  k/cut {d[2]:6.2f}  swaps {d[3]:6.2f}  children {nxt:6.2f} us")
