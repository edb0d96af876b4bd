"""ls_sort alone (micro/ls_bench.so): one workgroup, n leaf keys of a synthetic scan at 0.2-0.8 m, checked
against libstdc++ std::sort (oracle) and timed (mean of 50 launches)."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import oracle_binding as ob
from lvo_amd_loader import lvo
L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get("LS_SO", "ls_bench.so")))
pts = lvo.synth.scan("hdl64", 3)
for n in [int(a) for a in sys.argv[1:]] or [1300, 2000, 6000, 11000]:
    for leaf in (0.2, 0.8):
        p = pts[:n, :3]
        ix = np.floor(p / leaf).astype(np.int64)
        ix -= ix.min(0)
        d = ix.max(0) + 1
        key = (ix[:, 0] + ix[:, 1] * d[0] + ix[:, 2] * d[0] * d[1]).astype(np.uint64)
        # keys compressed to ranks (< 2^24, exact in float32 for the oracle; same order)
        key = np.unique(key, return_inverse=True)[1].astype(np.uint64)
        E = (key << np.uint64(32)) | np.arange(n, dtype=np.uint64)
        out = np.zeros(n, np.uint64)
        ms = C.c_float(0)
        ph = np.zeros(8, np.uint64)
        L.ls_phases(ph.ctypes.data_as(C.c_void_p))
        wst = np.zeros((16, 8), np.uint64)
        L.ws_stats(wst.ctypes.data_as(C.c_void_p))
        rc = L.ls_run(E.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p), n, 50, C.byref(ms))
        L.ls_phases(ph.ctypes.data_as(C.c_void_p))
        L.ws_stats(wst.ctypes.data_as(C.c_void_p))
        runs = 51
        lv = ph[7] / runs
        print(f"   levels {lv:.1f}; cycles/level A {ph[0]/runs/lv:.0f} B {ph[1]/runs/lv:.0f} C {ph[2]/runs/lv:.0f} D {ph[3]/runs/lv:.0f} E {ph[4]/runs/lv:.0f} next {ph[5]/runs/lv:.0f}; final {ph[6]/runs:.0f}")
        ref = ob.introsort_perm(key.astype(np.float32), libstdcxx=True)
        ok = np.array_equal((out & np.uint64(0xffffffff)).astype(np.int64), ref.astype(np.int64))
        print(f"n {n} leaf {leaf}: rc {rc} {'OK' if ok else 'MISMATCH'} {ms.value * 1e3:.1f} us, distinct {int(key.max()) + 1}", flush=True)
