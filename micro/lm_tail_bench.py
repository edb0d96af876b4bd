"""Cycles (s_memtime) of the LM tail (micro/lm_tail_bench.hip) on a random 6x6 normal-equation system."""
import ctypes as C, os
import numpy as np
L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "lm_tail_bench.so"))
rng = np.random.default_rng(7)
J = rng.normal(size=(2000, 6)); r = rng.normal(size=2000) * 0.05
A = J.T @ J; g = J.T @ r
tot = np.zeros(32)
k = 0
for a in range(6):
    for b in range(a, 6):
        tot[k] = A[a, b]; k += 1
tot[21:27] = g; tot[27] = 0.5 * float(r @ r); tot[28] = 2000
x = np.array([0.01, -0.02, 0.03, 0.9993, 1.0, 2.0, 0.5])
x[:4] /= np.linalg.norm(x[:4])
cyc = (C.c_ulonglong * 2)(); out = np.zeros(8)
rc = L.tail_run(tot.ctypes.data_as(C.c_void_p), x.ctypes.data_as(C.c_void_p), cyc, out.ctypes.data_as(C.c_void_p))
print(f"rc {rc}: tail pass 0 {cyc[0]} cycles ({cyc[0] / 2.4e3:.2f} us), accepted pass {cyc[1]} cycles ({cyc[1] / 2.4e3:.2f} us); cand {out[:7]}")
cy = (C.c_ulonglong * 4)(); o = np.zeros(8)
L.parts_run(tot.ctypes.data_as(C.c_void_p), cy, o.ctypes.data_as(C.c_void_p))
print(f"pieces: chol_solve6 {cy[0]}, plus7 {cy[1]}, 3 dependent fp64 divisions {cy[2]}, rsqrt_nr {cy[3]} cycles")
cyr = (C.c_ulonglong * 2)(); outr = np.zeros(8)
rc = L.tail_run_reg(tot.ctypes.data_as(C.c_void_p), x.ctypes.data_as(C.c_void_p), cyr, outr.ctypes.data_as(C.c_void_p))
print(f"state in registers: rc {rc}: tail pass 0 {cyr[0]} cycles ({cyr[0] / 2.4e3:.2f} us), accepted pass {cyr[1]} cycles "
      f"({cyr[1] / 2.4e3:.2f} us); same candidate {bool(np.array_equal(outr[:7], out[:7]))}")
