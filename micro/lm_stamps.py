"""Per-pass phase stamps of one persistent LM solve (k_lm_coop, profiling build -DALOAM_LM_TIMING=<solve>,
solve = odometry round r or ALOAM_MAX_ROUNDS (16) + mapping round r): a serial context runs N HDL-64 frames;
after each frame workgroup 0's stamps (100 MHz) give per pass: eval (slot accumulation), block reduce,
exchange (publish + wait for every workgroup's record), record reduce, LM tail. Profiling aid only.

usage: ALOAM_LIB_PATH=micro/_var_lm16/libaloam_hip.so python micro/lm_stamps.py [frames]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import abi, lvo, synth  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 60
L = lvo.lib()
L.aloam_dbg_lm_ts.argtypes = [C.c_void_p]
ctx = lvo.Context(abi.default_params(64))
buf = np.zeros(42, np.uint64)
rows = []
for k in range(frames):
    buf[:] = 0
    L.aloam_dbg_lm_ts(buf.ctypes.data)   # clear is not possible: keep frames whose entry stamp moved
    ctx.process_scan(synth.scan("hdl64", k))
    b2 = np.zeros(42, np.uint64)
    L.aloam_dbg_lm_ts(b2.ctypes.data)
    if k < frames // 2 or b2[40] == buf[40]:
        continue
    ts = b2[:40].astype(np.int64).reshape(8, 5)
    e0, e1 = int(b2[40]), int(b2[41])
    passes = []
    start = e0
    for p in range(8):
        t = ts[p]
        if not (t[3] >= start and t[4] >= start) or t[3] > e1:
            break
        passes.append([(t[4] - start) / 100, (t[0] - t[4]) / 100, (t[1] - t[0]) / 100, (t[2] - t[1]) / 100, (t[3] - t[2]) / 100])
        start = t[3]
    rows.append(((e1 - e0) / 100, passes))
print(f"{len(rows)} solves; kernel (workgroup 0 entry -> exit) mean {np.mean([r[0] for r in rows]):.2f} us; passes mean {np.mean([len(r[1]) for r in rows]):.2f}")
names = ("eval", "blockred", "exchange", "recred", "tail")
for p in range(8):
    v = [r[1][p] for r in rows if len(r[1]) > p]
    if not v:
        break
    v = np.array(v)
    print(f"  pass {p} ({len(v)} solves): " + "  ".join(f"{n} {m:.2f}" for n, m in zip(names, v.mean(0))))
