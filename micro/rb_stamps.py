"""Phase stamps of the per-cube map filter (k_rb_cubevox, profiling build -DALOAM_WSTAMP_RB): a serial context
runs N HDL-64 frames; after each frame the stamp table gives, per surrounding cube and kind, the wall-clock
(100 MHz) at: 0 start, 1 keys, 3 order-free sort (R2), 2 relevance marks, 4 exact replay (LDS cubes),
5 leaf sums, 6 split (big cubes with relevant leaves; their segment sorts run in k_rb_cubeseg). Prints the
per-frame slowest cube's phases and means by path. Profiling aid only.

usage: ALOAM_LIB_PATH=micro/_var_rbst/libaloam_hip.so python micro/rb_stamps.py [frames]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import abi, lvo, synth  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 120
L = lvo.lib()
L.aloam_dbg_wstamps.argtypes = [C.c_void_p]
ctx = lvo.Context(abi.default_params(64))
tab = np.zeros((8192, 8), np.uint64)
rows = []
for k in range(frames):
    ctx.process_scan(synth.scan("hdl64", k))
    L.aloam_dbg_wstamps(tab.ctypes.data)
    t = tab[:256].astype(np.int64)
    live = t[:, 0] > 0
    if not live.any():
        continue
    t0max = t[live, 0].max()
    live &= t[:, 0] > t0max - 100000           # this frame's cubes (1 ms window)
    for r in np.nonzero(live)[0]:
        s = t[r]
        n = int(s[7] & 0xffffffff)
        fits = int((s[7] >> 32) & 0xff)
        nnew = int(s[7] >> 40)
        d = lambda a, b: (s[b] - s[a]) / 100.0 if s[b] >= s[a] > 0 and s[b] > t0max - 100000 else float("nan")
        end = max(v for v in s[:7] if v > t0max - 100000)
        rows.append(dict(frame=k, kind=int(r >= 128), n=n, fits=fits, nnew=nnew, total=(end - s[0]) / 100.0,
                         keys=d(0, 1), r2=d(1, 3), mark=d(3, 2), replay=d(2, 4), reduce_fit=d(4, 5),
                         reduce_big=d(2, 5), split=d(2, 6)))
import collections
late = [r for r in rows if r["frame"] >= frames // 2]
print(f"{len(late)} cube filters in frames {frames // 2}..{frames - 1}")
byf = collections.defaultdict(list)
for r in late:
    byf[r["frame"]].append(r)
worst = [max(v, key=lambda r: r["total"]) for v in byf.values()]
print("slowest cube per frame: mean total %.1f us, max %.1f us" % (np.mean([w["total"] for w in worst]), max(w["total"] for w in worst)))
for key in ("fits", "big"):
    sel = [r for r in late if (r["fits"] == 1) == (key == "fits") and r["nnew"] > 0]
    if not sel:
        continue
    m = lambda f: np.nanmean([r[f] for r in sel])
    print(f"{key}: {len(sel)} touched cubes, n mean {np.mean([r['n'] for r in sel]):.0f}, total {m('total'):.1f} us | keys {m('keys'):.1f} "
          f"R2 {m('r2'):.1f} mark {m('mark'):.1f} replay {m('replay'):.1f} reduce(fit) {m('reduce_fit'):.1f} "
          f"reduce(big) {m('reduce_big'):.1f} split {m('split'):.1f}")
for w in sorted(worst, key=lambda r: -r["total"])[:5]:
    print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in w.items()})
