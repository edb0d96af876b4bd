"""ps_heap_sort (one lane) vs ws_heap_sort (one wave) on one LDS segment: identical output, cycles per pop."""
import ctypes as C, os, sys
import numpy as np
L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "heap_bench.so"))
rng = np.random.default_rng(3)
for n in [int(a) for a in sys.argv[1:]] or [64, 300, 1000, 3000]:
    for kinds in (n // 3, n * 4):
        key = rng.integers(0, kinds, n).astype(np.uint64)
        E = (key << np.uint64(32)) | np.arange(n, dtype=np.uint64)
        outs, cyc = [], []
        for mode in (0, 1):
            o = np.zeros(n, np.uint64); c = C.c_ulonglong(0)
            rc = L.heap_run(E.ctypes.data_as(C.c_void_p), o.ctypes.data_as(C.c_void_p), n, mode, C.byref(c))
            outs.append(o); cyc.append(c.value)
        same = np.array_equal(outs[0], outs[1])
        srt = np.all(np.diff((outs[1] >> np.uint64(32)).astype(np.int64)) >= 0)
        print(f"n {n} kinds {kinds}: lane {cyc[0]} cyc ({cyc[0] / n:.0f}/elem)  wave {cyc[1]} cyc ({cyc[1] / n:.0f}/elem)  identical {same} sorted {srt}", flush=True)
