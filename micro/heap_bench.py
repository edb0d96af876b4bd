"""ps_heap_sort (one lane) vs ws_heap_sort (one wave: six-level pops, child-flag pops) on one LDS segment: identical
output, cycles per pop (s_memtime ticks) and kernel time per pop (HIP events). First a clock calibration: a chain of
dependent v_fma_f32 (about 4 cycles each for one wave alone, MI355X_MICROARCH.md) timed both ways."""
import ctypes as C, os, sys
import numpy as np
L = C.CDLL(os.environ.get("HEAP_SO") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "heap_bench.so"))
L.heap_run.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_ulonglong), C.POINTER(C.c_float)]
for n in (100000, 1000000):
    buf = np.zeros(64, np.uint64); c = C.c_ulonglong(0); ms = C.c_float(0)
    L.heap_run(buf.ctypes.data_as(C.c_void_p), buf.ctypes.data_as(C.c_void_p), n, 3, C.byref(c), C.byref(ms))
    print(f"calib: {n} dependent fma: {c.value} ticks ({c.value / n:.2f}/fma), kernel {ms.value * 1e3:.1f} us "
          f"-> {c.value / (ms.value * 1e-3) / 1e9:.2f} G ticks/s", flush=True)
for mode, per, what in ((4, 64, "dependent v_fma_f32"), (5, 64, "dependent s_add_u32"), (6, 16, "dependent v_readlane chain"),
                        (7, 16, "dependent ds_read_b32"), (8, 1, "empty loop iteration (taken back-edge)")):
    buf = np.zeros(64, np.uint64); c = C.c_ulonglong(0); ms = C.c_float(0)
    L.heap_run(buf.ctypes.data_as(C.c_void_p), buf.ctypes.data_as(C.c_void_p), 20000, mode, C.byref(c), C.byref(ms))
    print(f"cost: {what}: {c.value / (20000 * per):.2f} cycles each", flush=True)
rng = np.random.default_rng(3)
for n in [int(a) for a in sys.argv[1:]] or [64, 300, 1000, 3000]:
    for kinds in (n // 3, n * 4):
        key = rng.integers(0, kinds, n).astype(np.uint64)
        E = (key << np.uint64(32)) | np.arange(n, dtype=np.uint64)
        outs, cyc, tms = [], [], []
        for mode in (0, 1, 2):
            o = np.zeros(n, np.uint64); c = C.c_ulonglong(0); ms = C.c_float(0)
            L.heap_run(E.ctypes.data_as(C.c_void_p), o.ctypes.data_as(C.c_void_p), n, mode, C.byref(c), C.byref(ms))
            outs.append(o); cyc.append(c.value); tms.append(ms.value)
        same = np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
        srt = np.all(np.diff((outs[2] >> np.uint64(32)).astype(np.int64)) >= 0)
        print(f"n {n} kinds {kinds}: lane {cyc[0] / n:.0f}/elem {tms[0] * 1e6 / n:.0f} ns/elem | wave {cyc[1] / n:.0f}/elem "
              f"{tms[1] * 1e6 / n:.0f} ns/elem | flags {cyc[2] / n:.0f}/elem {tms[2] * 1e6 / n:.0f} ns/elem | identical {same} sorted {srt}",
              flush=True)
