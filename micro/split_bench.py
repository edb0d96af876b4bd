"""The workgroup split (ls_split_to_list) alone on synthetic key arrays shaped like its two callers: the mapping
stack VoxelGrid (less-flat cloud, ~27k points, ~2 points per 0.8 m leaf, limit 10240) and a big map cube (~14k
old points one per leaf in leaf order + ~2.7k appended ones, limit 4096). Prints the kernel time (HIP events),
levels and per-level phase times (thread 0 stamps: count + scan, k, swaps + cuts, children); saves the split
array and segment list under gpurun_out/ and, given a second tag, checks them against that tag's files
(bit-identical output across split variants). Profiling aid.

usage: python micro/split_bench.py SO TAG [REF_TAG]"""
import ctypes as C
import os
import sys

import numpy as np

so, tag = sys.argv[1], sys.argv[2]
ref = sys.argv[3] if len(sys.argv) > 3 else None
L = C.CDLL(os.path.abspath(so))
L.split_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_ulonglong)]
L.split_stamps.argtypes = [C.c_void_p, C.c_void_p]
os.makedirs("gpurun_out", exist_ok=True)
rng = np.random.default_rng(11)


def pack(keys):
    return (keys.astype(np.uint64) << np.uint64(32)) | np.arange(len(keys), dtype=np.uint64)


cases = []
for i in range(3):
    cases.append((f"stack{i}", pack(rng.integers(0, 13000, 27000 - 500 * i)), 10240))
for i in range(3):
    old = np.sort(rng.choice(1 << 22, 14000 - 700 * i, replace=False))
    new = rng.choice(old, 2700)
    new[::3] = rng.integers(0, 1 << 22, len(new[::3]))
    cases.append((f"cube{i}", pack(np.concatenate([old, new])), 4096))
ok = True
tot_ms = {}
for name, E, limit in cases:
    n = len(E)
    out = np.zeros(n, np.uint64)
    seg = np.zeros(1 + 3 * 1024, np.int32)
    ms = C.c_float(0)
    cyc = C.c_ulonglong(0)
    rc = L.split_run(E.ctypes.data, out.ctypes.data, seg.ctypes.data, n, limit, 20, C.byref(ms), C.byref(cyc))
    ts = np.zeros((64, 6), np.uint64)
    nseg = np.zeros(64, np.int32)
    L.split_stamps(ts.ctypes.data, nseg.ctypes.data)
    t = ts.astype(np.int64)
    lv = [l for l in range(64) if t[l, 0] > 0 and t[l, 4] >= t[l, 0]]
    ph = np.array([np.diff(t[l, :5]) for l in lv]) / 2400.0 if lv else np.zeros((1, 4))
    ns = int(seg[0])
    # split output: every listed segment within bounds, the array a permutation of the input
    perm = np.array_equal(np.sort(out), np.sort(E))
    np.save(f"gpurun_out/split_{tag}_{name}.npy", np.concatenate([out, seg[:1 + 3 * ns].astype(np.uint64)]))
    same = ""
    if ref:
        r = np.load(f"gpurun_out/split_{ref}_{name}.npy")
        eq = np.array_equal(r, np.concatenate([out, seg[:1 + 3 * ns].astype(np.uint64)]))
        ok &= eq
        same = f" identical to {ref}: {eq}"
    ok &= perm and rc == 0
    tot_ms[name] = ms.value
    print(f"{name}: n {n} limit {limit}: {ms.value * 1e3:.1f} us/launch (thread-0 {cyc.value / 2400:.1f} us), {len(lv)} levels, "
          f"{ns} segments, permutation {perm}{same}", flush=True)
    print("   per level (us): " + " | ".join(f"n{nseg[l]}: " + "/".join(f"{x:.1f}" for x in ph[i]) for i, l in enumerate(lv)), flush=True)
print(f"{tag}: mean {np.mean(list(tot_ms.values())) * 1e3:.1f} us/launch, all ok {ok}")
sys.exit(0 if ok else 1)
