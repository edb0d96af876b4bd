"""ctypes binding of oracle/liboracle.so — the CPU restatement used as the parity checker.

Test infrastructure: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. Never on the product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from lvo_amd_loader import abi

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = os.path.join(_REPO, "oracle", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(_REPO, "oracle"), "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        vp = C.c_void_p
        L.oracle_create.restype = vp
        L.oracle_create.argtypes = [C.POINTER(abi.Params)]
        L.oracle_destroy.argtypes = [vp]
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_last_error.argtypes = [vp]
        L.oracle_set_voxel_order.argtypes = [vp, C.c_int]
        L.oracle_scan_registration.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
        L.oracle_feature_counts.argtypes = [vp, C.POINTER(C.c_int)]
        L.oracle_get_features.argtypes = [vp, C.POINTER(abi.Features)]
        L.oracle_set_features.argtypes = [vp] + [C.POINTER(C.c_float), C.c_int] * 4
        L.oracle_set_odom_state.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                            C.POINTER(C.c_double), C.POINTER(C.c_float), C.c_int,
                                            C.POINTER(C.c_float), C.c_int]
        L.oracle_odometry.argtypes = [vp, C.POINTER(abi.OdomResult)]
        L.oracle_set_mapping_input.argtypes = [vp, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_float), C.c_int,
                                               C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.oracle_mapping.argtypes = [vp, C.POINTER(abi.MapResult)]
        L.oracle_process_scan.argtypes = [vp, C.POINTER(C.c_float), C.c_int, C.POINTER(abi.OdomResult),
                                          C.POINTER(abi.MapResult)]
        L.oracle_stage_times.argtypes = [vp, C.POINTER(C.c_double)]
        L.oracle_tictoc.argtypes = [vp, C.POINTER(C.c_double)]
        L.oracle_get_map_cloud.argtypes = [vp, C.c_int, C.POINTER(abi.Cloud)]
        L.oracle_get_registered_cloud.argtypes = [vp, C.POINTER(abi.Cloud)]
        L.oracle_map_high_freq_pose.argtypes = [vp] + [C.POINTER(C.c_double)] * 4
        L.oracle_cube_check.argtypes = [vp, C.POINTER(C.c_int)]
        L.oracle_eval_factors.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_int,
                                          C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.oracle_lm_solve.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(abi.LMSummary)]
        L.oracle_voxel_grid.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_float, C.c_int, C.POINTER(abi.Cloud)]
        L.oracle_knn.argtypes = [C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_float), C.c_int, C.c_int, C.c_float,
                                 C.POINTER(C.c_int), C.POINTER(C.c_float)]
        L.oracle_s2m_register.argtypes = [C.POINTER(abi.Params)] + [C.POINTER(C.c_float), C.c_int] * 4 + [
            C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(abi.LMSummary)]
        L.oracle_eigen_sym3.argtypes = [C.POINTER(C.c_double)] * 3
        L.oracle_colpiv_qr_5x3.argtypes = [C.POINTER(C.c_double)] * 3
        L.oracle_introsort_keys.argtypes = [C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]
        L.oracle_libstdcxx_sort_keys.argtypes = [C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]
        L.oracle_pcl_replay_check.argtypes = [C.c_int, C.c_int, C.c_ulonglong]
        _lib = L
    return _lib


class Oracle:
    """Three reference nodes' state in one object, same call surface as the HIP context.
    voxel_order 1 (default): PCL's VoxelGrid order (libstdc++ std::sort), the reference's; 0: stable."""

    def __init__(self, params=None, voxel_order=1):
        self.p = params if params is not None else abi.default_params(64)
        self.h = lib().oracle_create(C.byref(self.p))
        lib().oracle_set_voxel_order(self.h, voxel_order)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_destroy(self.h)
            self.h = None

    def scan_registration(self, pts):
        pts = np.ascontiguousarray(pts, np.float32)
        rc = lib().oracle_scan_registration(self.h, abi.fptr(pts), len(pts))
        if rc:
            raise RuntimeError(lib().oracle_last_error(self.h))

    def features(self):
        cnt = (C.c_int * 5)()
        lib().oracle_feature_counts(self.h, cnt)
        n = list(cnt)
        bufs = {}
        f = abi.Features()
        for name, k in zip(["full", "sharp", "less_sharp", "flat", "less_flat"], n):
            c, b = abi.make_cloud(k)
            setattr(f, name, c)
            bufs[name] = b
        idx = {k: np.zeros(max(n[i], 1), np.int32) for k, i in (("sharp_idx", 1), ("less_sharp_idx", 2), ("flat_idx", 3))}
        curv = np.zeros(max(n[0], 1), np.float32)
        f.sharp_idx, f.less_sharp_idx, f.flat_idx = abi.iptr(idx["sharp_idx"]), abi.iptr(idx["less_sharp_idx"]), abi.iptr(idx["flat_idx"])
        f.curvature = abi.fptr(curv)
        lib().oracle_get_features(self.h, C.byref(f))
        out = {name: bufs[name][:k].copy() for name, k in zip(["full", "sharp", "less_sharp", "flat", "less_flat"], n)}
        out["sharp_idx"] = idx["sharp_idx"][:n[1]].copy()
        out["less_sharp_idx"] = idx["less_sharp_idx"][:n[2]].copy()
        out["flat_idx"] = idx["flat_idx"][:n[3]].copy()
        out["curvature"] = curv[:n[0]].copy()
        return out

    def set_features(self, sharp, less_sharp, flat, less_flat):
        arrs = [np.ascontiguousarray(a, np.float32).reshape(-1, 4) for a in (sharp, less_sharp, flat, less_flat)]
        args = []
        for a in arrs:
            args += [abi.fptr(a), len(a)]
        lib().oracle_set_features(self.h, *args)

    def set_odom_state(self, q, t, qw, tw, corner_last, surf_last):
        q, t, qw, tw = (np.ascontiguousarray(v, np.float64) for v in (q, t, qw, tw))
        cl = np.ascontiguousarray(corner_last, np.float32).reshape(-1, 4)
        sl = np.ascontiguousarray(surf_last, np.float32).reshape(-1, 4)
        lib().oracle_set_odom_state(self.h, abi.dptr(q), abi.dptr(t), abi.dptr(qw), abi.dptr(tw),
                                    abi.fptr(cl), len(cl), abi.fptr(sl), len(sl))

    def odometry(self):
        r = abi.OdomResult()
        rc = lib().oracle_odometry(self.h, C.byref(r))
        if rc:
            raise RuntimeError(lib().oracle_last_error(self.h))
        return abi.odom_to_dict(r)

    def set_mapping_input(self, corner, surf, q, t):
        cl = np.ascontiguousarray(corner, np.float32).reshape(-1, 4)
        sl = np.ascontiguousarray(surf, np.float32).reshape(-1, 4)
        q, t = np.ascontiguousarray(q, np.float64), np.ascontiguousarray(t, np.float64)
        lib().oracle_set_mapping_input(self.h, abi.fptr(cl), len(cl), abi.fptr(sl), len(sl), abi.dptr(q), abi.dptr(t))

    def mapping(self):
        r = abi.MapResult()
        rc = lib().oracle_mapping(self.h, C.byref(r))
        if rc:
            raise RuntimeError(lib().oracle_last_error(self.h))
        return abi.map_to_dict(r)

    def process_scan(self, pts):
        pts = np.ascontiguousarray(pts, np.float32)
        o, m = abi.OdomResult(), abi.MapResult()
        rc = lib().oracle_process_scan(self.h, abi.fptr(pts), len(pts), C.byref(o), C.byref(m))
        if rc:
            raise RuntimeError(lib().oracle_last_error(self.h))
        return abi.odom_to_dict(o), abi.map_to_dict(m)

    def stage_times(self):
        t = (C.c_double * 3)()
        lib().oracle_stage_times(self.h, t)
        return list(t)

    def tictoc(self):
        """The reference's TicToc stage times (ms) of the last calls, keyed by the printed names."""
        t = (C.c_double * len(abi.TICTOC_NAMES))()
        lib().oracle_tictoc(self.h, t)
        return dict(zip(abi.TICTOC_NAMES, list(t)))

    def map_cloud(self, which, cap=4_000_000):
        c, b = abi.make_cloud(cap)
        lib().oracle_get_map_cloud(self.h, which, C.byref(c))
        return b[:min(c.n, cap)].copy()

    def cube_check(self):
        """{cen: (W, H, D), points, misplaced, cubes}: every stored point re-bucketed directly with the
        current cube centre (oracle_cube_check)."""
        o = (C.c_int * 6)()
        lib().oracle_cube_check(self.h, o)
        return {"cen": (o[0], o[1], o[2]), "points": o[3], "misplaced": o[4], "cubes": o[5]}

    def registered_cloud(self, cap=400_000):
        c, b = abi.make_cloud(cap)
        lib().oracle_get_registered_cloud(self.h, C.byref(c))
        return b[:min(c.n, cap)].copy()

    def high_freq_pose(self, q_wodom, t_wodom):
        q, t = np.ascontiguousarray(q_wodom, np.float64), np.ascontiguousarray(t_wodom, np.float64)
        qo, to = np.zeros(4), np.zeros(3)
        lib().oracle_map_high_freq_pose(self.h, abi.dptr(q), abi.dptr(t), abi.dptr(qo), abi.dptr(to))
        return qo, to


def eval_factors(factors, x, robust=True):
    f = np.ascontiguousarray(factors, abi.FACTOR_DTYPE)
    n = len(f)
    x = np.ascontiguousarray(x, np.float64)
    res = np.zeros(3 * n)
    jac = np.zeros(3 * n * 6)
    neq = np.zeros(28)
    lib().oracle_eval_factors(f.ctypes.data_as(C.c_void_p), n, abi.dptr(x), int(robust), abi.dptr(res), abi.dptr(jac), abi.dptr(neq))
    return res.reshape(n, 3), jac.reshape(n, 3, 6), neq


def lm_solve(factors, x, max_iter=4):
    f = np.ascontiguousarray(factors, abi.FACTOR_DTYPE)
    x = np.array(x, np.float64)
    s = abi.LMSummary()
    lib().oracle_lm_solve(f.ctypes.data_as(C.c_void_p), len(f), abi.dptr(x), max_iter, C.byref(s))
    return x, (s.iterations, s.successful_steps, s.termination, s.num_residual_blocks, s.initial_cost, s.final_cost)


def voxel_grid(pts, leaf, order=1):
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 4)
    c, b = abi.make_cloud(len(pts))
    lib().oracle_voxel_grid(abi.fptr(pts), len(pts), leaf, order, C.byref(c))
    return b[:c.n].copy()


def knn(pts, queries, k, radius=0.0):
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 4)
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 4)
    idx = np.zeros((len(q), k), np.int32)
    d2 = np.zeros((len(q), k), np.float32)
    lib().oracle_knn(abi.fptr(pts), len(pts), abi.fptr(q), len(q), k, radius, abi.iptr(idx), abi.fptr(d2))
    return idx, d2


def eigen_sym3(A):
    A = np.ascontiguousarray(A, np.float64).reshape(9)
    ev = np.zeros(3)
    evec = np.zeros(9)
    lib().oracle_eigen_sym3(abi.dptr(A), abi.dptr(ev), abi.dptr(evec))
    return ev, evec.reshape(3, 3)


def colpiv_qr_5x3(A, b):
    A = np.ascontiguousarray(A, np.float64).reshape(15)
    b = np.ascontiguousarray(b, np.float64).reshape(5)
    x = np.zeros(3)
    lib().oracle_colpiv_qr_5x3(abi.dptr(A), abi.dptr(b), abi.dptr(x))
    return x


def pcl_replay_check(trials, max_n, seed=7):
    """Mismatches of the level-parallel std::sort replay (the device algorithm's host twin) vs libstdc++."""
    return lib().oracle_pcl_replay_check(trials, max_n, seed)


def introsort_perm(keys, libstdcxx=False):
    k = np.ascontiguousarray(keys, np.float32)
    p = np.zeros(len(k), np.int32)
    fn = lib().oracle_libstdcxx_sort_keys if libstdcxx else lib().oracle_introsort_keys
    fn(abi.fptr(k), len(k), abi.iptr(p))
    return p


def s2m_register(params, corner_map, surf_map, corner_q, surf_q, x):
    """oracle_s2m_register: the laserMapping registration rounds against a given map (kd-tree 5-NN,
    Eigen line / plane fits, Ceres-style LM). Returns a dict shaped like Context.s2m_register's."""
    arrs = [np.ascontiguousarray(a, np.float32).reshape(-1, 4) for a in (corner_map, surf_map, corner_q, surf_q)]
    x = np.array(x, np.float64)
    res = np.zeros(2 + 2 * abi.ALOAM_MAX_ROUNDS, np.int32)
    lm_ = (abi.LMSummary * abi.ALOAM_MAX_ROUNDS)()
    args = []
    for a in arrs:
        args += [abi.fptr(a), len(a)]
    lib().oracle_s2m_register(C.byref(params), *args, abi.dptr(x), abi.iptr(res), lm_)
    n = int(res[1])
    return {"x": x, "q_w_curr": x[:4].copy(), "t_w_curr": x[4:].copy(), "optimized": int(res[0]), "rounds": n,
            "corner_num": [int(v) for v in res[2:2 + n]],
            "surf_num": [int(v) for v in res[2 + abi.ALOAM_MAX_ROUNDS:2 + abi.ALOAM_MAX_ROUNDS + n]],
            "lm": [(lm_[i].iterations, lm_[i].successful_steps, lm_[i].termination, lm_[i].num_residual_blocks,
                    lm_[i].initial_cost, lm_[i].final_cost) for i in range(n)]}
