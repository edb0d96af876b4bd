"""MI355X-native A-LOAM per-scan hot path (host mirror of the reference's three nodes).

The compute lives in ``csrc/`` (hand-written HIP for gfx950) behind the C ABI declared in
``include/aloam_hip.h`` and built as ``csrc/libaloam_hip.so``. This module is a thin ctypes
host over that ABI with the reference's call surface:

  * ``Context.scan_registration(points)``  ~ ``laserCloudHandler``   (src/scanRegistration.cpp:114)
  * ``Context.odometry()``                  ~ laserOdometry main loop (src/laserOdometry.cpp:311)
  * ``Context.mapping()``                   ~ laserMapping ``process`` (src/laserMapping.cpp:231)

There is no CPU fallback: creating a ``Context`` without the HIP library or without a GPU
raises. The CPU restatement in ``oracle/`` is test infrastructure and is never imported here.
"""
import ctypes as C
import os
import sys

import numpy as np

from . import _abi as abi  # noqa: F401
from . import replicas  # noqa: F401
from . import synth  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ALOAM_LIB_PATH") or os.path.join(_HERE, "csrc", "libaloam_hip.so")   # override: profiling builds only
_lib = None


class ALOAMError(RuntimeError):
    pass


def _declare(L):
    vp = C.c_void_p
    F, I, D = C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_double)
    L.aloam_abi_version.restype = C.c_int
    L.aloam_default_params.argtypes = [C.POINTER(abi.Params), C.c_int]
    L.aloam_create.restype = vp
    L.aloam_create.argtypes = [C.POINTER(abi.Params), C.c_int]
    L.aloam_destroy.argtypes = [vp]
    L.aloam_last_error.restype = C.c_char_p
    L.aloam_last_error.argtypes = [vp]
    L.aloam_knn_kernel.restype = C.c_char_p
    L.aloam_knn_kernel.argtypes = [vp]
    L.aloam_scan_registration.argtypes = [vp, C.c_void_p, C.c_int, C.c_int]
    L.aloam_feature_counts.argtypes = [vp, I]
    L.aloam_get_features.argtypes = [vp, C.POINTER(abi.Features)]
    L.aloam_odometry.argtypes = [vp, C.POINTER(abi.OdomResult)]
    L.aloam_set_features.argtypes = [vp] + [F, C.c_int] * 4
    L.aloam_set_odom_state.argtypes = [vp, D, D, D, D, F, C.c_int, F, C.c_int]
    L.aloam_mapping.argtypes = [vp, C.POINTER(abi.MapResult)]
    L.aloam_set_mapping_input.argtypes = [vp, F, C.c_int, F, C.c_int, D, D]
    L.aloam_get_map_cloud.argtypes = [vp, C.c_int, C.POINTER(abi.Cloud)]
    L.aloam_get_registered_cloud.argtypes = [vp, C.POINTER(abi.Cloud)]
    L.aloam_map_high_freq_pose.argtypes = [vp, D, D, D, D]
    L.aloam_map_high_freq_pose.restype = C.c_int
    L.aloam_process_scan.argtypes = [vp, C.c_void_p, C.c_int, C.c_int, C.POINTER(abi.OdomResult), C.POINTER(abi.MapResult)]
    L.aloam_eval_factors.argtypes = [vp, C.c_void_p, C.c_int, D, C.c_int, D, D, D]
    L.aloam_lm_solve.argtypes = [vp, C.c_void_p, C.c_int, D, C.POINTER(abi.LMSummary)]
    L.aloam_voxel_grid.argtypes = [vp, F, C.c_int, C.c_float, C.POINTER(abi.Cloud)]
    L.aloam_knn.argtypes = [vp, F, C.c_int, F, C.c_int, C.c_int, C.c_float, I, F]
    L.aloam_set_profiling.argtypes = [vp, C.c_int]
    L.aloam_get_timing.argtypes = [vp, C.POINTER(abi.Timing)]
    L.aloam_forward_mapping_input.argtypes = [vp, vp]
    L.aloam_knn_device.argtypes = [vp, vp, C.c_int, vp, C.c_int, C.c_int, C.c_float, vp, vp]
    L.aloam_knn_build.argtypes = [vp, vp, C.c_int, C.c_float]
    L.aloam_knn_query.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp]
    L.aloam_forward_features.argtypes = [vp, vp]
    L.aloam_s2m_set_map.argtypes = [vp, vp, C.c_int, vp, C.c_int, C.c_int]
    L.aloam_s2m_set_queries.argtypes = [vp, vp, C.c_int, vp, C.c_int, C.c_int]
    L.aloam_s2m_register.argtypes = [vp, D, C.POINTER(abi.S2MResult)]
    L.aloam_s2m_register_group.argtypes = [C.POINTER(vp), C.c_int, D, C.POINTER(abi.S2MResult)]
    L.aloam_shard_unique_id.argtypes = [C.c_char_p]
    L.aloam_shard_init.argtypes = [vp, C.c_int, C.c_int, C.c_char_p]
    L.aloam_shard_slot_range.argtypes = [C.c_int, C.c_int, C.c_int, I, I]
    L.aloam_shard_peer_handle.argtypes = [vp, C.c_char_p]
    L.aloam_shard_peer_open.argtypes = [vp, C.c_char_p, C.c_int, C.c_int]
    L.aloam_shard_peer_close.argtypes = [vp]
    L.aloam_set_cu_mask.argtypes = [vp, C.POINTER(C.c_uint), C.c_int]
    L.aloam_set_cu_mask.restype = C.c_int
    L.aloam_serial_sort_fallbacks.argtypes = [C.POINTER(C.c_ulonglong)]
    L.aloam_serial_sort_fallbacks.restype = C.c_int
    L.aloam_scan_registration_pc2.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int]
    L.aloam_scan_registration_pc2.restype = C.c_int
    L.aloam_pipeline_create.restype = vp
    L.aloam_pipeline_create.argtypes = [C.POINTER(abi.Params), C.c_int, C.c_int]
    L.aloam_pipeline_destroy.argtypes = [vp]
    L.aloam_pipeline_last_error.restype = C.c_char_p
    L.aloam_pipeline_last_error.argtypes = [vp]
    L.aloam_pipeline_context.restype = vp
    L.aloam_pipeline_context.argtypes = [vp, C.c_int]
    L.aloam_pipeline_push.argtypes = [vp, vp, C.c_int, C.c_int, C.POINTER(abi.OdomResult), I,
                                      C.POINTER(abi.MapResult), I]
    L.aloam_pipeline_flush.argtypes = [vp, C.POINTER(abi.OdomResult), I, C.POINTER(abi.MapResult), I,
                                       C.POINTER(abi.MapResult), I]
    L.aloam_pipeline_set_profiling.argtypes = [vp, C.c_int]
    L.aloam_pipeline_timing.argtypes = [vp, C.c_int, C.POINTER(abi.Timing)]
    for name in ("aloam_pipeline_push", "aloam_pipeline_flush", "aloam_pipeline_set_profiling", "aloam_pipeline_timing"):
        getattr(L, name).restype = C.c_int
    for name in ("aloam_s2m_set_map", "aloam_s2m_set_queries", "aloam_s2m_register", "aloam_s2m_register_group",
                 "aloam_shard_unique_id", "aloam_shard_init", "aloam_shard_slot_range",
                 "aloam_shard_peer_handle", "aloam_shard_peer_open", "aloam_shard_peer_close"):
        getattr(L, name).restype = C.c_int
    for name in ("aloam_forward_mapping_input", "aloam_knn_device", "aloam_knn_build", "aloam_knn_query", "aloam_forward_features", "aloam_scan_registration", "aloam_feature_counts", "aloam_get_features", "aloam_odometry",
                 "aloam_set_features", "aloam_set_odom_state", "aloam_mapping", "aloam_set_mapping_input",
                 "aloam_get_map_cloud", "aloam_get_registered_cloud", "aloam_process_scan", "aloam_eval_factors",
                 "aloam_lm_solve", "aloam_voxel_grid", "aloam_knn", "aloam_set_profiling", "aloam_get_timing"):
        getattr(L, name).restype = C.c_int
    return L


def lib():
    """Load csrc/libaloam_hip.so (built in-tree by __graft_entry__.build()). Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ALOAMError(f"HIP extension not built: {LIB_PATH} (run __graft_entry__.build())")
        # One HIP runtime per process: the PyTorch wheel bundles its own libamdhip64.so.7, which
        # libtorch_hip requests under a different name; if our library loaded /opt/rocm's copy first,
        # torch would load a second runtime that then sees no device. Importing torch first makes
        # our NEEDED libamdhip64.so.7 resolve to the copy already in the process.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = _declare(C.CDLL(LIB_PATH))
    return _lib


EXPORTED_SYMBOLS = [
    "aloam_abi_version", "aloam_default_params", "aloam_create", "aloam_destroy", "aloam_last_error",
    "aloam_scan_registration", "aloam_feature_counts", "aloam_get_features", "aloam_odometry",
    "aloam_set_features", "aloam_set_odom_state", "aloam_mapping", "aloam_set_mapping_input",
    "aloam_get_map_cloud", "aloam_get_registered_cloud", "aloam_process_scan", "aloam_eval_factors",
    "aloam_lm_solve", "aloam_voxel_grid", "aloam_knn", "aloam_set_profiling", "aloam_get_timing",
    "aloam_forward_mapping_input", "aloam_knn_device", "aloam_forward_features",
    "aloam_s2m_set_map", "aloam_s2m_set_queries", "aloam_s2m_register", "aloam_s2m_register_group",
    "aloam_shard_unique_id", "aloam_shard_init", "aloam_shard_slot_range",
    "aloam_scan_registration_pc2", "aloam_set_cu_mask", "aloam_serial_sort_fallbacks",
    "aloam_pipeline_create", "aloam_pipeline_destroy", "aloam_pipeline_last_error", "aloam_pipeline_context",
    "aloam_pipeline_push", "aloam_pipeline_flush", "aloam_pipeline_set_profiling", "aloam_pipeline_timing",
    "aloam_map_high_freq_pose", "aloam_knn_kernel", "aloam_knn_build", "aloam_knn_query",
    "aloam_shard_peer_handle", "aloam_shard_peer_open", "aloam_shard_peer_close",
]


class Context:
    """One aloam_ctx: the state of scanRegistration + laserOdometry + laserMapping on one GPU."""

    def __init__(self, params=None, device=0):
        self.p = params if params is not None else abi.default_params(64)
        L = lib()
        self.h = L.aloam_create(C.byref(self.p), int(device))
        if not self.h:
            raise ALOAMError("aloam_create failed (no HIP device?)")
        self._fail_on(L.aloam_last_error(self.h), creating=True)

    def _fail_on(self, msg, creating=False):
        if creating and msg:
            m = msg.decode()
            if m:
                self.close()
                raise ALOAMError(m)

    def _check(self, rc):
        if rc != 0:
            raise ALOAMError(f"rc={rc}: {lib().aloam_last_error(self.h).decode()}")

    def close(self):
        if getattr(self, "h", None):
            lib().aloam_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- stage 1 ----
    def scan_registration(self, pts, device_ptr=None):
        if device_ptr is not None:
            self._check(lib().aloam_scan_registration(self.h, C.c_void_p(device_ptr), int(pts), abi.ALOAM_INPUT_DEVICE))
            return
        pts = np.ascontiguousarray(pts, np.float32)
        self._check(lib().aloam_scan_registration(self.h, pts.ctypes.data_as(C.c_void_p), len(pts), 0))

    def scan_registration_pc2(self, blob, n=None, point_step=32, device_ptr=None):
        """aloam_scan_registration_pc2: a PointCloud2 data blob (bytes / uint8 array of n records of
        point_step bytes, x y z float32 at offsets 0 4 8), or a device pointer with n given."""
        if device_ptr is not None:
            self._check(lib().aloam_scan_registration_pc2(self.h, C.c_void_p(device_ptr), int(n), int(point_step),
                                                          abi.ALOAM_INPUT_DEVICE))
            return
        b = np.ascontiguousarray(np.frombuffer(blob, np.uint8) if isinstance(blob, (bytes, bytearray)) else blob).view(np.uint8)
        n = len(b) // point_step if n is None else int(n)
        self._check(lib().aloam_scan_registration_pc2(self.h, b.ctypes.data_as(C.c_void_p), n, int(point_step), 0))

    def feature_counts(self):
        cnt = (C.c_int * 5)()
        self._check(lib().aloam_feature_counts(self.h, cnt))
        return list(cnt)

    def features(self):
        n = self.feature_counts()
        names = ["full", "sharp", "less_sharp", "flat", "less_flat"]
        f = abi.Features()
        bufs = {}
        for name, k in zip(names, n):
            c, b = abi.make_cloud(k)
            setattr(f, name, c)
            bufs[name] = b
        idx = {k: np.zeros(max(n[i], 1), np.int32) for k, i in (("sharp_idx", 1), ("less_sharp_idx", 2), ("flat_idx", 3))}
        curv = np.zeros(max(n[0], 1), np.float32)
        f.sharp_idx, f.less_sharp_idx, f.flat_idx = (abi.iptr(idx[k]) for k in ("sharp_idx", "less_sharp_idx", "flat_idx"))
        f.curvature = abi.fptr(curv)
        self._check(lib().aloam_get_features(self.h, C.byref(f)))
        out = {name: bufs[name][:k].copy() for name, k in zip(names, n)}
        out["sharp_idx"] = idx["sharp_idx"][:n[1]].copy()
        out["less_sharp_idx"] = idx["less_sharp_idx"][:n[2]].copy()
        out["flat_idx"] = idx["flat_idx"][:n[3]].copy()
        out["curvature"] = curv[:n[0]].copy()
        return out

    # ---- stage 2 ----
    def set_features(self, sharp, less_sharp, flat, less_flat):
        arrs = [np.ascontiguousarray(a, np.float32).reshape(-1, 4) for a in (sharp, less_sharp, flat, less_flat)]
        args = []
        for a in arrs:
            args += [abi.fptr(a), len(a)]
        self._check(lib().aloam_set_features(self.h, *args))

    def set_odom_state(self, q, t, qw, tw, corner_last, surf_last):
        q, t, qw, tw = (np.ascontiguousarray(v, np.float64) for v in (q, t, qw, tw))
        cl = np.ascontiguousarray(corner_last, np.float32).reshape(-1, 4)
        sl = np.ascontiguousarray(surf_last, np.float32).reshape(-1, 4)
        self._check(lib().aloam_set_odom_state(self.h, abi.dptr(q), abi.dptr(t), abi.dptr(qw), abi.dptr(tw),
                                               abi.fptr(cl), len(cl), abi.fptr(sl), len(sl)))

    def odometry(self):
        r = abi.OdomResult()
        self._check(lib().aloam_odometry(self.h, C.byref(r)))
        return abi.odom_to_dict(r)

    # ---- stage 3 ----
    def set_mapping_input(self, corner, surf, q, t):
        cl = np.ascontiguousarray(corner, np.float32).reshape(-1, 4)
        sl = np.ascontiguousarray(surf, np.float32).reshape(-1, 4)
        q, t = np.ascontiguousarray(q, np.float64), np.ascontiguousarray(t, np.float64)
        self._check(lib().aloam_set_mapping_input(self.h, abi.fptr(cl), len(cl), abi.fptr(sl), len(sl), abi.dptr(q), abi.dptr(t)))

    def mapping(self):
        r = abi.MapResult()
        self._check(lib().aloam_mapping(self.h, C.byref(r)))
        return abi.map_to_dict(r)

    def map_cloud(self, which, cap=4_000_000):
        c, b = abi.make_cloud(cap)
        self._check(lib().aloam_get_map_cloud(self.h, which, C.byref(c)))
        return b[:min(c.n, cap)].copy()

    def registered_cloud(self, cap=400_000):
        c, b = abi.make_cloud(cap)
        self._check(lib().aloam_get_registered_cloud(self.h, C.byref(c)))
        return b[:min(c.n, cap)].copy()

    def high_freq_pose(self, q_wodom, t_wodom):
        """/aft_mapped_to_init_high_frec of an odometry pose (laserMapping.cpp:197-229): (q, t)."""
        q, t = np.ascontiguousarray(q_wodom, np.float64), np.ascontiguousarray(t_wodom, np.float64)
        qo, to = np.zeros(4), np.zeros(3)
        self._check(lib().aloam_map_high_freq_pose(self.h, abi.dptr(q), abi.dptr(t), abi.dptr(qo), abi.dptr(to)))
        return qo, to

    # ---- whole pipeline ----
    def process_scan(self, pts=None, device_ptr=None, n=None, mapping=True):
        o, m = abi.OdomResult(), abi.MapResult()
        fl = 0 if mapping else abi.ALOAM_NO_MAPPING
        if device_ptr is not None:
            self._check(lib().aloam_process_scan(self.h, C.c_void_p(device_ptr), int(n), abi.ALOAM_INPUT_DEVICE | fl,
                                                 C.byref(o), C.byref(m)))
        else:
            pts = np.ascontiguousarray(pts, np.float32)
            self._check(lib().aloam_process_scan(self.h, pts.ctypes.data_as(C.c_void_p), len(pts), fl, C.byref(o), C.byref(m)))
        return abi.odom_to_dict(o), abi.map_to_dict(m)

    def forward_features(self, dst):
        """Hand this context's scanRegistration output to `dst`'s laserOdometry (device to device)."""
        self._check(lib().aloam_forward_features(self.h, dst.h))

    def forward_mapping_input(self, dst):
        """Hand this context's published odometry output to `dst`'s laserMapping (device to device)."""
        self._check(lib().aloam_forward_mapping_input(self.h, dst.h))

    # ---- low level ----
    def eval_factors(self, factors, x, robust=True):
        f = np.ascontiguousarray(factors, abi.FACTOR_DTYPE)
        n = len(f)
        x = np.ascontiguousarray(x, np.float64)
        res, jac, neq = np.zeros(3 * n), np.zeros(3 * n * 6), np.zeros(28)
        self._check(lib().aloam_eval_factors(self.h, f.ctypes.data_as(C.c_void_p), n, abi.dptr(x), int(robust),
                                             abi.dptr(res), abi.dptr(jac), abi.dptr(neq)))
        return res.reshape(n, 3), jac.reshape(n, 3, 6), neq

    def lm_solve(self, factors, x):
        f = np.ascontiguousarray(factors, abi.FACTOR_DTYPE)
        x = np.array(x, np.float64)
        s = abi.LMSummary()
        self._check(lib().aloam_lm_solve(self.h, f.ctypes.data_as(C.c_void_p), len(f), abi.dptr(x), C.byref(s)))
        return x, (s.iterations, s.successful_steps, s.termination, s.num_residual_blocks, s.initial_cost, s.final_cost)

    def voxel_grid(self, pts, leaf):
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 4)
        c, b = abi.make_cloud(len(pts))
        self._check(lib().aloam_voxel_grid(self.h, abi.fptr(pts), len(pts), leaf, C.byref(c)))
        return b[:c.n].copy()

    def knn(self, pts, queries, k, radius=0.0):
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 4)
        q = np.ascontiguousarray(queries, np.float32).reshape(-1, 4)
        idx = np.zeros((len(q), k), np.int32)
        d2 = np.zeros((len(q), k), np.float32)
        self._check(lib().aloam_knn(self.h, abi.fptr(pts), len(pts), abi.fptr(q), len(q), k, radius, abi.iptr(idx), abi.fptr(d2)))
        return idx, d2

    @staticmethod
    def _producer_sync():
        """Device buffers handed over by pointer must be complete: torch fills / copies them on ITS current
        stream, which the library's stream does not wait for (a torch.full still running when the search
        writes its output would overwrite it). Not used on the per-scan path (the caller syncs once there)."""
        tm = sys.modules.get("torch")
        if tm is not None and tm.cuda.is_initialized():
            tm.cuda.current_stream().synchronize()

    def knn_device(self, d_pts, n, d_queries, nq, k, radius, d_idx, d_d2):
        """aloam_knn_device on device pointers (ints, e.g. torch tensor .data_ptr())."""
        self._producer_sync()
        self._check(lib().aloam_knn_device(self.h, C.c_void_p(d_pts), int(n), C.c_void_p(d_queries), int(nq), int(k),
                                           float(radius), C.c_void_p(d_idx), C.c_void_p(d_d2)))

    def knn_build(self, d_pts, n, radius):
        """aloam_knn_build: index n device float4 points for radius searches (built once, queried many times)."""
        self._producer_sync()
        self._check(lib().aloam_knn_build(self.h, C.c_void_p(d_pts), int(n), float(radius)))

    def knn_query(self, d_queries, nq, k, d_idx, d_d2):
        """aloam_knn_query against the last knn_build index (device pointers)."""
        self._producer_sync()
        self._check(lib().aloam_knn_query(self.h, C.c_void_p(d_queries), int(nq), int(k), C.c_void_p(d_idx),
                                          C.c_void_p(d_d2)))

    def knn_kernel(self):
        """Name of the search kernel the last knn_device call launched (aloam_knn_kernel)."""
        return lib().aloam_knn_kernel(self.h).decode()

    # ---- scan-to-map registration, sharded over ranks (laserMapping.cpp:556-727; BASELINE configs[3]) ----
    @staticmethod
    def _pts_arg(a, n):
        """(pointer, n, flags) for a float4 cloud: a numpy (n, 4) float32 array, or an int device pointer."""
        if isinstance(a, int):
            return C.c_void_p(a), int(n), abi.ALOAM_INPUT_DEVICE
        a = np.ascontiguousarray(a, np.float32).reshape(-1, 4)
        return a, len(a), 0

    def s2m_set_map(self, corner, surf, n_corner=None, n_surf=None):
        """The local map (laserCloudCornerFromMap / SurfFromMap) as host arrays or device pointers."""
        self._producer_sync()
        c, nc, fc = self._pts_arg(corner, n_corner)
        s, ns, fs = self._pts_arg(surf, n_surf)
        if fc != fs:
            raise ALOAMError("corner and surf map must both be host arrays or both device pointers")
        cp = c if fc else c.ctypes.data_as(C.c_void_p)
        sp = s if fs else s.ctypes.data_as(C.c_void_p)
        self._check(lib().aloam_s2m_set_map(self.h, cp, nc, sp, ns, fc))

    def s2m_set_queries(self, corner, surf, n_corner=None, n_surf=None):
        """The query stacks (laserCloudCornerStack / SurfStack, body frame)."""
        self._producer_sync()
        c, nc, fc = self._pts_arg(corner, n_corner)
        s, ns, fs = self._pts_arg(surf, n_surf)
        if fc != fs:
            raise ALOAMError("corner and surf stacks must both be host arrays or both device pointers")
        cp = c if fc else c.ctypes.data_as(C.c_void_p)
        sp = s if fs else s.ctypes.data_as(C.c_void_p)
        self._check(lib().aloam_s2m_set_queries(self.h, cp, nc, sp, ns, fc))

    def s2m_register(self, x):
        """10 rounds of association + Solve from x = (qx,qy,qz,qw,tx,ty,tz); collective when sharded."""
        x = np.array(x, np.float64)
        r = abi.S2MResult()
        self._check(lib().aloam_s2m_register(self.h, abi.dptr(x), C.byref(r)))
        return abi.s2m_to_dict(r)

    def shard_init(self, rank, world, uid=None):
        """Attach this context to an RCCL communicator of `world` ranks (uid: 128 bytes from rank 0)."""
        if world > 1 and (uid is None or len(uid) != 128):
            raise ALOAMError("shard_init needs the 128-byte unique id for world > 1")
        self._check(lib().aloam_shard_init(self.h, int(rank), int(world), bytes(uid) if uid is not None else None))

    def shard_peer_handle(self):
        """64-byte IPC handle of this context's exchange buffer (aloam_shard_peer_handle)."""
        buf = C.create_string_buffer(64)
        self._check(lib().aloam_shard_peer_handle(self.h, buf))
        return buf.raw

    def shard_peer_open(self, handles, rank):
        """Open the device-side exchange over the world's handles (rank order); collective, follow it with a
        barrier before the first s2m_register (aloam_shard_peer_open)."""
        if any(len(h) != 64 for h in handles):
            raise ALOAMError("peer handles are 64 bytes each")
        self._check(lib().aloam_shard_peer_open(self.h, b"".join(bytes(h) for h in handles), len(handles), int(rank)))

    def shard_peer_close(self):
        self._check(lib().aloam_shard_peer_close(self.h))

    def set_profiling(self, on):
        self._check(lib().aloam_set_profiling(self.h, int(on)))

    def timing(self):
        t = abi.Timing()
        self._check(lib().aloam_get_timing(self.h, C.byref(t)))
        return abi.timing_to_dict(t)


def serial_sort_fallbacks():
    """VoxelGrid / segment sorts that ran the exact one-thread std::sort (n > 65,536), process-wide."""
    v = C.c_ulonglong(0)
    rc = lib().aloam_serial_sort_fallbacks(C.byref(v))
    if rc:
        raise ALOAMError(f"aloam_serial_sort_fallbacks: {rc}")
    return int(v.value)


def s2m_register_group(contexts, x):
    """aloam_s2m_register_group: ranks = contexts (same map and stacks set on each), exchange by peer
    copies between their streams. Returns one result dict per rank."""
    world = len(contexts)
    arr = (C.c_void_p * world)(*[c.h for c in contexts])
    x = np.array(x, np.float64)
    res = (abi.S2MResult * world)()
    rc = lib().aloam_s2m_register_group(arr, world, abi.dptr(x), res)
    if rc != 0:
        raise ALOAMError(f"rc={rc}: {lib().aloam_last_error(contexts[0].h).decode()}")
    return [abi.s2m_to_dict(res[r]) for r in range(world)]


def shard_unique_id():
    """128-byte RCCL unique id (call on rank 0 only, then distribute)."""
    buf = C.create_string_buffer(128)
    rc = lib().aloam_shard_unique_id(buf)
    if rc != 0:
        raise ALOAMError(f"aloam_shard_unique_id rc={rc}: {lib().aloam_last_error(None).decode()}")
    return buf.raw


def shard_slot_range(n_slots, rank, world):
    """[begin, end) query slots of `rank` (the library's own decomposition; no device needed)."""
    b, e = C.c_int(), C.c_int()
    rc = lib().aloam_shard_slot_range(int(n_slots), int(rank), int(world), C.byref(b), C.byref(e))
    if rc != 0:
        raise ALOAMError(f"aloam_shard_slot_range rc={rc}")
    return b.value, e.value


class Pipeline:
    """The reference's node split on one GPU, run by the library's native pipeline
    (aloam_pipeline_*, csrc/aloam_pipeline.hip): one context (own HIP stream) and one native worker
    thread per later stage — the three ROS processes of the reference (src/scanRegistration.cpp,
    src/laserOdometry.cpp, src/laserMapping.cpp:934 `process` thread) — handing over device to device.
    stages=2 (default; measured faster on one MI355X): [scanRegistration + laserOdometry] of scan k on
    the caller's thread || laserMapping of scan k-1 on a worker. stages=3: one stage per node.
    Every scan still goes through all three stages, in order; results equal Context.process_scan's."""

    def __init__(self, params=None, device=0, stages=2):
        self.p = params if params is not None else abi.default_params(64)
        self.stages = stages
        L = lib()
        self.h = L.aloam_pipeline_create(C.byref(self.p), int(device), int(stages))
        if not self.h:
            raise ALOAMError(f"aloam_pipeline_create failed: {L.aloam_last_error(None).decode()}")
        self._profiling = False
        self.last_back_timing = None
        self.last_odom_timing = None
        self.last_front_timing = None

    def _check(self, rc):
        if rc != 0:
            raise ALOAMError(f"rc={rc}: {lib().aloam_pipeline_last_error(self.h).decode()}")

    def context_handle(self, stage):
        return lib().aloam_pipeline_context(self.h, int(stage))

    def _timing(self, stage):
        t = abi.Timing()
        self._check(lib().aloam_pipeline_timing(self.h, stage, C.byref(t)))
        return abi.timing_to_dict(t)

    def set_profiling(self, on):
        self._check(lib().aloam_pipeline_set_profiling(self.h, int(on)))
        self._profiling = bool(on)

    def push(self, pts=None, device_ptr=None, n=None):
        """Feed one scan. Returns (odometry result, mapping result) of the scans that completed those
        stages during this step (None while the pipeline fills)."""
        if device_ptr is not None:
            ptr, cnt, flags = C.c_void_p(device_ptr), int(n), abi.ALOAM_INPUT_DEVICE
        else:
            pts = np.ascontiguousarray(pts, np.float32)
            ptr, cnt, flags = pts.ctypes.data_as(C.c_void_p), len(pts), 0
        od, mp = abi.OdomResult(), abi.MapResult()
        ho, hm = C.c_int(), C.c_int()
        self._check(lib().aloam_pipeline_push(self.h, ptr, cnt, flags, C.byref(od), C.byref(ho), C.byref(mp), C.byref(hm)))
        # the scan is read until the next push / flush completes it (2 stages): keep a host array alive
        self._held = pts if device_ptr is None else None
        if self._profiling:
            self.last_front_timing = self._timing(0)
            self.last_odom_timing = self._timing(1)
            self.last_back_timing = self._timing(2)
        return ((abi.LazyResult(od, abi.odom_to_dict) if ho.value else None),
                (abi.LazyResult(mp, abi.map_to_dict) if hm.value else None))

    def flush(self):
        """Drain the pipeline: the (odometry, mapping) results that complete while draining (the C call
        returns at most one odometry and two mapping results; it is repeated until nothing is left)."""
        out = []
        while True:
            od, mp, mp2 = abi.OdomResult(), abi.MapResult(), abi.MapResult()
            ho, hm, hm2 = C.c_int(), C.c_int(), C.c_int()
            self._check(lib().aloam_pipeline_flush(self.h, C.byref(od), C.byref(ho), C.byref(mp), C.byref(hm),
                                                   C.byref(mp2), C.byref(hm2)))
            if self._profiling:
                self.last_back_timing = self._timing(2)
            if hm.value:
                out.append((None, abi.map_to_dict(mp)))
            if ho.value:
                out.append((abi.odom_to_dict(od), abi.map_to_dict(mp2) if hm2.value else None))
            elif hm2.value:
                out.append((None, abi.map_to_dict(mp2)))
            if not (ho.value or hm.value or hm2.value):
                break
        self._held = None
        return out

    def close(self):
        if getattr(self, "h", None):
            self.flush()
            lib().aloam_pipeline_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
