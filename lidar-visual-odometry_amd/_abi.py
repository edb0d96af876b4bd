"""ctypes mirror of include/aloam_hip.h (the C ABI of the HIP hot path).

Kept in one place so the product binding (``__init__.py``) and the test-only oracle binding
(``tests/oracle_binding.py``) describe the same structs.
"""
import ctypes as C
from collections.abc import Mapping

import numpy as np

ALOAM_OK = 0
ALOAM_E_ARG = -1
ALOAM_E_CAPACITY = -2
ALOAM_E_HIP = -3
ALOAM_E_SCAN_LINES = -4
ALOAM_E_STATE = -5
ALOAM_E_NODEVICE = -6
ALOAM_INPUT_DEVICE = 1
ALOAM_NO_MAPPING = 2
ALOAM_MAX_ROUNDS = 16


class Params(C.Structure):
    _fields_ = [
        ("scan_line", C.c_int),
        ("minimum_range", C.c_float),
        ("mapping_skip_frame", C.c_int),
        ("mapping_line_resolution", C.c_float),
        ("mapping_plane_resolution", C.c_float),
        ("input_is_dense", C.c_int),
        ("generic_scan_lines", C.c_int),
        ("generic_min_elev_deg", C.c_float),
        ("generic_max_elev_deg", C.c_float),
        ("odom_rounds", C.c_int),
        ("map_rounds", C.c_int),
        ("max_solver_iterations", C.c_int),
        ("max_scan_points", C.c_int),
        ("max_map_points", C.c_int),
    ]


def default_params(scan_line=64):
    """The launch-file values (launch/aloam_velodyne_{VLP_16,HDL_32,HDL_64}.launch:3-13)."""
    p = Params()
    p.scan_line = scan_line
    p.minimum_range = 5.0 if scan_line == 64 else 0.3
    p.mapping_skip_frame = 1
    p.mapping_line_resolution = 0.4 if scan_line == 64 else 0.2
    p.mapping_plane_resolution = 0.8 if scan_line == 64 else 0.4
    p.input_is_dense = 1
    p.generic_scan_lines = 0 if scan_line in (16, 32, 64) else 1
    p.generic_min_elev_deg = -25.0
    p.generic_max_elev_deg = 15.0
    p.odom_rounds = 10
    p.map_rounds = 10
    p.max_solver_iterations = 4
    p.max_scan_points = 400000
    p.max_map_points = 4000000
    return p


class Cloud(C.Structure):
    _fields_ = [("pts", C.POINTER(C.c_float)), ("n", C.c_int), ("cap", C.c_int)]


class Features(C.Structure):
    _fields_ = [
        ("full", Cloud), ("sharp", Cloud), ("less_sharp", Cloud), ("flat", Cloud), ("less_flat", Cloud),
        ("sharp_idx", C.POINTER(C.c_int)), ("less_sharp_idx", C.POINTER(C.c_int)),
        ("flat_idx", C.POINTER(C.c_int)), ("curvature", C.POINTER(C.c_float)),
    ]


class LMSummary(C.Structure):
    _fields_ = [
        ("iterations", C.c_int), ("successful_steps", C.c_int), ("termination", C.c_int),
        ("num_residual_blocks", C.c_int), ("initial_cost", C.c_double), ("final_cost", C.c_double),
    ]


class OdomResult(C.Structure):
    _fields_ = [
        ("q_w_curr", C.c_double * 4), ("t_w_curr", C.c_double * 3),
        ("q_last_curr", C.c_double * 4), ("t_last_curr", C.c_double * 3),
        ("optimized", C.c_int), ("rounds", C.c_int),
        ("corner_correspondence", C.c_int * ALOAM_MAX_ROUNDS),
        ("plane_correspondence", C.c_int * ALOAM_MAX_ROUNDS),
        ("lm", LMSummary * ALOAM_MAX_ROUNDS),
        ("publish_to_mapping", C.c_int),
    ]


class MapResult(C.Structure):
    _fields_ = [
        ("q_w_curr", C.c_double * 4), ("t_w_curr", C.c_double * 3),
        ("optimized", C.c_int), ("map_corner_num", C.c_int), ("map_surf_num", C.c_int),
        ("corner_stack_num", C.c_int), ("surf_stack_num", C.c_int), ("rounds", C.c_int),
        ("corner_num", C.c_int * ALOAM_MAX_ROUNDS), ("surf_num", C.c_int * ALOAM_MAX_ROUNDS),
        ("lm", LMSummary * ALOAM_MAX_ROUNDS),
        ("map_total_points", C.c_int),
        ("q_wmap_wodom", C.c_double * 4), ("t_wmap_wodom", C.c_double * 3),
        ("frame_count", C.c_int), ("pub_surround", C.c_int), ("pub_map", C.c_int),
        ("uncached_queries", C.c_int),
    ]


ALOAM_S2M_RECORDS = 256


class S2MResult(C.Structure):
    _fields_ = [
        ("q_w_curr", C.c_double * 4), ("t_w_curr", C.c_double * 3),
        ("optimized", C.c_int), ("rounds", C.c_int),
        ("corner_num", C.c_int * ALOAM_MAX_ROUNDS), ("surf_num", C.c_int * ALOAM_MAX_ROUNDS),
        ("lm", LMSummary * ALOAM_MAX_ROUNDS),
        ("slot_begin", C.c_int), ("slot_end", C.c_int), ("world", C.c_int),
    ]


class Factor(C.Structure):
    _fields_ = [("type", C.c_int), ("pad", C.c_int),
                ("cp", C.c_double * 3), ("a", C.c_double * 3), ("b", C.c_double * 3)]


FACTOR_DTYPE = np.dtype([("type", "<i4"), ("pad", "<i4"), ("cp", "<f8", 3), ("a", "<f8", 3), ("b", "<f8", 3)])
assert FACTOR_DTYPE.itemsize == C.sizeof(Factor) == 80


class Timing(C.Structure):
    _fields_ = [
        ("scan_registration_ms", C.c_float), ("odometry_ms", C.c_float), ("mapping_ms", C.c_float),
        ("odom_search_ms", C.c_float), ("map_search_ms", C.c_float),
        ("odom_search_launches", C.c_int), ("map_search_launches", C.c_int),
        ("map_search_bytes", C.c_double), ("odom_search_bytes", C.c_double),
        ("knn_ms", C.c_float), ("knn_launches", C.c_int), ("knn_bytes", C.c_double), ("knn_streamed_bytes", C.c_double),
        ("knn_build_ms", C.c_float),
        ("tictoc_ms", C.c_float * 17),
    ]


def timing_to_dict(t):
    """aloam_timing -> dict (tictoc_ms as a list in ALOAM_TT_* order, see TICTOC_NAMES)."""
    d = {k: getattr(t, k) for k, _ in Timing._fields_}
    d["tictoc_ms"] = list(d["tictoc_ms"])
    return d


# the reference's TicToc stage names (include/aloam_hip.h ALOAM_TT_*), in tictoc_ms order
TICTOC_NAMES = ["prepare time", "seperate points time", "scan registration time", "data association time", "solver time",
                "optimization twice time", "publication time", "whole laserOdometry time", "map prepare time",
                "build tree time", "mapping data assosiation time", "mapping solver time", "mapping optimization time",
                "add points time", "filter time", "mapping pub time", "whole mapping time"]


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def iptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def make_cloud(cap):
    buf = np.zeros((max(cap, 1), 4), np.float32)
    c = Cloud(fptr(buf), 0, cap)
    return c, buf


class LazyResult(Mapping):
    """Read-only mapping over a result struct, converted on first use: the pipeline returns one per
    stage per scan, and building every list/array eagerly sat between one scan's completion and the
    next scan's launches. The pose keys are read straight from the struct; any other access converts
    the whole struct once (the dict odom_to_dict / map_to_dict would have built)."""
    __slots__ = ("_raw", "_conv", "_d")
    _POSE = ("q_w_curr", "t_w_curr")

    def __init__(self, raw, conv):
        self._raw, self._conv, self._d = raw, conv, None

    def _full(self):
        if self._d is None:
            self._d = self._conv(self._raw)
        return self._d

    def __getitem__(self, k):
        if self._d is None and k in self._POSE:
            return np.array(getattr(self._raw, k)[:])
        return self._full()[k]

    def __iter__(self):
        return iter(self._full())

    def __len__(self):
        return len(self._full())

    def __repr__(self):
        return repr(self._full())


def odom_to_dict(r):
    n = r.rounds
    return {
        "q_w_curr": np.array(r.q_w_curr[:]), "t_w_curr": np.array(r.t_w_curr[:]),
        "q_last_curr": np.array(r.q_last_curr[:]), "t_last_curr": np.array(r.t_last_curr[:]),
        "optimized": r.optimized, "rounds": n,
        "corner_correspondence": list(r.corner_correspondence[:n]),
        "plane_correspondence": list(r.plane_correspondence[:n]),
        "lm": [(r.lm[i].iterations, r.lm[i].successful_steps, r.lm[i].termination,
                r.lm[i].num_residual_blocks, r.lm[i].initial_cost, r.lm[i].final_cost) for i in range(n)],
        "publish_to_mapping": r.publish_to_mapping,
    }


def map_to_dict(r):
    n = r.rounds
    return {
        "q_w_curr": np.array(r.q_w_curr[:]), "t_w_curr": np.array(r.t_w_curr[:]),
        "optimized": r.optimized, "map_corner_num": r.map_corner_num, "map_surf_num": r.map_surf_num,
        "corner_stack_num": r.corner_stack_num, "surf_stack_num": r.surf_stack_num, "rounds": n,
        "corner_num": list(r.corner_num[:n]), "surf_num": list(r.surf_num[:n]),
        "lm": [(r.lm[i].iterations, r.lm[i].successful_steps, r.lm[i].termination,
                r.lm[i].num_residual_blocks, r.lm[i].initial_cost, r.lm[i].final_cost) for i in range(n)],
        "map_total_points": r.map_total_points,
        "q_wmap_wodom": np.array(r.q_wmap_wodom[:]), "t_wmap_wodom": np.array(r.t_wmap_wodom[:]),
        "frame_count": r.frame_count, "pub_surround": r.pub_surround, "pub_map": r.pub_map,
        "uncached_queries": r.uncached_queries,
    }


def s2m_to_dict(r):
    n = r.rounds
    return {
        "q_w_curr": np.array(r.q_w_curr[:]), "t_w_curr": np.array(r.t_w_curr[:]),
        "x": np.array(r.q_w_curr[:] + r.t_w_curr[:]),
        "optimized": r.optimized, "rounds": n,
        "corner_num": list(r.corner_num[:n]), "surf_num": list(r.surf_num[:n]),
        "lm": [(r.lm[i].iterations, r.lm[i].successful_steps, r.lm[i].termination,
                r.lm[i].num_residual_blocks, r.lm[i].initial_cost, r.lm[i].final_cost) for i in range(n)],
        "slot_begin": r.slot_begin, "slot_end": r.slot_end, "world": r.world,
    }
