"""Seeded synthetic lidar sweeps in the KITTI velodyne .bin layout.

The ray caster is C (tools/synth_scan.c -> tools/libaloam_synth.so, built by
``__graft_entry__.build()``), so a 100k-point HDL-64 sweep takes tens of milliseconds and is
bit-identical on this container and on the GPU box.

Configs (BASELINE.json ``configs``):
  * ``vlp16``  — C1: VLP-16, 1,800 azimuths (~29k points)
  * ``hdl64``  — C2/C3: HDL-64E elevation table of scanRegistration.cpp:189-192, 2,083 azimuths
                 (~100-125k points after the 5 m minimum range)
  * ``l128``   — C4: 128 lines uniform -25..+15 deg, 1,875 azimuths (~240k points)
  * ``c5``     — C5 stand-in: HDL-64E, 271 frames of a straight road (seed 5; KITTI-04 is not on the box)
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "tools", "libaloam_synth.so")


class SynthConfig(C.Structure):
    _fields_ = [("model", C.c_int), ("n_azimuth", C.c_int), ("range_sigma", C.c_double),
                ("max_range", C.c_double), ("seed", C.c_ulonglong), ("speed", C.c_double),
                ("yaw_amp_deg", C.c_double)]


PRESETS = {
    "vlp16": dict(model=16, n_azimuth=1800, range_sigma=0.02, max_range=100.0, seed=1, speed=1.0, yaw_amp_deg=2.0),
    "hdl64": dict(model=64, n_azimuth=2083, range_sigma=0.02, max_range=120.0, seed=2, speed=1.0, yaw_amp_deg=2.0),
    "l128": dict(model=128, n_azimuth=1875, range_sigma=0.02, max_range=120.0, seed=4, speed=1.0, yaw_amp_deg=2.0),
    # C5 stand-in (KITTI-04 is 271 frames of a straight road; no KITTI data on the box)
    "c5": dict(model=64, n_azimuth=2083, range_sigma=0.02, max_range=120.0, seed=5, speed=1.0, yaw_amp_deg=0.0),
}
SCAN_LINES = {"vlp16": 16, "hdl64": 64, "l128": 128, "c5": 64}
C5_FRAMES = 271

_lib = None


def build_lib(force=False):
    src = os.path.join(_HERE, "tools", "synth_scan.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        rc = os.system(f"gcc -O2 -ffp-contract=off -fPIC -shared -o {_LIB} {src} -lm")
        if rc != 0:
            raise RuntimeError("building libaloam_synth.so failed")
    return _LIB


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build_lib()
        _lib = C.CDLL(_LIB)
        _lib.synth_generate.restype = C.c_int
        _lib.synth_generate.argtypes = [C.POINTER(SynthConfig), C.c_int, C.POINTER(C.c_float), C.c_int]
        _lib.synth_pose.restype = None
        _lib.synth_pose.argtypes = [C.POINTER(SynthConfig), C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        _lib.synth_dense_map.restype = C.c_int
        _lib.synth_dense_map.argtypes = [C.c_ulonglong, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                         C.POINTER(C.c_float), C.c_int]
    return _lib


def config(name, **over):
    d = dict(PRESETS[name])
    d.update(over)
    return SynthConfig(**d)


def scan(name, frame, **over):
    """One sweep: float32 array (n, 4) of x, y, z, reflectance in the sensor frame."""
    lib = _load()
    cfg = config(name, **over)
    cap = cfg.model * cfg.n_azimuth
    out = np.empty((cap, 4), np.float32)
    n = lib.synth_generate(C.byref(cfg), int(frame), out.ctypes.data_as(C.POINTER(C.c_float)), cap)
    if n < 0:
        raise RuntimeError("synth capacity")
    return out[:n].copy()


def sequence(name, n_frames, start=0, **over):
    return [scan(name, start + k, **over) for k in range(n_frames)]


def pose(name, frame, **over):
    """Ground-truth sensor pose (R 3x3, origin 3) of a frame in the scene frame."""
    lib = _load()
    cfg = config(name, **over)
    R = (C.c_double * 9)()
    o = (C.c_double * 3)()
    lib.synth_pose(C.byref(cfg), int(frame), R, o)
    return np.array(R[:]).reshape(3, 3), np.array(o[:])


def dense_map(seed, cx, cy, half=50.0, step=0.15, noise=0.01, max_pts=4_000_000):
    lib = _load()
    out = np.empty((max_pts, 4), np.float32)
    n = lib.synth_dense_map(int(seed), cx, cy, half, step, noise, out.ctypes.data_as(C.POINTER(C.c_float)), max_pts)
    return out[:n].copy()


def write_kitti_bin(path, pts):
    """KITTI velodyne .bin: float32 x, y, z, r (src/kittiHelper.cpp:25-35)."""
    np.asarray(pts, np.float32).reshape(-1, 4).tofile(path)


def read_kitti_bin(path):
    return np.fromfile(path, dtype=np.float32).reshape(-1, 4)


def quat_from_rot(R):
    """Unit quaternion (x, y, z, w) of a rotation matrix (Eigen's Quaternion(Matrix3) branch rule)."""
    R = np.asarray(R, np.float64)
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = np.sqrt(tr + 1.0)
        w = 0.5 * s
        s = 0.5 / s
        q = [(R[2, 1] - R[1, 2]) * s, (R[0, 2] - R[2, 0]) * s, (R[1, 0] - R[0, 1]) * s, w]
    else:
        i = int(np.argmax([R[0, 0], R[1, 1], R[2, 2]]))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q = [0.0, 0.0, 0.0, 0.0]
        q[i] = 0.5 * s
        s = 0.5 / s
        q[3] = (R[k, j] - R[j, k]) * s
        q[j] = (R[j, i] + R[i, j]) * s
        q[k] = (R[k, i] + R[i, k]) * s
    return np.array(q)


def c4_registration(name="l128", frame=0, half=50.0, map_step=0.107, seed=4, surf_stride=1, corner_stride=8,
                    dyaw_deg=1.0, dt=(0.3, -0.2, 0.05)):
    """BASELINE configs[3] registration workload: one sweep (sensor frame) as the query stacks against a
    dense local map of the scene around the sensor (map frame = scene frame), starting from the true
    pose perturbed by dyaw_deg of yaw and dt metres. Corner stack = every corner_stride-th point, surf
    stack = every surf_stride-th point (surf_stride 1: the whole sweep, the C4 stress set); both map
    kinds are the dense map. Returns (corner_map, surf_map, corner_q, surf_q, x0, x_true)."""
    R, o = pose(name, frame)
    m = dense_map(seed, float(o[0]), float(o[1]), half=half, step=map_step)
    s = scan(name, frame)
    qt = quat_from_rot(R)
    x_true = np.concatenate([qt, o])
    a = np.deg2rad(dyaw_deg) / 2
    dq = np.array([0.0, 0.0, np.sin(a), np.cos(a)])
    x, y, z, w = dq
    X, Y, Z, W = qt
    q0 = np.array([w * X + x * W + y * Z - z * Y, w * Y - x * Z + y * W + z * X, w * Z + x * Y - y * X + z * W,
                   w * W - x * X - y * Y - z * Z])
    x0 = np.concatenate([q0 / np.linalg.norm(q0), o + np.asarray(dt, np.float64)])
    return m, m, np.ascontiguousarray(s[::corner_stride]), np.ascontiguousarray(s[::surf_stride]), x0, x_true


def to_pointcloud2(pts, point_step=32, seed=0):
    """A sensor_msgs/PointCloud2 data blob of a sweep: x, y, z float32 at byte offsets 0, 4, 8 and,
    when the record has room, intensity at 16 (pcl::PointXYZI, point_step 32) or 12; every other byte
    is filled with seeded noise so a reader that touches them is caught."""
    pts = np.asarray(pts, np.float32).reshape(-1, 4)
    n = len(pts)
    rec = np.random.default_rng(seed).integers(0, 256, size=(n, point_step), dtype=np.uint8)
    rec[:, 0:12] = pts[:, :3].view(np.uint8).reshape(n, 12)
    off = 16 if point_step >= 20 else (12 if point_step >= 16 else None)
    if off is not None:
        rec[:, off:off + 4] = pts[:, 3:4].view(np.uint8).reshape(n, 4)
    return rec.tobytes()
