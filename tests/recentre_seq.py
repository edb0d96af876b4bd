"""Teacher-forced mapping sequences that drive laserMapping's cube recentring (laserMapping.cpp:325-507).

Mapping inputs are the oracle's scanRegistration features of synthetic HDL-64 frames with their
ground-truth poses (synth.pose: p_scene = R p_sensor + o), mapped through a global rigid transform
(Rg, delta) so the vehicle's +x travel (1 m/frame) points along the chosen axis and starts half a
metre short of the recentring threshold (|x|,|y| >= 375 m with 21x21 cubes centred at 10; |z| >= 125 m
with 11 cubes centred at 5). The frame list then jumps far enough (e.g. 109 m) that one frame moves
the cube centre twice while the grid already holds map points. Test infrastructure (oracle only).
"""
import functools

import numpy as np

import oracle_binding as ob
from lvo_amd_loader import abi, synth

FRAMES = (0, 1, 40, 41, 150, 151)


def _rot(axis):
    """Rg mapping the vehicle's +x travel onto axis ('+x', '-x', '+y', '-y', '+z', '-z')."""
    c = {"+x": np.eye(3),
         "-x": np.diag([-1.0, -1.0, 1.0]),
         "+y": np.array([[0.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]]),
         "-y": np.array([[0.0, 1.0, 0.0], [-1.0, 0.0, 0.0], [0.0, 0.0, 1.0]]),
         "+z": np.array([[0.0, 0.0, -1.0], [0.0, 1.0, 0.0], [1.0, 0.0, 0.0]]),
         "-z": np.array([[0.0, 0.0, 1.0], [0.0, 1.0, 0.0], [-1.0, 0.0, 0.0]])}
    return c[axis]


def _quat(R):
    """Rotation matrix -> unit quaternion (x, y, z, w), w >= 0."""
    t = np.trace(R)
    if t > 0:
        s = 2.0 * np.sqrt(t + 1.0)
        q = np.array([(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s])
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = 2.0 * np.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k])
        q = np.zeros(4)
        q[i] = 0.25 * s
        q[j] = (R[j, i] + R[i, j]) / s
        q[k] = (R[k, i] + R[i, k]) / s
        q[3] = (R[k, j] - R[j, k]) / s
    q /= np.linalg.norm(q)
    return q if q[3] >= 0 else -q


def sequence(axis, frames=FRAMES, name="hdl64"):
    """[(corner, surf, q_wodom_curr, t_wodom_curr)] for the frames, start 0.5 m before the threshold."""
    Rg = _rot(axis)
    along = "xyz".index(axis[1])
    lim = 125.0 if axis[1] == "z" else 375.0
    sign = 1.0 if axis[0] == "+" else -1.0
    delta = np.zeros(3)
    R0, o0 = synth.pose(name, frames[0])
    delta[along] = sign * (lim - 0.5) - (Rg @ o0)[along]
    out = []
    for k in frames:
        corner, surf = _features(name, k)
        R, o = synth.pose(name, k)
        out.append((corner, surf, _quat(Rg @ R), Rg @ o + delta))
    return out


@functools.lru_cache(maxsize=None)
def _features(name, k):
    orc = ob.Oracle(abi.default_params(synth.SCAN_LINES[name]))
    orc.scan_registration(synth.scan(name, k))
    f = orc.features()
    return f["less_sharp"], f["less_flat"]


AXES = ("+x", "-x", "+y", "-y", "+z", "-z")
