"""GPU: laserMapping's publication surface and the map at grown sizes, through the C ABI against the oracle.

* /aft_mapped_to_init_high_frec (laserMapping.cpp:197-229) and the surround / map publish cadence
  (:806, :823, frameCount :888) — aloam_map_result.{q,t}_wmap_wodom, frame_count, pub_surround, pub_map
  and aloam_map_high_freq_pose.
* The whole cube map bit for bit against the PCL-order oracle after long sequences, where touched cubes
  hold thousands of points and the per-cube VoxelGrid (laserMapping.cpp:788-801) takes its split and
  heap-sort paths.
"""
import numpy as np
import pytest

import oracle_binding as ob
from lvo_amd_loader import abi, lvo, synth

pytestmark = pytest.mark.gpu

POSE_RTOL = 1e-6


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _qmul(a, b):
    """Eigen's double quaternion product, quat_product<SSE> operation order (aloam_device.hpp qmul)."""
    ax, ay, az, aw = (float(v) for v in a)
    bx, by, bz, bw = (float(v) for v in b)
    return [(aw * bx + ay * bz) - (az * by - ax * bw), (aw * by + ay * bw) + (az * bx - ax * bz),
            (aw * bz - ay * bx) + (az * bw + ax * by), (aw * bw - ay * by) - (az * bz + ax * bx)]


def _qrot(q, v):
    """QuaternionBase::_transformVector (Quaternion.h:476-485) in its operation order."""
    qx, qy, qz, qw = (float(c) for c in q)
    vx, vy, vz = (float(c) for c in v)
    ux, uy, uz = qy * vz - qz * vy, qz * vx - qx * vz, qx * vy - qy * vx
    ux, uy, uz = ux + ux, uy + uy, uz + uz
    cx, cy, cz = qy * uz - qz * uy, qz * ux - qx * uz, qx * uy - qy * ux
    return [vx + qw * ux + cx, vy + qw * uy + cy, vz + qw * uz + cz]


def test_mapping_publication_surface(gpu_ctx_factory):
    """25 frames: every frame's frameCount and publish flags equal the reference cadence (surround every 5,
    map every 20); the exported odometry->map correction q/t_wmap_wodom matches the oracle's transformUpdate
    (pose bar); aloam_map_high_freq_pose of the next frame's odometry pose is bit for bit the reference's
    formula (laserMapping.cpp:212-213) applied to that correction, and within the pose bar of the oracle's."""
    ctx = gpu_ctx_factory(16)
    orc = ob.Oracle(abi.default_params(16))
    frames = synth.sequence("vlp16", 25)
    # before any mapping frame: identity correction
    q0, t0 = ctx.high_freq_pose([0.1, 0.2, 0.3, np.sqrt(1 - 0.14)], [1.0, 2.0, 3.0])
    np.testing.assert_array_equal(q0, [0.1, 0.2, 0.3, np.sqrt(1 - 0.14)])
    np.testing.assert_array_equal(t0, [1.0, 2.0, 3.0])
    for k, pts in enumerate(frames):
        og, mg = ctx.process_scan(pts)
        oo, mo = orc.process_scan(pts)
        assert mg["frame_count"] == mo["frame_count"] == k, (k, mg["frame_count"], mo["frame_count"])
        assert mg["pub_surround"] == mo["pub_surround"] == int(k % 5 == 0), k
        assert mg["pub_map"] == mo["pub_map"] == int(k % 20 == 0), k
        np.testing.assert_allclose(mg["q_wmap_wodom"], mo["q_wmap_wodom"], rtol=POSE_RTOL, atol=1e-9, err_msg=str(k))
        np.testing.assert_allclose(mg["t_wmap_wodom"], mo["t_wmap_wodom"], rtol=POSE_RTOL, atol=1e-7, err_msg=str(k))
        # high-frequency pose of an odometry pose (this frame's own laser_odom_to_init)
        qg, tg = ctx.high_freq_pose(og["q_w_curr"], og["t_w_curr"])
        q_ref = _qmul(mg["q_wmap_wodom"], og["q_w_curr"])
        r = _qrot(mg["q_wmap_wodom"], og["t_w_curr"])
        t_ref = [r[i] + float(mg["t_wmap_wodom"][i]) for i in range(3)]
        assert np.array_equal(np.array(qg).view(np.uint64), np.array(q_ref).view(np.uint64)), (k, qg, q_ref)
        assert np.array_equal(np.array(tg).view(np.uint64), np.array(t_ref).view(np.uint64)), (k, tg, t_ref)
        qo, to = orc.high_freq_pose(oo["q_w_curr"], oo["t_w_curr"])
        np.testing.assert_allclose(qg, qo, rtol=POSE_RTOL, atol=1e-9)
        np.testing.assert_allclose(tg, to, rtol=POSE_RTOL, atol=1e-7)
        # the mapped pose itself is this frame's high-frequency pose of its own odometry pose (the
        # correction was computed from exactly these two poses, transformUpdate :148-152)
        np.testing.assert_allclose(tg, mg["t_w_curr"], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("name,n_frames", [("hdl64", 200), ("c5", 100)])
def test_map_bit_exact_after_sequence(gpu_ctx_factory, name, n_frames):
    """The whole cube map (every cube's points in cube order) and the surround after a free-running
    sequence equal the PCL-order oracle's bit for bit. By the end touched cubes hold thousands of points
    (corner cubes > 10k), so the map filter's split cubes, segment sorts and heap-sorted (depth-exhausted)
    introsort segments all run; the trajectories agree to ~1e-16 m, far below the float rounding of the
    inserted points."""
    ctx = gpu_ctx_factory(64)
    orc = ob.Oracle(abi.default_params(64))
    serial0 = lvo.serial_sort_fallbacks()
    big = 0
    for k in range(n_frames):
        pts = synth.scan(name, k)
        _, mg = ctx.process_scan(pts)
        _, mo = orc.process_scan(pts)
        assert mg["map_total_points"] == mo["map_total_points"], (k, mg["map_total_points"], mo["map_total_points"])
        big = max(big, mo["map_corner_num"])
    for which in (0, 1):
        g, o = ctx.map_cloud(which), orc.map_cloud(which)
        assert g.shape == o.shape, (which, g.shape, o.shape)
        nd = int(np.sum(np.any(bits(g) != bits(o), axis=1)))
        assert nd == 0, f"map {which}: {nd} of {len(o)} points differ"
    assert big > 10000, big
    # every line, stack and cube sort stayed on the workgroup replay (no one-thread fallback)
    assert lvo.serial_sort_fallbacks() == serial0
