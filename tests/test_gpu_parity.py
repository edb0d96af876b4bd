"""GPU parity: the HIP path through the C ABI against the CPU oracle on identical seeded inputs.

Bars (BASELINE.json north_star): bit-exact feature indices / laserCloud / curvature; poses within
1e-6 relative; per-factor residuals and Jacobians within 1e-9 relative (fp64, different op order).
"""
import numpy as np
import pytest

import oracle_binding as ob
from lvo_amd_loader import abi, lvo, synth

pytestmark = pytest.mark.gpu

POSE_RTOL = 1e-6


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def assert_features_equal(fg, fo, less_flat_exact=True):
    for k in ("sharp_idx", "less_sharp_idx", "flat_idx"):
        assert np.array_equal(fg[k], fo[k]), f"{k}: {len(fg[k])} vs {len(fo[k])}"
    for k in ("full", "sharp", "less_sharp", "flat"):
        assert np.array_equal(bits(fg[k]), bits(fo[k])), k
    assert np.array_equal(bits(fg["curvature"]), bits(fo["curvature"])), "curvature"
    assert len(fg["less_flat"]) == len(fo["less_flat"])
    if less_flat_exact:
        assert np.array_equal(bits(fg["less_flat"]), bits(fo["less_flat"])), "less_flat"


@pytest.mark.parametrize("name,frame", [("vlp16", 0), ("vlp16", 7), ("hdl64", 0), ("hdl64", 3), ("l128", 0)])
def test_scan_registration_bit_exact(gpu_ctx_factory, name, frame):
    lines = synth.SCAN_LINES[name]
    ctx = gpu_ctx_factory(lines)
    orc = ob.Oracle(abi.default_params(lines))
    pts = synth.scan(name, frame)
    ctx.scan_registration(pts)
    orc.scan_registration(pts)
    assert_features_equal(ctx.features(), orc.features())


def test_scan_registration_edge_cases(gpu_ctx_factory):
    ctx = gpu_ctx_factory(16)
    orc = ob.Oracle(abi.default_params(16))
    pts = synth.scan("vlp16", 1)
    # NaNs + points inside the minimum range + an empty cloud
    bad = pts.copy()
    bad[::97, 0] = np.nan
    bad[5::101, :3] *= 0.001
    ctx2 = gpu_ctx_factory(16, input_is_dense=0)
    p = abi.default_params(16)
    p.input_is_dense = 0
    orc2 = ob.Oracle(p)
    ctx2.scan_registration(bad)
    orc2.scan_registration(bad)
    assert_features_equal(ctx2.features(), orc2.features())
    # tiny cloud (fewer points than one segment)
    small = pts[:40]
    ctx.scan_registration(small)
    orc.scan_registration(small)
    assert_features_equal(ctx.features(), orc.features())
    ctx.scan_registration(pts[:0])
    assert ctx.feature_counts() == [0, 0, 0, 0, 0]


def test_unsupported_scan_lines_is_an_error(gpu_ctx_factory):
    """scanRegistration.cpp:201-205 aborts on N_SCANS outside {16, 32, 64}: an error code here."""
    ctx = gpu_ctx_factory(40, generic_scan_lines=0)
    with pytest.raises(lvo.ALOAMError):
        ctx.scan_registration(synth.scan("vlp16", 0))


@pytest.mark.parametrize("lines,preset,lattice", [(16, "vlp16", 20), (64, "hdl64", 20), (64, "hdl64", 100), (64, "hdl64", 1000)])
def test_tied_curvatures_follow_std_sort(gpu_ctx_factory, lines, preset, lattice):
    """Quantised coordinates create exact curvature ties: where the selection reads a tie group's sorted
    slots the order must be libstdc++'s (k_scan.hip redoes such segments and reruns the selection);
    coarse lattices put ties everywhere, fine ones only here and there."""
    ctx = gpu_ctx_factory(lines)
    orc = ob.Oracle(abi.default_params(lines))
    for k in range(2):
        q = synth.scan(preset, 2 + k).copy()
        q[:, :3] = np.round(q[:, :3] * lattice) / lattice
        ctx.scan_registration(q)
        orc.scan_registration(q)
        assert_features_equal(ctx.features(), orc.features())


def random_factors(rng, n):
    f = np.zeros(n, abi.FACTOR_DTYPE)
    f["type"] = rng.integers(0, 4, n)
    f["cp"] = rng.normal(0, 10, (n, 3))
    f["a"] = rng.normal(0, 10, (n, 3))
    f["b"] = rng.normal(0, 10, (n, 3))
    for i in range(n):
        if f["type"][i] == 1:
            v = rng.normal(size=3)
            f["b"][i] = v / np.linalg.norm(v)
        if f["type"][i] == 2:
            v = rng.normal(size=3)
            f["a"][i] = v / np.linalg.norm(v)
            f["b"][i] = [rng.normal(), 0, 0]
    return f


def random_pose(rng, scale=0.1):
    q = np.concatenate([rng.normal(0, scale, 3), [1.0]])
    q /= np.linalg.norm(q)
    return np.concatenate([q, rng.normal(0, 1, 3)])


@pytest.mark.parametrize("robust", [True, False])
def test_factor_residuals_and_jacobians(gpu_ctx_factory, robust):
    ctx = gpu_ctx_factory(64)
    rng = np.random.default_rng(5)
    f = random_factors(rng, 257)
    x = random_pose(rng)
    rg, jg, ng = ctx.eval_factors(f, x, robust)
    ro, jo, no = ob.eval_factors(f, x, robust)
    np.testing.assert_allclose(rg, ro, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(jg, jo, rtol=1e-8, atol=1e-8)
    np.testing.assert_allclose(ng, no, rtol=1e-8, atol=1e-8)


def test_lm_solve_matches_ceres_restatement(gpu_ctx_factory):
    ctx = gpu_ctx_factory(64)
    rng = np.random.default_rng(11)
    # a consistent problem: factors generated from a true pose, solved from a perturbed start
    x_true = random_pose(rng, 0.05)
    f = random_factors(rng, 300)
    res, _, _ = ob.eval_factors(f, x_true, robust=False)
    # shift plane offsets so the true pose is (nearly) a zero of the plane residuals
    for i in np.where(f["type"] == 2)[0]:
        f["b"][i][0] -= res[i, 0]
    x0 = x_true.copy()
    x0[4:] += 0.05
    xg, sg = ctx.lm_solve(f, x0)
    xo, so = ob.lm_solve(f, x0)
    assert sg[:4] == so[:4], (sg, so)
    np.testing.assert_allclose(xg, xo, rtol=1e-7, atol=1e-9)


def test_knn_radius(gpu_ctx_factory):
    ctx = gpu_ctx_factory(64)
    rng = np.random.default_rng(2)
    pts = np.zeros((20000, 4), np.float32)
    pts[:, :3] = rng.uniform(-20, 20, (20000, 3))
    q = np.zeros((3000, 4), np.float32)
    q[:, :3] = rng.uniform(-22, 22, (3000, 3))
    for k, r in ((1, 5.0), (5, 1.0), (8, 2.0)):
        ig, dg = ctx.knn(pts, q, k, r)
        io, do = ob.knn(pts, q, k, r)
        assert np.array_equal(ig, io), (k, r)
        assert np.array_equal(bits(dg), bits(do))


def test_voxel_grid_matches_pcl_semantics(gpu_ctx_factory):
    """aloam_voxel_grid vs PCL 1.8's applyFilter (the oracle, order 1 = libstdc++ std::sort of the
    (leaf, index) pairs): bit-exact centroids, across the device's three sort paths — in LDS (ls_sort.hpp,
    n <= 11264), split in global scratch then staged through LDS (11264 < n <= 65536), one-thread serial
    replay (beyond) — and degenerate key sets."""
    ctx = gpu_ctx_factory(64)
    pts = synth.scan("hdl64", 4)
    pts[:, 3] = np.arange(len(pts)) % 64 * 0.01
    serial0 = lvo.serial_sort_fallbacks()
    for n in (1, 2, 15, 16, 17, 300, 6144, 11264, 11265, 20000, 60000, len(pts)):
        for leaf in ((0.2, 0.4, 0.8) if n in (300, 20000) else (0.4,)):
            vg = ctx.voxel_grid(pts[:n], leaf)
            vp = ob.voxel_grid(pts[:n], leaf, order=1)
            assert vg.shape == vp.shape, (n, leaf)
            assert np.array_equal(bits(vg), bits(vp)), (n, leaf)
    # exactly the one cloud beyond 65,536 points took the one-thread sort, and it is counted
    assert len(pts) > 65536
    assert lvo.serial_sort_fallbacks() - serial0 == 1
    rng = np.random.default_rng(11)
    for case in ("one_leaf", "two_leaves", "sorted", "descending", "few_leaves"):
        m = 5000
        q = np.zeros((m, 4), np.float32)
        if case == "one_leaf":
            q[:, :3] = rng.uniform(0.01, 0.19, (m, 3))
        elif case == "two_leaves":
            q[:, :3] = rng.uniform(0.01, 0.19, (m, 3)) + (rng.integers(0, 2, (m, 1)) * 0.4)
        elif case == "sorted":
            q[:, 0] = np.arange(m) * 0.25 + 0.1
        elif case == "descending":
            q[:, 0] = (m - np.arange(m)) * 0.25 + 0.1
        else:
            q[:, :3] = rng.integers(0, 4, (m, 3)) * 0.2 + rng.uniform(0.01, 0.19, (m, 3))
        q[:, 3] = rng.uniform(0, 1, m)
        vg = ctx.voxel_grid(q, 0.2)
        vp = ob.voxel_grid(q, 0.2, order=1)
        assert np.array_equal(bits(vg), bits(vp)), case


def teacher_forced_odometry_inputs(name, k):
    """Features of frames k-1 and k from the oracle (identical inputs for both sides)."""
    lines = synth.SCAN_LINES[name]
    o = ob.Oracle(abi.default_params(lines))
    o.scan_registration(synth.scan(name, k - 1))
    prev = o.features()
    o.scan_registration(synth.scan(name, k))
    cur = o.features()
    return prev, cur


@pytest.mark.parametrize("name,k,shuffled", [("vlp16", 3, False), ("hdl64", 2, False), ("vlp16", 4, True)])
def test_odometry_frame_teacher_forced(gpu_ctx_factory, name, k, shuffled):
    """shuffled: last clouds not ordered by scan line -> the device must fall back from the grid
    window search to the literal forward/backward scan and still match the reference loop."""
    lines = synth.SCAN_LINES[name]
    prev, cur = teacher_forced_odometry_inputs(name, k)
    if shuffled:
        rng = np.random.default_rng(5)
        prev = dict(prev)
        prev["less_sharp"] = prev["less_sharp"][rng.permutation(len(prev["less_sharp"]))]
        prev["less_flat"] = prev["less_flat"][rng.permutation(len(prev["less_flat"]))]
    q0 = np.array([0.001, -0.002, 0.003, 1.0]); q0 /= np.linalg.norm(q0)
    t0 = np.array([0.9, 0.02, 0.01])
    qw = np.array([0, 0, 0, 1.0]); tw = np.zeros(3)
    ctx = gpu_ctx_factory(lines)
    orc = ob.Oracle(abi.default_params(lines))
    for side in (ctx, orc):
        side.set_odom_state(q0, t0, qw, tw, prev["less_sharp"], prev["less_flat"])
        side.set_features(cur["sharp"], cur["less_sharp"], cur["flat"], cur["less_flat"])
    rg = ctx.odometry()
    ro = orc.odometry()
    assert rg["corner_correspondence"] == ro["corner_correspondence"]
    assert rg["plane_correspondence"] == ro["plane_correspondence"]
    for key in ("q_last_curr", "t_last_curr", "q_w_curr", "t_w_curr"):
        np.testing.assert_allclose(rg[key], ro[key], rtol=POSE_RTOL, atol=1e-9, err_msg=key)
    assert [l[:4] for l in rg["lm"]] == [l[:4] for l in ro["lm"]]


def test_mapping_frames_teacher_forced(gpu_ctx_factory):
    """Three mapping frames from identical odometry outputs (map built on device vs oracle)."""
    name = "hdl64"
    o = ob.Oracle(abi.default_params(64))
    frames = []
    for k in range(4):
        od, _ = o.process_scan(synth.scan(name, k))
        f = o.features()
        frames.append((f["less_sharp"], f["less_flat"], od["q_w_curr"], od["t_w_curr"]))
    ctx = gpu_ctx_factory(64)
    orc = ob.Oracle(abi.default_params(64))
    for k, (c, s, q, t) in enumerate(frames):
        ctx.set_mapping_input(c, s, q, t)
        orc.set_mapping_input(c, s, q, t)
        mg = ctx.mapping()
        mo = orc.mapping()
        for key in ("optimized", "map_corner_num", "map_surf_num", "corner_stack_num", "surf_stack_num",
                    "corner_num", "surf_num", "map_total_points"):
            assert mg[key] == mo[key], (k, key, mg[key], mo[key])
        np.testing.assert_allclose(mg["q_w_curr"], mo["q_w_curr"], rtol=POSE_RTOL, atol=1e-9)
        np.testing.assert_allclose(mg["t_w_curr"], mo["t_w_curr"], rtol=POSE_RTOL, atol=1e-7)
    mc_g = ctx.map_cloud(1)
    mc_o = orc.map_cloud(1)
    assert mc_g.shape == mc_o.shape
    assert np.array_equal(bits(mc_g), bits(mc_o)), int(np.sum(bits(mc_g) != bits(mc_o)))


@pytest.mark.parametrize("axis", ["+x", "-x", "+y", "-y", "+z", "-z"])
def test_mapping_cube_recentring(gpu_ctx_factory, axis):
    """Cube recentring (laserMapping.cpp:325-507) on the device: teacher-forced frames cross the +-x, +-y
    (375 m) / +-z (125 m) thresholds while the grid holds points, one frame shifting twice
    (tests/recentre_seq.py). Every frame's counts and pose, and the whole cube grid (every cube's points
    in cube order) match the oracle bit for bit."""
    import recentre_seq
    ctx = gpu_ctx_factory(64)
    orc = ob.Oracle(abi.default_params(64))
    cen = []
    for k, (c, s, q, t) in enumerate(recentre_seq.sequence(axis)):
        ctx.set_mapping_input(c, s, q, t)
        orc.set_mapping_input(c, s, q, t)
        mg = ctx.mapping()
        mo = orc.mapping()
        for key in ("optimized", "map_corner_num", "map_surf_num", "corner_stack_num", "surf_stack_num",
                    "corner_num", "surf_num", "map_total_points"):
            assert mg[key] == mo[key], (axis, k, key, mg[key], mo[key])
        np.testing.assert_allclose(mg["q_w_curr"], mo["q_w_curr"], rtol=POSE_RTOL, atol=1e-9)
        np.testing.assert_allclose(mg["t_w_curr"], mo["t_w_curr"], rtol=POSE_RTOL, atol=1e-7)
        cen.append(orc.cube_check()["cen"])
        for which in (0, 1):
            g, o = ctx.map_cloud(which), orc.map_cloud(which)
            assert g.shape == o.shape, (axis, k, which, g.shape, o.shape)
            assert np.array_equal(bits(g), bits(o)), (axis, k, which, int(np.sum(bits(g) != bits(o))))
    assert len(set(cen)) >= 4, cen


def test_pipeline_sequence_ate(gpu_ctx_factory):
    """Free-running pipeline over a short HDL-64 sequence: trajectories agree (ATE delta)."""
    ctx = gpu_ctx_factory(64)
    orc = ob.Oracle(abi.default_params(64))
    tg, to = [], []
    for k in range(6):
        pts = synth.scan("hdl64", k)
        og, mg = ctx.process_scan(pts)
        oo, mo = orc.process_scan(pts)
        assert np.array_equal(ctx.features()["less_sharp_idx"], orc.features()["less_sharp_idx"])
        tg.append(mg["t_w_curr"])
        to.append(mo["t_w_curr"])
    ate = np.sqrt(np.mean(np.sum((np.array(tg) - np.array(to)) ** 2, axis=1)))
    print(f"ATE delta vs oracle {ate:.3e} m")
    assert ate <= 1e-4, ate


@pytest.mark.gpu
def test_knn_device_c4_scale(gpu_ctx_factory):
    """C4: a 128-line sweep against a dense ~1.1M-point local map through
    aloam_knn_device; 3000 sampled queries must equal the oracle's kd-tree 5-NN (indices exact,
    distance bits exact) and every query's 5th distance must be < 1 when found."""
    import torch
    m = synth.dense_map(4, 0.0, 0.0, step=0.15)
    R, o = synth.pose("l128", 0)
    s = synth.scan("l128", 0)
    q = s.copy()
    q[:, :3] = (s[:, :3].astype(np.float64) @ R.T + o).astype(np.float32)
    dm, dq = torch.from_numpy(m).cuda(), torch.from_numpy(q).cuda()
    idx = torch.full((len(q), 5), -7, dtype=torch.int32, device="cuda")
    d2 = torch.empty((len(q), 5), dtype=torch.float32, device="cuda")
    ctx = gpu_ctx_factory(128)
    ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr(), len(q), 5, 1.0, idx.data_ptr(), d2.data_ptr())
    gi, gd = idx.cpu().numpy(), d2.cpu().numpy()
    assert (gi >= -1).all()                                   # every slot written
    sel = np.random.default_rng(1).choice(len(q), 3000, replace=False)
    oi, od = ob.knn(m, q[sel], 5, 1.0)
    assert np.array_equal(gi[sel], oi)
    ok = oi >= 0
    assert np.array_equal(gd[sel][ok].view(np.uint32), od[ok].view(np.uint32))
    assert (gd[gi[:, 4] >= 0, 4] < 1.0).all()
    # k < 5 through the same kernel: prefixes of the 5-NN lists
    idx3 = torch.empty((len(q), 3), dtype=torch.int32, device="cuda")
    d3 = torch.empty((len(q), 3), dtype=torch.float32, device="cuda")
    ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr(), len(q), 3, 1.0, idx3.data_ptr(), d3.data_ptr())
    assert np.array_equal(idx3.cpu().numpy(), gi[:, :3])


@pytest.mark.gpu
def test_knn_build_once_query_many(gpu_ctx_factory):
    """aloam_knn_build + aloam_knn_query (the kd-tree built once per map, laserMapping.cpp:558-559, queried
    every round, :582/:648): several queries against one build equal aloam_knn_device call for call (bit
    for bit), the index holds its own copy of the points (the map buffer may change after the build), a
    rebuild over another map answers for that map, and a query before any build is ALOAM_E_STATE."""
    import torch
    m = synth.dense_map(4, 0.0, 0.0, step=0.25)
    R, o = synth.pose("l128", 0)
    s = synth.scan("l128", 0)
    q = s.copy()
    q[:, :3] = (s[:, :3].astype(np.float64) @ R.T + o).astype(np.float32)
    dm, dq = torch.from_numpy(m).cuda(), torch.from_numpy(q).cuda()
    ctx = gpu_ctx_factory(128)
    with pytest.raises(lvo.ALOAMError):
        ctx.knn_query(dq.data_ptr(), len(q), 5, dq.data_ptr(), dq.data_ptr())

    def run(fn, k, n_q):
        idx = torch.full((n_q, k), -7, dtype=torch.int32, device="cuda")
        d2 = torch.full((n_q, k), -7.0, dtype=torch.float32, device="cuda")
        fn(idx, d2)
        return idx.cpu().numpy(), d2.cpu().numpy().view(np.uint32)

    ref5 = run(lambda i, d: ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr(), len(q), 5, 1.0, i.data_ptr(), d.data_ptr()), 5, len(q))
    ref3 = run(lambda i, d: ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr() + 16 * 1000, 5000, 3, 1.0, i.data_ptr(),
                                           d.data_ptr()), 3, 5000)
    ctx.knn_build(dm.data_ptr(), len(m), 1.0)
    dm.fill_(1e6)                                         # the index keeps its own sorted copy
    for _ in range(2):
        g5 = run(lambda i, d: ctx.knn_query(dq.data_ptr(), len(q), 5, i.data_ptr(), d.data_ptr()), 5, len(q))
        g3 = run(lambda i, d: ctx.knn_query(dq.data_ptr() + 16 * 1000, 5000, 3, i.data_ptr(), d.data_ptr()), 3, 5000)
        assert np.array_equal(g5[0], ref5[0]) and np.array_equal(g5[1], ref5[1])
        assert np.array_equal(g3[0], ref3[0]) and np.array_equal(g3[1], ref3[1])
    assert (ref5[0][:, 4] >= 0).mean() > 0.3
    # rebuild over another map (a shifted half): the oracle on a sample
    m2 = m[::2].copy()
    m2[:, 0] += 0.05
    dm2 = torch.from_numpy(m2).cuda()
    ctx.knn_build(dm2.data_ptr(), len(m2), 1.0)
    gi, gd = run(lambda i, d: ctx.knn_query(dq.data_ptr(), len(q), 5, i.data_ptr(), d.data_ptr()), 5, len(q))
    sel = np.random.default_rng(3).choice(len(q), 2000, replace=False)
    oi, od = ob.knn(m2, q[sel], 5, 1.0)
    assert np.array_equal(gi[sel], oi)
    assert np.array_equal(gd[sel][oi >= 0], od[oi >= 0].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("fine", ["0.3", "0"])
def test_knn_device_edge_cases_vs_oracle(gpu_ctx_factory, monkeypatch, fine):
    """aloam_knn_build / _query at the edges the reference's kd-tree meets (laserMapping.cpp:558-559 build,
    :582/:648 nearestKSearch + the 1 m gate): an empty map (every slot -1), no queries, a one-point map,
    heavy duplicates (40 copies of each of 50 points: ties by index, the kd-tree restatement's order),
    queries far outside the map, a map 5 km wide (the cell grows until the grid fits its cap) and k = 8 at
    r = 2 m; both the two-phase and the single-phase search. Indices equal the oracle's, distances bit for
    bit where found."""
    import torch
    monkeypatch.setenv("ALOAM_KNN_FINE", fine)
    ctx = gpu_ctx_factory(64)
    rng = np.random.default_rng(11)

    def gpu(m, q, k, r):
        dm = torch.from_numpy(np.ascontiguousarray(m, np.float32).reshape(-1, 4)).cuda()
        dq = torch.from_numpy(np.ascontiguousarray(q, np.float32).reshape(-1, 4)).cuda()
        idx = torch.full((max(len(q), 1), k), -7, dtype=torch.int32, device="cuda")
        d2 = torch.full((max(len(q), 1), k), -7.0, dtype=torch.float32, device="cuda")
        ctx.knn_build(dm.data_ptr() if len(m) else 0, len(m), r)
        ctx.knn_query(dq.data_ptr() if len(q) else 0, len(q), k, idx.data_ptr(), d2.data_ptr())
        return idx.cpu().numpy()[:len(q)], d2.cpu().numpy()[:len(q)]

    def check(m, q, k, r, what):
        gi, gd = gpu(m, q, k, r)
        oi, od = ob.knn(m, q, k, r) if len(m) else (np.full((len(q), k), -1, np.int32), None)
        assert np.array_equal(gi, oi), what
        if od is not None:
            ok = oi >= 0
            assert np.array_equal(gd[ok].view(np.uint32), od[ok].view(np.uint32)), what
        return gi

    def cloud(xyz):
        a = np.zeros((len(xyz), 4), np.float32)
        a[:, :3] = xyz
        return a

    q = cloud(rng.uniform(-3, 3, (500, 3)))
    assert (check(np.zeros((0, 4), np.float32), q, 5, 1.0, "empty map") == -1).all()
    gpu(cloud(rng.uniform(-3, 3, (100, 3))), np.zeros((0, 4), np.float32), 5, 1.0)     # no queries: a no-op
    one = check(cloud(np.array([[0.2, -0.1, 0.3]])), q, 5, 1.0, "one-point map")
    assert (one[:, 1:] == -1).all() and (one[:, 0] >= 0).any()
    base = rng.uniform(-2, 2, (50, 3))
    dup = cloud(np.repeat(base, 40, axis=0)[rng.permutation(2000)])
    di = check(dup, cloud(base + rng.normal(0, 0.05, base.shape)), 8, 1.0, "duplicates")
    assert (di[:, 7] >= 0).all()
    far = q.copy()
    far[:, 0] += 1e4
    assert (check(cloud(rng.uniform(-3, 3, (3000, 3))), far, 5, 1.0, "far queries") == -1).all()
    wide = np.concatenate([rng.uniform(-3, 3, (20000, 3)), rng.uniform(-3, 3, (20000, 3)) + [5000.0, 0.0, 0.0]])
    qw = np.concatenate([rng.uniform(-3.5, 3.5, (1500, 3)), rng.uniform(-3.5, 3.5, (1500, 3)) + [5000.0, 0.0, 0.0]])
    wi = check(cloud(wide), cloud(qw), 5, 1.0, "5 km map")
    assert (wi[:, 4] >= 0).mean() > 0.5
    check(cloud(rng.uniform(-10, 10, (30000, 3))), cloud(rng.uniform(-11, 11, (2000, 3))), 8, 2.0, "k 8, r 2")


@pytest.mark.gpu
@pytest.mark.parametrize("step,k,radius,frac", [(0.107, 5, 1.0, "0.3"), (0.15, 8, 1.0, "0.2"), (0.5, 5, 1.0, "0.3"),
                                                (0.107, 3, 0.5, "0.45")])
def test_knn_device_two_phase_bit_identical(gpu_ctx_factory, monkeypatch, step, k, radius, frac):
    """The two-phase search (fine 3x3x3 block first, settled when the k-th neighbour is closer than
    0.99 fine cells) returns exactly the single-phase radius-block result for EVERY query: indices,
    distance bits and order. Dense maps (most queries settle in phase 1), a sparse one (0.5 m lattice:
    most fall through to phase 2), k = 3/5/8 and a smaller radius."""
    import torch
    m = synth.dense_map(4, 0.0, 0.0, step=step)
    R, o = synth.pose("l128", 0)
    s = synth.scan("l128", 0)
    q = s.copy()
    q[:, :3] = (s[:, :3].astype(np.float64) @ R.T + o).astype(np.float32)
    dm, dq = torch.from_numpy(m).cuda(), torch.from_numpy(q).cuda()
    ctx = gpu_ctx_factory(128)
    out = {}
    for mode in ("0", frac):
        monkeypatch.setenv("ALOAM_KNN_FINE", mode)
        idx = torch.full((len(q), k), -7, dtype=torch.int32, device="cuda")
        d2 = torch.full((len(q), k), -7.0, dtype=torch.float32, device="cuda")
        ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr(), len(q), k, radius, idx.data_ptr(), d2.data_ptr())
        out[mode] = (idx.cpu().numpy(), d2.cpu().numpy())
    (i1, e1), (i2, e2) = out["0"], out[frac]
    assert (i1 >= -1).all() and (i2 >= -1).all()
    assert np.array_equal(i1, i2)
    assert np.array_equal(e1.view(np.uint32), e2.view(np.uint32))
    assert (i1[:, k - 1] >= 0).mean() > 0.3          # the case exercises found neighbourhoods


@pytest.mark.gpu
@pytest.mark.parametrize("step,frac", [(0.107, "0.3"), (0.107, "0.1"), (0.107, "0.45")])
def test_knn_device_kernels_bit_identical(gpu_ctx_factory, monkeypatch, step, frac):
    """Every phase-1 variant of aloam_knn_device returns the single-phase result bit for bit, and the library
    names the kernel it launched (aloam_knn_kernel): k_knn_keys (default, 64-bit keys; 4 or 8 loads in flight),
    k_knn_2phase (ALOAM_KNN_KEYS=0), k_knn_shared (+ ALOAM_KNN_SHARED=1), k_knn_tile (+ ALOAM_KNN_TILE=1,
    per call) and k_knn_tile with every tile over its LDS budget (ALOAM_KNN_TILE=2: phase 1 from global
    memory inside the tile kernel). frac 0.1 puts the far tiles' boxes over 768 fine cells and frac 0.45 over
    2048 points (~5 m of arc at 50 m for 32 ring-ordered queries), so the natural overflow path runs too."""
    import torch
    m = synth.dense_map(4, 0.0, 0.0, step=step)
    R, o = synth.pose("l128", 0)
    s = synth.scan("l128", 0)
    q = s.copy()
    q[:, :3] = (s[:, :3].astype(np.float64) @ R.T + o).astype(np.float32)
    dm, dq = torch.from_numpy(m).cuda(), torch.from_numpy(q).cuda()
    ctx = gpu_ctx_factory(128)
    out, names = {}, {}
    variants = {                                   # env -> the kernel aloam_knn_kernel must name
        ("0", ""): "k_knn_group<5,8>",
        (frac, ""): "k_knn_keys<5,8>",
        (frac, "ALOAM_KNN_U=8"): "k_knn_keys<5,8,U8>",
        (frac, "ALOAM_KNN_PK=1"): "k_knn_keys<5,8,PK>",
        (frac, "ALOAM_KNN_KEYS=0"): "k_knn_2phase<5,8>",
        (frac, "ALOAM_KNN_KEYS=0,ALOAM_KNN_SHARED=1"): "k_knn_shared<5,4>",
        (frac, "ALOAM_KNN_KEYS=0,ALOAM_KNN_SHARED=1,ALOAM_KNN_SU=2"): "k_knn_shared<5,2>",
        (frac, "ALOAM_KNN_KEYS=0,ALOAM_KNN_TILE=1"): "k_knn_tile<5,8>",
        (frac, "ALOAM_KNN_KEYS=0,ALOAM_KNN_TILE=2"): "k_knn_tile<5,8>",
    }
    knobs = ("ALOAM_KNN_U", "ALOAM_KNN_PK", "ALOAM_KNN_KEYS", "ALOAM_KNN_SHARED", "ALOAM_KNN_SU", "ALOAM_KNN_TILE")
    for (fine, env), name in variants.items():
        for kn in knobs:
            monkeypatch.delenv(kn, raising=False)
        for kv in filter(None, env.split(",")):
            a, b = kv.split("=")
            monkeypatch.setenv(a, b)
        monkeypatch.setenv("ALOAM_KNN_FINE", fine)
        idx = torch.full((len(q), 5), -7, dtype=torch.int32, device="cuda")
        d2 = torch.full((len(q), 5), -7.0, dtype=torch.float32, device="cuda")
        ctx.knn_device(dm.data_ptr(), len(m), dq.data_ptr(), len(q), 5, 1.0, idx.data_ptr(), d2.data_ptr())
        out[(fine, env)] = (idx.cpu().numpy(), d2.cpu().numpy())
        names[(fine, env)] = ctx.knn_kernel()
        assert names[(fine, env)] == name, (env, names[(fine, env)])
    i0, e0 = out[("0", "")]
    assert (i0 >= -1).all() and (i0[:, 4] >= 0).mean() > 0.3
    for key, (i1, e1) in out.items():
        assert np.array_equal(i0, i1), key
        assert np.array_equal(e0.view(np.uint32), e1.view(np.uint32)), key


@pytest.mark.gpu
@pytest.mark.parametrize("stages", [2, 3])
def test_pipeline_matches_single_context(lvo, stages):
    """The node-split pipelines (aloam_forward_features / aloam_forward_mapping_input between
    contexts) produce the single-context trajectory: same correspondences, poses to 1e-9."""
    p = abi.default_params(16)
    frames = [synth.scan("vlp16", k) for k in range(7)]
    ref = lvo.Context(p)
    ro = [ref.process_scan(f) for f in frames]
    ref.close()
    pipe = lvo.Pipeline(p, stages=stages)
    ods, mps = [], []
    for f in frames:
        od, mp = pipe.push(f)
        if od is not None:
            ods.append(od)
        if mp is not None:
            mps.append(mp)
    for od, mp in pipe.flush():
        if od is not None:
            ods.append(od)
        if mp is not None:
            mps.append(mp)
    pipe.close()
    assert len(ods) == len(frames) and len(mps) == len(frames)
    for (o_ref, m_ref), o, m in zip(ro, ods, mps):
        assert o["corner_correspondence"] == o_ref["corner_correspondence"]
        assert o["plane_correspondence"] == o_ref["plane_correspondence"]
        np.testing.assert_allclose(o["t_w_curr"], o_ref["t_w_curr"], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(m["t_w_curr"], m_ref["t_w_curr"], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(m["q_w_curr"], m_ref["q_w_curr"], rtol=1e-9, atol=1e-12)


def _run_pipeline(lvo, p, frames, stages):
    pipe = lvo.Pipeline(p, stages=stages)
    ods, mps = [], []
    for f in frames:
        od, mp = pipe.push(f)
        if od is not None:
            ods.append(od)
        if mp is not None:
            mps.append(mp)
    for od, mp in pipe.flush():
        if od is not None:
            ods.append(od)
        if mp is not None:
            mps.append(mp)
    pipe.close()
    return ods, mps


def _assert_pipeline_vs_oracle(p, frames, ods, mps):
    orc = ob.Oracle(p)
    ref = [orc.process_scan(f) for f in frames]
    published = [k for k, (o, _) in enumerate(ref) if o["publish_to_mapping"]]
    assert len(ods) == len(frames) and len(mps) == len(published), (len(ods), len(mps), published)
    for k, (od, (oo, _)) in enumerate(zip(ods, ref)):
        for key in ("publish_to_mapping", "corner_correspondence", "plane_correspondence"):
            assert od[key] == oo[key], (k, key, od[key], oo[key])
        np.testing.assert_allclose(od["t_w_curr"], oo["t_w_curr"], rtol=POSE_RTOL, atol=1e-7)
    for mp, k in zip(mps, published):
        mo = ref[k][1]
        for key in ("optimized", "map_corner_num", "map_surf_num", "corner_stack_num", "surf_stack_num",
                    "corner_num", "surf_num", "map_total_points"):
            assert mp[key] == mo[key], (k, key, mp[key], mo[key])
        np.testing.assert_allclose(mp["t_w_curr"], mo["t_w_curr"], rtol=POSE_RTOL, atol=1e-7)
        np.testing.assert_allclose(mp["q_w_curr"], mo["q_w_curr"], rtol=POSE_RTOL, atol=1e-9)
    return published


_PIPE_MODES = [(2, "2"), (2, "1"), (3, "2")]          # (stages, ALOAM_PIPE_LAG): results returned 2 or 1 scans late


@pytest.mark.parametrize("stages,lag", _PIPE_MODES)
def test_pipeline_mapping_skip_frame_two(lvo, monkeypatch, stages, lag):
    """mapping_skip_frame = 2 (laserOdometry.cpp:274, :643): odometry publishes every second scan to
    mapping; the native pipeline maps exactly those, as the oracle."""
    monkeypatch.setenv("ALOAM_PIPE_LAG", lag)
    p = abi.default_params(64)
    p.mapping_skip_frame = 2
    frames = [synth.scan("hdl64", k) for k in range(7)]
    ods, mps = _run_pipeline(lvo, p, frames, stages)
    assert _assert_pipeline_vs_oracle(p, frames, ods, mps) == [0, 2, 4, 6]


@pytest.mark.parametrize("stages,lag", _PIPE_MODES)
def test_pipeline_feature_count_jump(lvo, monkeypatch, stages, lag):
    """Sparse sweeps (every 5th return) followed by full ones: the feature and stack counts jump past the
    sizes the previous frame's launches were sized for (the hinted stack VoxelGrid redoes at the exact
    size); every stage still matches the oracle."""
    monkeypatch.setenv("ALOAM_PIPE_LAG", lag)
    p = abi.default_params(64)
    frames = _jump_frames()
    ods, mps = _run_pipeline(lvo, p, frames, stages)
    _assert_pipeline_vs_oracle(p, frames, ods, mps)


def _jump_frames():
    return [synth.scan("hdl64", k)[::5] for k in range(3)] + [synth.scan("hdl64", k) for k in range(3, 6)]


_POLL_SCRIPT = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from lvo_amd_loader import lvo
import test_gpu_parity as T
p = lvo.abi.default_params(64)
p.mapping_skip_frame = int(sys.argv[2])
frames = T._jump_frames()
ods, mps = T._run_pipeline(lvo, p, frames, 2)
T._assert_pipeline_vs_oracle(p, frames, ods, mps)
print("ok", len(ods), len(mps))
"""


@pytest.mark.parametrize("skip", [1, 2])
def test_pipeline_poll_mode(skip):
    """ALOAM_PIPE_POLL=1 (read once per process, so in a child): mapping results are handed back as
    they complete instead of at a fixed lag; sparse -> dense jump, skip_frame 1 and 2, against the
    oracle."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, ALOAM_PIPE_POLL="1")
    here = os.path.dirname(os.path.abspath(__file__))
    out = subprocess.run([sys.executable, "-c", _POLL_SCRIPT, here, str(skip)], env=env, capture_output=True,
                         text=True, timeout=110, cwd=here)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert out.stdout.strip().splitlines()[-1].startswith("ok 6")


_SIDE_SCRIPT = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from lvo_amd_loader import lvo
synth = lvo.synth
p = lvo.abi.default_params(16)
pipe = lvo.Pipeline(p)
mps = []
for k in range(7):
    od, mp = pipe.push(synth.scan("vlp16", k))
    if mp is not None:
        mps.append(list(mp["t_w_curr"]) + list(mp["q_w_curr"]))
for od, mp in pipe.flush():
    if mp is not None:
        mps.append(list(mp["t_w_curr"]) + list(mp["q_w_curr"]))
pipe.close()
print(json.dumps(mps))
"""


def test_pipeline_side_stream_stacks(lvo):
    """ALOAM_SIDE_STACKS=1 (opt-in): hand-off copy and stack VoxelGrid on the mapping context's third
    stream, overlapping the previous frame, over double-buffered input sets — same trajectory."""
    import json
    import os
    import subprocess
    import sys
    p = abi.default_params(16)
    ref = lvo.Context(p)
    ro = [ref.process_scan(synth.scan("vlp16", k))[1] for k in range(7)]
    ref.close()
    env = dict(os.environ, ALOAM_SIDE_STACKS="1")
    out = subprocess.run([sys.executable, "-c", _SIDE_SCRIPT, os.path.dirname(os.path.abspath(__file__))], env=env,
                         capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    mps = json.loads(out.stdout.strip().splitlines()[-1])
    assert len(mps) == 7
    for m, m_ref in zip(mps, ro):
        np.testing.assert_allclose(m[:3], m_ref["t_w_curr"], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(m[3:], m_ref["q_w_curr"], rtol=1e-9, atol=1e-12)


_EARLY_SCRIPT = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from lvo_amd_loader import lvo
synth = lvo.synth
p = lvo.abi.default_params(64)
frames = [synth.scan("hdl64", k) for k in range(3)]
frames = frames + [frames[0][:0]] + [synth.scan("hdl64", k) for k in range(3, 6)]
pipe = lvo.Pipeline(p)
rows = []
def keep(od, mp):
    if mp is not None:
        rows.append([int(mp[k]) for k in ("corner_stack_num", "surf_stack_num", "map_corner_num", "map_surf_num")]
                    + [float(v).hex() for v in list(mp["t_w_curr"]) + list(mp["q_w_curr"])])
for f in frames:
    keep(*pipe.push(f))
for od, mp in pipe.flush():
    keep(od, mp)
pipe.close()
print(json.dumps(rows))
"""


def test_pipeline_early_stacks_with_empty_sweep():
    """ALOAM_EARLY_STACKS (read once per process, so each schedule in a child): the mapping stacks read from the
    last-cloud buffers with counts copied on stream2 (1, default) and from the publish copy (0) give the same
    stack counts, map counts and bit-identical poses, over a sequence with an EMPTY sweep between full ones
    (stream2 must be ordered after the empty registration's k_meta_init, not read the previous scan's counts)."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for early in ("0", "1"):
        env = dict(os.environ, ALOAM_EARLY_STACKS=early)
        out = subprocess.run([sys.executable, "-c", _EARLY_SCRIPT, here], env=env, capture_output=True, text=True,
                             timeout=110, cwd=here)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
        res[early] = json.loads(out.stdout.strip().splitlines()[-1])
    assert len(res["1"]) == 7, len(res["1"])
    assert res["0"] == res["1"]
    assert res["1"][3][:2] == [0, 0]                  # the empty sweep's stacks are empty, not the previous scan's


def test_pipeline_errors_and_timing(lvo):
    """The native pipeline reports stage errors through aloam_pipeline_last_error and stays usable;
    with profiling on, every stage's HIP-event timing of its last job is available."""
    p = abi.default_params(16)
    pipe = lvo.Pipeline(p, stages=2)
    with pytest.raises(lvo.ALOAMError):
        pipe.push(np.zeros((p.max_scan_points + 1, 4), np.float32))
    pipe.set_profiling(True)
    for k in range(3):
        pipe.push(synth.scan("vlp16", k))
    out = pipe.flush()
    assert len(out) == 1 and out[0][1] is not None
    assert pipe.last_front_timing["scan_registration_ms"] > 0 and pipe.last_front_timing["odometry_ms"] > 0
    assert pipe.last_back_timing["mapping_ms"] > 0
    pipe.close()


@pytest.mark.parametrize("step", [16, 20, 32, 48])
def test_pointcloud2_ingestion_bit_exact(gpu_ctx_factory, step):
    """aloam_scan_registration_pc2 (sensor_msgs/PointCloud2 blob, x y z at offsets 0 4 8, noise in every
    other byte) gives the oracle's features bit for bit, from host and from device memory."""
    import torch
    ctx = gpu_ctx_factory(64)
    orc = ob.Oracle(abi.default_params(64))
    pts = synth.scan("hdl64", 2)
    blob = synth.to_pointcloud2(pts, step, seed=step)
    orc.scan_registration(pts)
    fo = orc.features()
    ctx.scan_registration_pc2(blob, point_step=step)
    assert_features_equal(ctx.features(), fo)
    d = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to("cuda:0")
    ctx.scan_registration_pc2(None, n=len(pts), point_step=step, device_ptr=d.data_ptr())
    assert_features_equal(ctx.features(), fo)
    with pytest.raises(lvo.ALOAMError):
        ctx.scan_registration_pc2(blob[:100], n=5, point_step=10)


def test_cpp_host_tool_matches_python_host(lvo, tmp_path):
    """The C++ headless host (tools/aloam_kitti: KITTI .bin files -> native pipeline -> KITTI poses)
    reproduces the single-context trajectory."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(lvo.LIB_PATH), "..", "tools", "aloam_kitti")
    frames = [synth.scan("hdl64", k) for k in range(6)]
    paths = []
    for k, f in enumerate(frames):
        pth = str(tmp_path / f"{k:06d}.bin")
        synth.write_kitti_bin(pth, f)
        paths.append(pth)
    out = str(tmp_path / "poses.txt")
    mpath, opath, hpath = (str(tmp_path / n) for n in ("map_path.txt", "odom_path.txt", "hf.txt"))
    subprocess.check_call([exe, "-l", "64", "-o", out, "--map-path", mpath, "--odom-path", opath, "--hf", hpath] + paths,
                          timeout=120)
    poses = np.loadtxt(out).reshape(-1, 3, 4)
    ctx = lvo.Context(abi.default_params(64))
    res = [ctx.process_scan(f) for f in frames]
    ctx.close()
    ref = [m for _, m in res]
    assert len(poses) == len(frames)
    for P, m in zip(poses, ref):
        np.testing.assert_allclose(P[:, 3], m["t_w_curr"], rtol=1e-9, atol=1e-9)
    # the Paths: one pose appended per mapped / odometry scan (laserMapping.cpp:866-873, laserOdometry.cpp:598-607)
    mp, op, hf = np.loadtxt(mpath, ndmin=2), np.loadtxt(opath, ndmin=2), np.loadtxt(hpath, ndmin=2)
    assert mp.shape == (len(frames), 8) and op.shape == (len(frames), 8) and hf.shape == (len(frames), 8)
    np.testing.assert_array_equal(mp[:, 0], np.arange(len(frames)))
    for k, (o, m) in enumerate(res):
        np.testing.assert_allclose(mp[k, 1:4], m["t_w_curr"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(mp[k, 4:8], m["q_w_curr"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(op[k, 1:4], o["t_w_curr"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(op[k, 4:8], o["q_w_curr"], rtol=1e-9, atol=1e-9)
    # high-frequency poses: each odometry pose through one of the map corrections published so far
    def through(qm, tm, qo, to):
        x1, y1, z1, w1 = qm
        x2, y2, z2, w2 = qo
        q = np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                      w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])
        u = np.array([x1, y1, z1])
        v = np.asarray(to, float)
        t = v + 2.0 * w1 * np.cross(u, v) + 2.0 * np.cross(u, np.cross(u, v))
        return q, t + np.asarray(tm, float)
    corrections = [([0.0, 0.0, 0.0, 1.0], [0.0, 0.0, 0.0])] + [(m["q_wmap_wodom"], m["t_wmap_wodom"]) for m in ref]
    for k, (o, _) in enumerate(res):
        ok = False
        for qm, tm in corrections[:k + 1]:
            q, t = through(qm, tm, o["q_w_curr"], o["t_w_curr"])
            ok = ok or (np.allclose(hf[k, 4:8], q, rtol=0, atol=1e-9) and np.allclose(hf[k, 1:4], t, rtol=0, atol=1e-9))
        assert ok, (k, hf[k])


def test_cu_mask_contexts_match(gpu_ctx_factory):
    """A context restricted to a CU subset (aloam_set_cu_mask; the pipeline's per-stage partitions)
    computes the same results — the persistent LM solver's grid is capped by the mask, so its fixed
    reduction order (and the last bits of the pose) may differ: poses to 1e-9."""
    import ctypes as C
    frames = [synth.scan("vlp16", k) for k in range(4)]
    a = gpu_ctx_factory(16)
    b = gpu_ctx_factory(16)
    mask = (C.c_uint * 8)(*([0xF] + [0] * 7))          # 4 CUs
    assert lvo.lib().aloam_set_cu_mask(b.h, mask, 8) == 0
    for f in frames:
        oa, ma = a.process_scan(f)
        ob_, mb = b.process_scan(f)
        assert oa["corner_correspondence"] == ob_["corner_correspondence"]
        np.testing.assert_allclose(ma["t_w_curr"], mb["t_w_curr"], rtol=1e-9, atol=1e-12)
    assert lvo.lib().aloam_set_cu_mask(b.h, mask, 0) == 0
    zero = (C.c_uint * 8)()
    assert lvo.lib().aloam_set_cu_mask(b.h, zero, 8) != 0


def test_cu_mask_solver_with_a_busy_neighbour(gpu_ctx_factory):
    """The persistent LM solver's workgroups exchange records across the grid, so they must all run at
    once: a context restricted to 4 CUs (grid capped at 4 workgroups) keeps solving correctly while a
    second context runs its own frames concurrently from another thread on the next 60 CUs (disjoint CU
    sets, as the pipeline gives its stages: INTEGRATION.md). Poses equal the same context's unshared run
    to 1e-9."""
    import ctypes as C
    import threading
    frames = [synth.scan("vlp16", k) for k in range(6)]
    mask = (C.c_uint * 8)(*([0xF] + [0] * 7))
    other = (C.c_uint * 8)(*([0xFFFFFFF0, 0xFFFFFFFF] + [0] * 6))
    ref_ctx = gpu_ctx_factory(16)
    assert lvo.lib().aloam_set_cu_mask(ref_ctx.h, mask, 8) == 0
    ref = [ref_ctx.process_scan(f)[1]["t_w_curr"] for f in frames]
    a, b = gpu_ctx_factory(16), gpu_ctx_factory(64)
    assert lvo.lib().aloam_set_cu_mask(a.h, mask, 8) == 0
    assert lvo.lib().aloam_set_cu_mask(b.h, other, 8) == 0
    out, errs = {}, []

    def run(ctx, key, seq):
        try:
            out[key] = [ctx.process_scan(f)[1]["t_w_curr"] for f in seq]
        except Exception as e:   # surfaced below
            errs.append(e)
    busy = [synth.scan("hdl64", k) for k in range(4)]
    t1 = threading.Thread(target=run, args=(a, "a", frames))
    t2 = threading.Thread(target=run, args=(b, "b", busy))
    t1.start(); t2.start(); t1.join(timeout=300); t2.join(timeout=300)
    assert not errs, errs
    assert len(out["a"]) == len(frames)
    for x, y in zip(out["a"], ref):
        np.testing.assert_allclose(x, y, rtol=1e-9, atol=1e-12)


def test_c5_sequence_ate_vs_oracle(lvo):
    """BASELINE configs[4] stand-in (KITTI-04 is not on the box): the 271-frame synthetic straight road
    end to end through the native pipeline against the oracle run of the same frames. North-star bar:
    ATE delta <= 1e-4 m (RMSE of the mapped-position difference, same frame, no alignment)."""
    frames = synth.sequence("c5", synth.C5_FRAMES)
    pipe = lvo.Pipeline(abi.default_params(64))
    traj = []
    for f in frames:
        _, mp = pipe.push(f)
        if mp is not None:
            traj.append(mp["t_w_curr"])
    traj += [mp["t_w_curr"] for _, mp in pipe.flush() if mp is not None]
    pipe.close()
    orc = ob.Oracle(abi.default_params(64))
    otraj = [orc.process_scan(f)[1]["t_w_curr"] for f in frames]
    assert len(traj) == len(otraj) == synth.C5_FRAMES
    ate = float(np.sqrt(np.mean(np.sum((np.array(traj) - np.array(otraj)) ** 2, axis=1))))
    print(f"C5 ATE delta vs oracle {ate:.3e} m")
    assert ate <= 1e-4, ate
    # and both track the synthetic ground truth (straight road, 1 m per frame)
    R0, o0 = synth.pose("c5", 0)
    gt = np.array([R0.T @ (synth.pose("c5", k)[1] - o0) for k in range(synth.C5_FRAMES)])
    drift = np.linalg.norm(np.array(traj) - gt, axis=1).max()
    print(f"C5 max drift vs ground truth {drift:.3f} m over {synth.C5_FRAMES} m")
    assert drift < 0.01 * synth.C5_FRAMES, drift          # < 1% of the 271 m travelled


@pytest.mark.parametrize("n_azimuth,lattice", [(4200, 0), (9000, 0), (4200, 20)])
def test_scan_registration_oversized_lines_bit_exact(gpu_ctx_factory, n_azimuth, lattice):
    """Lines longer than the kernel's LDS capacity (4096 points) take the global-scratch instantiation of
    the line kernel (k_scan.hip line_features_body<true>); its features must match the oracle bit for
    bit like the LDS instantiation's (also with lattice-quantised points: many exact curvature ties)."""
    pts = synth.scan("vlp16", 3, n_azimuth=n_azimuth)
    if lattice:
        pts[:, :3] = np.round(pts[:, :3] * lattice) / lattice
    ctx = gpu_ctx_factory(16, max_scan_points=max(len(pts), 1024) + 1024)
    orc = ob.Oracle(abi.default_params(16))
    ctx.scan_registration(pts)
    orc.scan_registration(pts)
    assert_features_equal(ctx.features(), orc.features())
