"""Committed golden vectors (tests/golden/pipeline_golden.npz, made by tests/golden/make_golden.py).

CPU: the generator and the oracle reproduce the stored fixtures exactly.
GPU: the HIP pipeline reproduces the stored feature indices / hashes and the poses within 1e-6.
"""
import hashlib
import os

import numpy as np
import pytest

import oracle_binding as ob
from lvo_amd_loader import abi, synth

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "pipeline_golden.npz"))
CASES = [("vlp16", 16, 4), ("hdl64", 64, 3)]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def check(name, k, f, od, mp, exact_poses):
    key = f"{name}_{k}"
    for fk in ("sharp_idx", "less_sharp_idx", "flat_idx"):
        assert np.array_equal(f[fk], G[f"{key}_{fk}"]), (key, fk)
    assert sha(f["full"]) == str(G[key + "_full_sha"])
    assert sha(f["curvature"]) == str(G[key + "_curv_sha"])
    assert sha(f["less_flat"]) == str(G[key + "_less_flat_sha"])
    for a, b in ((od["q_w_curr"], G[key + "_odom_q"]), (od["t_w_curr"], G[key + "_odom_t"]),
                 (mp["q_w_curr"], G[key + "_map_q"]), (mp["t_w_curr"], G[key + "_map_t"])):
        if exact_poses:
            assert np.array_equal(a, b)
        else:
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-8)
    assert list(od["corner_correspondence"]) == list(G[key + "_corner_corr"])
    assert list(od["plane_correspondence"]) == list(G[key + "_plane_corr"])


@pytest.mark.parametrize("name,lines,nframes", CASES)
def test_inputs_are_reproducible(name, lines, nframes):
    for k in range(nframes):
        pts = synth.scan(name, k)
        assert sha(pts) == str(G[f"{name}_{k}_input_sha"])


@pytest.mark.parametrize("name,lines,nframes", CASES)
def test_oracle_reproduces_golden(name, lines, nframes):
    o = ob.Oracle(abi.default_params(lines))
    for k in range(nframes):
        od, mp = o.process_scan(synth.scan(name, k))
        check(name, k, o.features(), od, mp, exact_poses=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name,lines,nframes", CASES)
def test_gpu_reproduces_golden(gpu_ctx_factory, name, lines, nframes):
    ctx = gpu_ctx_factory(lines)
    for k in range(nframes):
        od, mp = ctx.process_scan(synth.scan(name, k))
        check(name, k, ctx.features(), od, mp, exact_poses=False)
