"""include/aloam_lidar_factor.hpp keeps the reference's lidarFactor.hpp functor API
(src/lidarFactor.hpp:12-172): compiled with g++ here, its residuals must agree with the oracle's
Jet evaluation of the same factors, and to_device() must produce the record the HIP solver reads."""
import os
import subprocess

import numpy as np
import pytest

import oracle_binding as ob
from lvo_amd_loader import abi

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "_build", "lidar_factor_api_check")


@pytest.fixture(scope="module")
def exe():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    src = os.path.join(HERE, "lidar_factor_api_check.cpp")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall", "-Werror", src, "-o", EXE])
    return EXE


def test_functors_match_oracle(exe):
    rng = np.random.default_rng(11)
    n = 200
    q = rng.normal(0, 0.2, 4)
    q[3] = 1.0
    q /= np.linalg.norm(q)
    x = np.concatenate([q, rng.normal(0, 1, 3)])
    types = rng.integers(0, 4, n)
    pts = rng.normal(0, 5, (n, 4, 3))
    lines = [" ".join(repr(float(v)) for v in x), str(n)]
    for i in range(n):
        if types[i] == 2:   # unit normal + offset
            nrm = rng.normal(size=3)
            pts[i, 1] = nrm / np.linalg.norm(nrm)
            pts[i, 2] = [rng.normal(), 0, 0]
        lines.append(f"{types[i]} " + " ".join(repr(float(v)) for v in pts[i].ravel()))
    out = subprocess.run([exe], input="\n".join(lines), capture_output=True, text=True, check=True).stdout.split("\n")
    res, norms = [], []
    for ln in out:
        if ln.startswith("N "):
            norms.append([float(v) for v in ln.split()[1:]])
        elif ln.startswith("R "):
            tok = ln.split()
            assert int(tok[5]) == 1
            res.append((int(tok[1]), [float(v) for v in tok[2:5]]))
    assert len(res) == n
    # the same factors through the oracle (device record layout)
    f = np.zeros(n, abi.FACTOR_DTYPE)
    k = 0
    for i in range(n):
        f["type"][i] = types[i]
        f["cp"][i] = pts[i, 0]
        if types[i] == 0:
            f["a"][i], f["b"][i] = pts[i, 1], pts[i, 2]
        elif types[i] == 1:
            f["a"][i], f["b"][i] = pts[i, 1], norms[k]
            k += 1
        elif types[i] == 2:
            f["a"][i], f["b"][i] = pts[i, 1], pts[i, 2]
        else:
            f["a"][i] = pts[i, 1]
        assert res[i][0] == types[i]
    r_or, _, _ = ob.eval_factors(f, x, robust=False)
    got = np.array([r for _, r in res])
    m = np.where(types[:, None] == 0, 3, np.where(types[:, None] == 3, 3, 1))
    mask = np.arange(3)[None, :] < m
    np.testing.assert_allclose(got[mask], r_or[mask], rtol=1e-12, atol=1e-12)
