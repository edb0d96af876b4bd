#!/usr/bin/env python3
"""Regenerates tests/golden/pipeline_golden.npz from the CPU oracle (oracle/liboracle.so).

Fixtures = seeded synthetic inputs (generator + seeds + sha256 of the generated sweeps) and the
oracle's outputs on them: feature index lists, curvature / laserCloud hashes, per-frame odometry and
mapping poses, correspondence counts. The reference itself is unbuildable here (ROS/PCL/Ceres
absent), so these pin the restatement against regressions and anchor the GPU parity tests on
stored vectors; see DESIGN.md "Parity status".

usage: python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_binding as ob  # noqa: E402
from lvo_amd_loader import abi, synth  # noqa: E402

CASES = [("vlp16", 16, 4), ("hdl64", 64, 3)]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out = {}
    for name, lines, nframes in CASES:
        o = ob.Oracle(abi.default_params(lines))
        for k in range(nframes):
            pts = synth.scan(name, k)
            od, mp = o.process_scan(pts)
            f = o.features()
            key = f"{name}_{k}"
            out[key + "_input_sha"] = np.array(sha(pts))
            out[key + "_n_input"] = np.array(len(pts))
            for fk in ("sharp_idx", "less_sharp_idx", "flat_idx"):
                out[f"{key}_{fk}"] = f[fk]
            out[key + "_full_sha"] = np.array(sha(f["full"]))
            out[key + "_curv_sha"] = np.array(sha(f["curvature"]))
            out[key + "_less_flat_sha"] = np.array(sha(f["less_flat"]))
            out[key + "_odom_q"] = od["q_w_curr"]
            out[key + "_odom_t"] = od["t_w_curr"]
            out[key + "_map_q"] = mp["q_w_curr"]
            out[key + "_map_t"] = mp["t_w_curr"]
            out[key + "_corner_corr"] = np.array(od["corner_correspondence"], np.int32)
            out[key + "_plane_corr"] = np.array(od["plane_correspondence"], np.int32)
    np.savez_compressed(os.path.join(HERE, "pipeline_golden.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
