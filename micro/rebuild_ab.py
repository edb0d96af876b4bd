"""A/B check (profiling aid): the map and trajectory after N frames, dumped for comparison across builds /
env settings (ALOAM_REBUILD_FUSED=0|1). usage: rebuild_ab.py N out.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

N = int(sys.argv[1])
ctx = lvo.Context(lvo.abi.default_params(64))
traj = []
for f in lvo.synth.sequence("hdl64", N, start=0):
    od, mp = ctx.process_scan(f)
    traj.append(np.concatenate([mp["q_w_curr"], mp["t_w_curr"]]))
maps = [ctx.map_cloud(w) for w in (0, 1)] if hasattr(ctx, "map_cloud") else []
np.savez(sys.argv[2], traj=np.array(traj), *maps)
print("saved", sys.argv[2], [m.shape for m in maps])
