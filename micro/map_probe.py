"""Profiling probe (not a test): per-frame mapping association timing on the bench sequence."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

frames = lvo.synth.sequence("hdl64", 14)
ctx = lvo.Context(lvo.abi.default_params(64))
dev = [torch.from_numpy(f).cuda() for f in frames]
for k in range(6):
    ctx.process_scan(device_ptr=dev[k].data_ptr(), n=len(frames[k]))
ctx.set_profiling(True)
ms, nb, st = [], [], []
for k in range(6, 14):
    od, mp = ctx.process_scan(device_ptr=dev[k].data_ptr(), n=len(frames[k]))
    t = ctx.timing()
    ms.append(t["map_search_ms"] / max(t["map_search_launches"], 1))
    nb.append(t["map_search_bytes"] / max(t["map_search_launches"], 1))
    st.append((mp["corner_stack_num"], mp["surf_stack_num"], mp["map_corner_num"], mp["map_surf_num"]))
print("EXP", os.environ.get("ALOAM_EXP", "0"), "assoc us/launch %.1f" % (1000 * np.mean(ms)), "bytes/launch %.0f" % np.mean(nb),
      "stacks/map", st[-1])
