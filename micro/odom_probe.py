"""Profiling probe (not a test): per-round odometry search time on the bench sequence."""
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
ms = []
for k in range(6, 14):
    od, mp = ctx.process_scan(device_ptr=dev[k].data_ptr(), n=len(frames[k]))
    t = ctx.timing()
    ms.append(t["odom_search_ms"] / max(t["odom_search_launches"], 1))
f = ctx.features()
print("ODOM_EXP", os.environ.get("ALOAM_ODOM_EXP", "0"), "search us/round %.1f" % (1000 * np.mean(ms)),
      "sharp", len(f["sharp_idx"]), "flat", len(f["flat_idx"]))
