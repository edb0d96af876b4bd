"""Step-by-step run of the PCL-order sort sites (check build: ALOAM_PS_CHECK prints bad indices)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from lvo_amd_loader import lvo
ctx = lvo.Context(lvo.abi.default_params(16), device=0)
pts = lvo.synth.scan("vlp16", 0)
steps = [("scanreg vlp16", lambda: (ctx.scan_registration(pts), ctx.features())),
         ("voxel 20", lambda: ctx.voxel_grid(pts[:20], 0.4)),
         ("voxel 2000", lambda: ctx.voxel_grid(pts[:2000], 0.4)),
         ("voxel 6000", lambda: ctx.voxel_grid(pts[:6000], 0.4)),
         ("voxel 20000", lambda: ctx.voxel_grid(pts[:20000], 0.4))]
for name, fn in steps:
    print("step", name, flush=True)
    fn()
    print("  ok", flush=True)
