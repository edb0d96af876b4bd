"""Kernel-time probe of the PCL-order VoxelGrid sites (run under rocprofv3 --kernel-trace --stats):
scanRegistration (k_line_features), aloam_voxel_grid at several sizes (k_vox_pcl), a few mapping frames
(k_rb_cubevox)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from lvo_amd_loader import lvo
ctx = lvo.Context(lvo.abi.default_params(64), device=0)
pts = lvo.synth.scan("hdl64", 3)
for _ in range(10):
    ctx.scan_registration(pts)
for n in (2000, 6000, 25000):
    for _ in range(10):
        ctx.voxel_grid(pts[:n], 0.8)
c2 = lvo.Context(lvo.abi.default_params(64), device=0)
for k in range(12):
    c2.process_scan(lvo.synth.scan("hdl64", k))
print("ok")
