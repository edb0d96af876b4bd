"""Diagnostic (not a test): torch HIP init after an aloam context was created/used/destroyed."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

mode = sys.argv[1]
ctx = lvo.Context(lvo.abi.default_params(16))
if mode in ("use", "use_close"):
    for k in range(3):
        ctx.process_scan(lvo.synth.scan("vlp16", k))
if mode in ("close", "use_close"):
    ctx.close()
import torch  # noqa: E402
try:
    print(mode, "torch available:", torch.cuda.is_available(), torch.cuda.device_count(), torch.zeros(1, device="cuda"))
except Exception as e:
    print(mode, "torch FAILED:", e)
