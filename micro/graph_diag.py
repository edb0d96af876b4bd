"""Diagnostic (not a test): does graph replay in the library disturb torch's HIP init afterwards?"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
ctx = lvo.Context(lvo.abi.default_params(16))
for k in range(4):
    ctx.process_scan(lvo.synth.scan("vlp16", k))
print("hipGetLastError after frames:", hip.hipGetLastError())
n = ctypes.c_int(-1)
print("hipGetDeviceCount:", hip.hipGetDeviceCount(ctypes.byref(n)), n.value)
st = ctypes.c_int(-1)
print("hipStreamIsCapturing(null):", hip.hipStreamIsCapturing(None, ctypes.byref(st)), st.value)
import torch  # noqa: E402
print("torch available:", torch.cuda.is_available(), torch.cuda.device_count())
print(torch.zeros(3, device="cuda"))
