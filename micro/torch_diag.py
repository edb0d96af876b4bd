"""Diagnostic (not a test): why torch sees no GPU after an aloam context exists."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from lvo_amd_loader import lvo  # noqa: E402

before = {k: v for k, v in os.environ.items() if "VISIBLE" in k or k.startswith("HIP") or k.startswith("ROC") or k.startswith("HSA")}
ctx = lvo.Context(lvo.abi.default_params(16))
after = {k: v for k, v in os.environ.items() if "VISIBLE" in k or k.startswith("HIP") or k.startswith("ROC") or k.startswith("HSA")}
print("env before", before)
print("env changed", {k: (before.get(k), after.get(k)) for k in set(before) | set(after) if before.get(k) != after.get(k)})
import torch  # noqa: E402
import torch.cuda as tc  # noqa: E402
for name in ("_raw_device_count_amdsmi", "_device_count_amdsmi", "_raw_device_count_nvml"):
    f = getattr(tc, name, None)
    if f:
        try:
            print(name, f())
        except Exception as e:
            print(name, "EXC", e)
try:
    print("_cuda_getDeviceCount", torch._C._cuda_getDeviceCount())
except Exception as e:
    print("getDeviceCount EXC", e)
print("is_available", torch.cuda.is_available())
