"""Probe: can two RCCL ranks share one GPU (torch.distributed nccl backend)? Prints the result."""
import os, torch, torch.distributed as dist
r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=r, world_size=w)
x = torch.full((29,), float(r + 1), device="cuda:0", dtype=torch.float64)
out = torch.empty((w * 29,), device="cuda:0", dtype=torch.float64)
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print("rank", r, "gather ok", out[::29].tolist(), flush=True)
dist.destroy_process_group()
