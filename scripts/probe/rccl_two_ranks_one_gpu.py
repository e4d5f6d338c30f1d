"""Probe: can two processes share the one GPU of a box as two RCCL ranks?
(torch.distributed nccl backend = RCCL).  Prints the all-reduce result per rank."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.full((4,), float(rank + 1), device="cuda:0")
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank}: {x.tolist()}", flush=True)
dist.destroy_process_group()
