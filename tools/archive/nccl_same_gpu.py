"""Probe: can two ranks share one GPU with the nccl (RCCL) backend on this box?"""
import os
import torch
import torch.distributed as dist
rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.ones(4, device="cuda") * (rank + 1)
dist.all_reduce(t)
print(rank, t.tolist(), flush=True)
dist.barrier()
dist.destroy_process_group()
