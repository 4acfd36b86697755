"""Probe (not a test): can two RCCL ranks share one GPU on this box? Launched as two processes
with WORLD_SIZE=2 / RANK / MASTER_*; each rank all-reduces ones and prints the result."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch.cuda.set_device(0)
dist.init_process_group('gloo')
from manette_amd.comm import RcclComm  # noqa: E402
rank = dist.get_rank()
c = RcclComm(rank, 2, 0)
x = torch.full((1024,), float(rank + 1), device='cuda')
c.allreduce(x)
torch.cuda.synchronize()
print('rank', rank, 'sum', float(x[0]), flush=True)
c.close()
dist.destroy_process_group()
