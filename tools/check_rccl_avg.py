"""Check that the RCCL backend accepts ReduceOp.AVG (one rank, cuda:0)."""
import os

import torch
import torch.distributed as d

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
d.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
t = torch.arange(8, dtype=torch.float32, device="cuda")
d.all_reduce(t, op=d.ReduceOp.AVG)
torch.cuda.synchronize()
print("AVG ok", t.tolist())
d.destroy_process_group()
