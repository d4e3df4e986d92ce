"""Two ranks on one GPU: all-reduce / reduce-scatter / all-gather over RCCL and check the values."""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(int(os.environ["LOCAL_RANK"]) % torch.cuda.device_count())
dist.init_process_group("nccl", init_method="env://")
x = torch.full((1 << 20,), float(rank + 1), device="cuda")
dist.all_reduce(x)
assert torch.all(x == world * (world + 1) / 2), x[:4]
out = torch.empty((1 << 20) // world, device="cuda")
dist.reduce_scatter_tensor(out, torch.ones(1 << 20, device="cuda"))
assert torch.all(out == world)
g = torch.empty(world * 4, device="cuda")
dist.all_gather_into_tensor(g, torch.full((4,), float(rank), device="cuda"))
assert g.tolist() == [float(r) for r in range(world) for _ in range(4)]
torch.cuda.synchronize()
dist.barrier()
print(f"rank {rank}: rccl probe ok", flush=True)
dist.destroy_process_group()
