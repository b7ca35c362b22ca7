"""Two RCCL ranks on one GPU: does RCCL accept it (all_reduce, all_gather,
all_to_all on device tensors)? usage (one box, one GPU):
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P tools/rccl_probe.py"""
import os
import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=rank, world_size=world)
x = torch.full((1024,), float(rank + 1), device=dev)
dist.all_reduce(x)
g = torch.empty(world * 4, device=dev)
dist.all_gather_into_tensor(g, torch.full((4,), float(rank), device=dev))
a = torch.empty(world * 2, device=dev)
dist.all_to_all_single(a, torch.arange(world * 2, device=dev, dtype=torch.float32) + 10 * rank)
torch.cuda.synchronize()
print("rank", rank, "all_reduce", x[0].item(), "all_gather", g.tolist(), "all_to_all", a.tolist(), flush=True)
dist.barrier()
dist.destroy_process_group()
