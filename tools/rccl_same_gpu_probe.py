"""Probe (GPU box, not part of the product): can two RCCL ranks share one GPU?
Run as: timeout -k 10 120 python -m torch.distributed.run --nproc-per-node 2
        --master-addr 127.0.0.1 --master-port 29611 tools/rccl_same_gpu_probe.py
If they can, the real-rank (world > 1) CUDA branch of sharded._SliceExchange
(batch_isend_irecv on a side stream) can run on a one-GPU box."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((4,), float(rank + 1), device="cuda")
dist.all_reduce(t)
peer = (rank + 1) % world
src = torch.full((1 << 20,), float(rank), device="cuda", dtype=torch.float64)
dst = torch.empty_like(src)
ops = [dist.P2POp(dist.isend, src, peer), dist.P2POp(dist.irecv, dst, (rank - 1) % world)]
for w in dist.batch_isend_irecv(ops):
    w.wait()
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {t.tolist()} recv {dst[0].item()} (expect {(rank - 1) % world})", flush=True)
dist.destroy_process_group()
