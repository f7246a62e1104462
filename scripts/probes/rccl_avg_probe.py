import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
t = torch.arange(8, dtype=torch.float32, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.AVG); torch.cuda.synchronize()
m = torch.tensor([1.0], dtype=torch.float64, device=dev); dist.all_reduce(m, op=dist.ReduceOp.MAX)
print("rccl avg ok", t.tolist(), m.item(), torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else "")
dist.destroy_process_group()
