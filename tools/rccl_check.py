"""GPU-box check of the calls bench.py's multi-rank path makes, at whatever world size torchrun gives
(one GPU box: world 1): init_process_group("nccl", device_id=...) over RCCL, broadcast of a conditioning-
sized tensor, barrier, all_reduce(MAX) of a float64 timer, destroy.  Prints one JSON line."""
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    rank, world, local = (int(os.environ.get(k, d)) for k, d in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    t0 = time.perf_counter()
    dist.init_process_group("nccl", device_id=dev)
    t_init = time.perf_counter() - t0
    enc = torch.full((1, 512, 2048), float(rank == 0), device=dev)
    dist.broadcast(enc, src=0)
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    ok = bool((enc == 1.0).all().item())
    if rank == 0:
        print(json.dumps({"backend": dist.get_backend(), "world": world, "init_s": round(t_init, 3),
                          "broadcast_ok": ok, "max_elapsed_s": round(float(el.item()), 3),
                          "torch": torch.__version__, "hip": torch.version.hip}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
