"""Probe: can RCCL run two ranks on ONE GPU (a multi-rank rehearsal of the
bench's RCCL gather on the 1-GPU box)?  Two spawned ranks, backend nccl, both
on cuda:0, one all_reduce + one gather; prints the outcome per rank."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def rank_main(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=dev)
        x = torch.ones(1, device=dev)
        dist.all_reduce(x)
        bufs = [torch.empty(4, device=dev) for _ in range(2)] if rank == 0 else None
        dist.gather(torch.full((4,), float(rank), device=dev), bufs, dst=0)
        torch.cuda.synchronize()
        q.put((rank, "ok", float(x.item()), [b.tolist() for b in bufs] if bufs else None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e)[:400], None))


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in range(2):
        print(q.get(timeout=90), flush=True)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    sys.exit(0)
