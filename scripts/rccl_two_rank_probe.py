"""Does RCCL run two ranks on ONE GPU?  If it does, the engine's RCCL code
paths (device all-gather of the C1 norm, barrier with device_ids, device
broadcast of packed setup data, batch_isend_irecv halos, gather to root) can
be exercised on a one-GPU box instead of only through gloo rehearsals.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
        --master-addr=127.0.0.1 --master-port=29633 scripts/rccl_two_rank_probe.py

Every rank uses cuda:0.  Prints one JSON line per rank."""
import datetime
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from kafka_inferenceengine_amd.parallel.comm import Comm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend="nccl", timeout=datetime.timedelta(seconds=60), device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    comm = Comm(rank, world, dev)
    res = {"rank": rank, "world": world, "backend": dist.get_backend()}
    # C1: async device all-gather of two norms, summed in rank order
    loc = torch.tensor([1.0 + rank, 10.0 * (rank + 1)], dtype=torch.float64, device=dev)
    pend = comm.sum_f64_async(loc)
    res["c1"] = [pend.result(0), pend.result(1)]
    comm.barrier()
    # C4: packed broadcast of a float64 buffer from rank 0
    hdr, buf = comm.broadcast_packed(["x"] if rank == 0 else None,
                                     np.arange(5, dtype=np.float64) if rank == 0 else None)
    res["c4"] = [hdr, buf.tolist()]
    # C2: halo rows to the neighbours (posted, then waited on the stream)
    rows = torch.full((2, 8), float(rank), device=dev)
    up = torch.empty((2, 8), device=dev)
    down = torch.empty((2, 8), device=dev)
    p = comm.exchange_halo_async(rows, rows, up, down)
    p.wait()
    torch.cuda.synchronize()
    res["c2_up"] = float(up[0, 0]) if rank > 0 else None
    res["c2_down"] = float(down[0, 0]) if rank < world - 1 else None
    # C3: variable-length gather to rank 0
    blk = torch.full((3, 4 + rank), float(rank), device=dev)
    g = comm.gather_to_root(blk, [4 + r for r in range(world)])
    res["c3"] = None if g is None else list(g.shape)
    res["max"] = comm.max_float(float(rank))
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
