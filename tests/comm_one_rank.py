"""Every Comm collective through the process group at world size 1
(KAFKA_FORCE_DIST=1 under torch.distributed.run): on a GPU box the RCCL
("nccl") code paths with device tensors -- C1 sums, the band all-reduce, C3
gather, C4 broadcasts, object gathers, device barrier, an empty C2 batch.
Run by tests/test_gpu.py and tests/test_distributed.py (gloo on the CPU);
prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from kafka_inferenceengine_amd.parallel.comm import Comm  # noqa: E402


def main():
    dev = None if torch.cuda.is_available() else "cpu"
    comm = Comm.from_env(device=dev)
    assert comm.distributed and comm.world == 1, (comm.distributed, comm.world)
    d = comm.device
    out = {"backend": torch.distributed.get_backend(), "device": str(d)}
    v = torch.tensor([1.25], dtype=torch.float64, device=d)
    out["sum_f64"] = comm.sum_f64(v)
    pend = comm.sum_f64_async(torch.tensor([0.5, 2.0], dtype=torch.float64, device=d))
    out["sum_f64_async"] = [pend.column(0).result(), pend.column(1).result()]
    out["sum_int"] = comm.sum_int(7)
    out["max_float"] = comm.max_float(3.5)
    t = torch.arange(6, dtype=torch.float32, device=d)
    comm.all_reduce_(t)
    out["all_reduce"] = t.cpu().tolist()
    comm.barrier()
    hdr, buf = comm.broadcast_packed([("k", 3)], np.arange(3.0))
    out["broadcast_packed"] = [hdr, buf.tolist()]
    out["broadcast_object"] = comm.broadcast_object({"a": 1})
    out["gather_object"] = comm.gather_object({"r": comm.rank})
    g = comm.gather_to_root(torch.ones((2, 3), device=d), [3])
    out["gather_to_root"] = list(g.shape)
    comm.exchange_fields_async([torch.zeros(4, device=d)], [None], [torch.zeros(4, device=d)], [None]).wait()
    if d.type == "cuda":
        torch.cuda.synchronize()
    print(json.dumps(out), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
