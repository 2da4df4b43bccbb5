"""Device-vs-host check of the packed Cholesky paths (invert, analysis)."""
import sys
import numpy as np
import torch
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/tests")
import kernel_cases as C  # noqa: E402
from kafka_inferenceengine_amd.ops import kernels as K  # noqa: E402

rng = np.random.default_rng(0)
B = C.spd_blocks(rng, 8, 7, 5.0)
for dev in ("cpu", "cuda"):
    out = torch.zeros((28, 8), device=dev)
    st = torch.zeros(8, dtype=torch.uint8, device=dev)
    K.invert(7, C.packed(B, dev), out, status=st)
    print(dev, "invert", out[:4, 0].cpu().numpy(), st.cpu().numpy())
prob = C.tip_problem(N=8, seed=11)
for dev in ("cpu", "cuda"):
    tab = C.table(prob, dev)
    xo = torch.zeros((7, 8), device=dev); ao = torch.zeros((28, 8), device=dev)
    st = torch.zeros(8, dtype=torch.uint8, device=dev)
    K.analysis(7, tab, C.soa(prob["x"], dev), C.soa(prob["xf"], dev), C.packed(prob["Pf"], dev), xo, ao, None, st, None)
    print(dev, "analysis fast", xo[:, 0].cpu().numpy(), st.cpu().numpy())
    K.analysis(7, tab, C.soa(prob["x"], dev), C.soa(prob["xf"], dev), C.packed(prob["Pf"], dev), xo, ao, None, st, None,
               fast=False)
    print(dev, "analysis generic", xo[:, 0].cpu().numpy(), st.cpu().numpy())
