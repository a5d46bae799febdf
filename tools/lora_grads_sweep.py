"""Sweep the K-split count of the LoRA weight-gradient products (dA = g^T x, dB = dy^T u, fp32
atomics) on one layer's shapes (Janus-Pro-7B, 4 pairs, T = 600).  Prints us per product and split."""
import json
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

Mk, D, F, r, Rp = 4864, 4096, 11008, 16, 64
GROUPS = [("qkv", 3, D, D), ("o", 1, D, D), ("gu", 2, D, F), ("down", 1, F, D)]  # name, nmods, Kin, Nmod
SPLITS = [4, 8, 16, 32, 64]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


torch.manual_seed(0)
for name, nm, kin, nmod in GROUPS:
    g = (torch.randn(Mk, Rp, device="cuda") * 0.1).bfloat16()
    x = torch.randn(Mk, kin, device="cuda").bfloat16()
    dy = torch.randn(Mk, nm * nmod, device="cuda").bfloat16()
    u = (torch.randn(Mk, Rp, device="cuda") * 0.1).bfloat16()
    used = nm * r
    dA = torch.zeros(used, kin, device="cuda")
    dB = torch.zeros(nm * nmod, r, device="cuda")
    line = {"group": name}
    for ks in SPLITS:
        ta = timeit(lambda: ops.gemm_f32acc(g[:, :used], x, dA, a_kmajor=True, b_kmajor=True, k_splits=ks))
        tb = timeit(lambda: ops.gemm_f32acc(dy, u, dB, a_kmajor=True, b_kmajor=True, k_splits=ks, diag=(nmod, r)))
        line[f"s{ks}"] = {"dA_us": round(ta, 1), "dB_us": round(tb, 1)}
    print(json.dumps(line), flush=True)
