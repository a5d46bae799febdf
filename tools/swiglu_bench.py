"""Time the SwiGLU forward / backward kernels at the step shape (M = 4800, F = 11008) and report the
HBM rate over the bytes they must move."""
import json
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops

M, F = 4800, 11008


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


gu = torch.randn(M, 2 * F, device="cuda").bfloat16()
h = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
dh = torch.randn(M, F, device="cuda").bfloat16()
dgu = torch.empty_like(gu)
f = timeit(lambda: ops.swiglu_fwd(gu, h))
b = timeit(lambda: ops.swiglu_bwd(dh, gu, dgu))
print(json.dumps({"fwd_us": round(f, 1), "fwd_TBps": round(3 * M * F * 2 / f / 1e6, 2),
                  "bwd_us": round(b, 1), "bwd_TBps": round(5 * M * F * 2 / b / 1e6, 2)}))
