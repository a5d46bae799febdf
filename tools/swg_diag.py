"""Step-by-step diagnostic of the fused down-proj dX + SwiGLU-backward GEMM (sync + print after each launch)."""
import sys
import time
import torch
from ospo_amd import _lib, ops
from ospo_amd._lib import call

_lib.lib()
torch.manual_seed(0)
dev = "cuda"


def rnd(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)


def step(name, fn):
    t = time.time()
    fn()
    torch.cuda.synchronize()
    print(f"{name}: ok {time.time() - t:.3f}s", flush=True)


for (M, F, K, K2, force) in [(600, 1024, 512, 64, 0), (4800, 11008, 4096, 64, 1), (4800, 11008, 4096, 64, 0)]:
    dy, w, a2, b2 = rnd(M, K), rnd(F, K, sc=0.05), rnd(M, K2), rnd(F, K2, sc=0.05)
    gu = rnd(M, 2 * F, sc=2.0)
    dh = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    ref = torch.empty(M, 2 * F, device=dev, dtype=torch.bfloat16)
    out = torch.zeros(M, 2 * F, device=dev, dtype=torch.bfloat16)
    call("ospo_gemm_force_split", force)
    tag = f"M{M} F{F} K{K} force{force}"
    step(tag + " gemm_nt+dropout", lambda: ops.gemm_nt(dy, w, dh, a2=a2, b2=b2, dropout=(7, 0.05)))
    step(tag + " swiglu_bwd", lambda: ops.swiglu_bwd(dh, gu, ref))
    step(tag + " fused no-drop", lambda: ops.gemm_nt_swiglu_bwd(dy, w, gu, out, a2=a2, b2=b2))
    step(tag + " fused drop", lambda: ops.gemm_nt_swiglu_bwd(dy, w, gu, out, a2=a2, b2=b2, dropout=(7, 0.05)))
    print(tag, "equal:", torch.equal(out, ref), flush=True)
call("ospo_gemm_force_split", 0)
