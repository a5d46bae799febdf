"""Run one GEMM shape/variant ITERS times (for rocprofv3 PMC collection)."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))  # A/B knobs: the ablation build
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops
from ospo_amd._lib import call

M, N, K, K2 = (int(x) for x in os.environ.get("GO_SHAPE", "4800,12288,4096,64").split(","))
V = int(os.environ.get("GO_VARIANT", "1"))
IT = int(os.environ.get("GO_ITERS", "20"))
torch.manual_seed(0)
a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
a2 = (torch.rand(M, K2, device="cuda") * 2 - 1).bfloat16() if K2 else None
b2 = (torch.rand(N, K2, device="cuda") * 2 - 1).bfloat16() if K2 else None
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
call("ospo_set_gemm_variant", V)
for _ in range(IT):
    ops.gemm_nt(a, b, out, a2=a2, b2=b2)
torch.cuda.synchronize()
if os.environ.get("GO_BLAS"):
    ref = torch.empty_like(out)
    for _ in range(IT):
        torch.matmul(a, b.t(), out=ref)
    torch.cuda.synchronize()
