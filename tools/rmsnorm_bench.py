"""Time the RMSNorm kernels at the step shape (M = 4864 rows, D = 4096): GB/s of the algorithmic bytes."""
import sys, os, torch, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops
M, D = 4864, 4096
x = torch.randn(M, D, device="cuda").bfloat16(); dy = torch.randn(M, D, device="cuda").bfloat16()
dres = torch.randn(M, D, device="cuda").bfloat16(); w = torch.randn(D, device="cuda").bfloat16()
y = torch.empty_like(x); rstd = torch.empty(M, device="cuda"); dx = torch.empty_like(x)
ops.rmsnorm_fwd(x, w, y, rstd, 1e-6)
def t(fn, it=50):
    fn(); e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / it * 1e3
ub = t(lambda: ops.rmsnorm_bwd(dy, x, w, rstd, dx, dres=dres))
uf = t(lambda: ops.rmsnorm_fwd(x, w, y, rstd, 1e-6))
print(json.dumps({"bwd_us": round(ub, 1), "bwd_TBps": round(4 * M * D * 2 / ub / 1e6, 2), "fwd_us": round(uf, 1), "fwd_TBps": round(2 * M * D * 2 / uf / 1e6, 2)}))
