"""Diagnostic: where does the MX8 GEMM differ from the dequantized fp32 product?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ospo_amd import ops
from oracle import mx8_ref as MX
torch.manual_seed(0)
DEV = "cuda"
for (M, N, K) in [(256, 256, 128), (256, 256, 256), (600, 512, 256)]:
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    b = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    A8, B8 = ops.MX8.of(a), ops.MX8.of(b)
    ops.gemm_nt_mx8(A8, B8, out)
    fa = MX.fake_quant(a.cpu()).double()
    fb = MX.fake_quant(b.cpu()).double()
    ref = fa @ fb.T
    d = (out.cpu().double() - ref)
    rel = d.abs() / ref.abs().clamp_min(1e-3)
    print(M, N, K, "max rel", float(rel.max()), "mean |d|", float(d.abs().mean()), "mean |ref|", float(ref.abs().mean()))
    r, c = divmod(int(rel.argmax()), N)
    print("  worst at", r, c, float(out[r, c]), float(ref[r, c]))
    # error pattern by row mod 64 and col mod 64
    e = d.abs()
    print("  row%64 err:", [round(float(e[i::64].mean()) * 1e4, 2) for i in range(0, 64, 8)])
    print("  col%64 err:", [round(float(e[:, i::64].mean()) * 1e4, 2) for i in range(0, 64, 8)])
    # check q bytes equal device vs oracle
    q, s = MX.quantize_mx8(a.cpu())
    print("  quant equal:", torch.equal(A8.q.cpu(), q), torch.equal(A8.s.cpu(), MX.scale_tile_layout(s)))
    # hypothesis: per-row scale vs the kernel -> compute implied ratio
    ratio = (out.cpu().double() / ref)
    print("  median ratio", float(ratio.median()))
