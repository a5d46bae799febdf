"""Diagnostic: ospo_decode_linear (plain, no residual) against the GEMV + split-sum path, per shape and R:
fraction of mismatching outputs, and the mismatching row groups / rows."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

DEV = "cuda"
for R in (4, 32):
    for name, N, K in (("o", 4096, 4096), ("qkv", 12288, 4096), ("gu", 22016, 4096), ("down", 4096, 11008),
                       ("n1k8", 1024, 8192), ("n128k4", 128, 4096)):
        torch.manual_seed(0)
        x = torch.randn(R, K, device=DEV).bfloat16()
        w = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
        wt = ops.tile_decode_weight(w)
        o1 = torch.zeros(R, N, device=DEV, dtype=torch.bfloat16)
        o2 = torch.zeros_like(o1)
        gws = ops.decode_gemv_ws(R, N, K, DEV)
        lws = ops.decode_linear_ws(R, N, K, DEV)
        ops.decode_gemv(x, wt, o1, ws=gws)
        ops.decode_linear(x, wt, o2, lws)
        torch.cuda.synchronize()
        bad = (o1 != o2)
        groups = sorted(set((bad.nonzero()[:, 1] // 128).tolist()))
        rows = sorted(set(bad.nonzero()[:, 0].tolist()))
        ref = (x.float() @ w.float().t())
        e1 = float((o1.float() - ref).abs().max())
        e2 = float((o2.float() - ref).abs().max())
        print(f"R={R} {name}: mismatch {float(bad.float().mean()):.4f} groups {groups[:12]}{'...' if len(groups) > 12 else ''} "
              f"({len(groups)}) rows {rows[:8]} err gemv {e1:.3g} dlin {e2:.3g}", flush=True)
