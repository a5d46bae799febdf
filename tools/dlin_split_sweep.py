"""K-split sweep of the one-launch decode Linear (ablation build: ospo_set_gemv_splits) on the T2I decode
shapes (R = 32, 7B): q|k|v + RMSNorm + KV store, o + residual + ss, gate|up + RMSNorm + SwiGLU, down + residual +
ss.  Two weight copies alternate so no launch re-reads its weight from the 256 MB MALL.  JSON lines."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

R, D, F, H, Tmax = 32, 4096, 11008, 32, 640
dev = "cuda"


def timeit(f, it=30):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


torch.manual_seed(0)
x = torch.randn(R, D, device=dev).bfloat16()
xf = torch.randn(R, F, device=dev).bfloat16()
lnw = (1 + 0.1 * torch.randn(D, device=dev)).bfloat16()
ss = torch.rand(D // 128, 32, device=dev) * 100
ss_out = torch.zeros(D // 128, 32, device=dev)
pos = torch.tensor([336], dtype=torch.int32, device=dev)
cos, sin = ops.rope_tables(Tmax, 128, 1e4, dev)
kc, vc = (torch.zeros(R, H, Tmax, 128, device=dev, dtype=torch.bfloat16) for _ in range(2))
shapes = {"qkv": (3 * D, D), "o": (D, D), "gu": (2 * F, D), "down": (D, F)}
W = {k: [ops.tile_decode_weight((torch.randn(n, kk, device=dev) * 0.02).bfloat16()) for _ in range(2)]
     for k, (n, kk) in shapes.items()}
W["gu"] = [ops.tile_decode_weight(ops.interleave_gate_up((torch.randn(2 * F, D, device=dev) * 0.02).bfloat16()))
           for _ in range(2)]
ws = torch.zeros(8 * max(ops.decode_linear_ws(R, n, k, dev).numel() for n, k in shapes.values()), device=dev)
outs = {"qkv": torch.empty(R, D, device=dev, dtype=torch.bfloat16), "o": torch.empty(R, D, device=dev, dtype=torch.bfloat16),
        "gu": torch.empty(R, F, device=dev, dtype=torch.bfloat16), "down": torch.empty(R, D, device=dev, dtype=torch.bfloat16)}
calls = {
    "qkv": lambda w: ops.decode_linear(x, w, outs["qkv"], ws, epi="kv", norm=(ss, lnw, 1e-6),
                                       kv=(pos, (cos, sin), kc, vc, H, Tmax)),
    "o": lambda w: ops.decode_linear(x, w, outs["o"], ws, residual=x, ss_out=ss_out),
    "gu": lambda w: ops.decode_linear(x, w, outs["gu"], ws, epi="swiglu", norm=(ss, lnw, 1e-6)),
    "down": lambda w: ops.decode_linear(xf, w, outs["down"], ws, residual=x, ss_out=ss_out),
}
for name, (n, k) in shapes.items():
    line = {"shape": name, "MB": round(n * k * 2 / 1e6, 1)}
    for s in (0, 2, 4, 8, 16):
        call("ospo_set_gemv_splits", s)
        i = [0]

        def f():
            i[0] ^= 1
            calls[name](W[name][i[0]])
        us = sorted(timeit(f) for _ in range(3))[1]
        line[f"s{s}"] = {"us": round(us, 1), "TBps": round(n * k * 2 / us / 1e6, 2)}
    call("ospo_set_gemv_splits", 0)
    print(json.dumps(line), flush=True)
