"""A/B of the LoRA skinny products (ospo_set_skinny_variant 1 / 2) on the step's shapes (M = 4800),
interleaved rounds, both checked against each other and against fp32 torch."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))  # A/B knobs: the ablation build
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

M = 4800
r = int(os.environ.get("SK_R", "16"))
VA, VB = (int(v) for v in os.environ.get("SK_VARIANTS", "1,2").split(","))
CASES = [  # name, K (contraction per module), nmods, dense(u)?, dropout
    ("u_qkv", 4096, 3, True, 0.05), ("u_o", 4096, 1, True, 0.05), ("u_gu", 4096, 2, True, 0.05),
    ("u_down", 11008, 1, True, 0.05), ("g_qkv", 4096, 3, False, 0), ("g_o", 4096, 1, False, 0),
    ("g_gu", 11008, 2, False, 0), ("g_down", 4096, 1, False, 0),
]


def timeit(fn, it=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


torch.manual_seed(0)
for name, K, nm, dense, p in CASES:
    used = nm * r
    Rp = (used + 63) // 64 * 64
    if dense:
        A = torch.randn(M, K, device="cuda").bfloat16()
        Bt = torch.zeros(Rp, K, device="cuda").bfloat16()
        Bt[:used] = (torch.randn(used, K, device="cuda") * 0.02).bfloat16()
        Ktot, nt, koff, mt = K, (used + 15) // 16, 0, 1
    else:
        A = torch.randn(M, nm * K, device="cuda").bfloat16()
        Bt = (torch.randn(used, K, device="cuda") * 0.02).bfloat16()
        Ktot, nt, koff, mt = K, nm * r // 16, K, r // 16
    out = torch.empty(M, Rp, device="cuda", dtype=torch.bfloat16)
    xd = torch.empty(M, K, device="cuda", dtype=torch.bfloat16) if dense and p > 0 else None
    ws = ops.lora_skinny_ws(M, Ktot, max(nt, 8), "cuda")
    kw = dict(b_rows=used, ws=ws)
    if dense and p > 0:
        kw.update(dropout=(1234, p), xd=xd)
    if not dense:
        kw = dict(ws=ws, module_tiles=mt)

    def run():
        ops.lora_skinny(A, Bt, out, M, M, Ktot, nt, koff, 2.0, **kw)
    res, outs = {VA: [], VB: []}, {}
    for _ in range(5):
        for v in (VA, VB):
            call("ospo_set_skinny_variant", v)
            res[v].append(timeit(run))
    for v in (VA, VB):
        call("ospo_set_skinny_variant", v)
        out.fill_(7)
        run()
        outs[v] = (out.clone(), xd.clone() if xd is not None else None)
    call("ospo_set_skinny_variant", 2)
    nbytes = A.numel() * 2 * (2 if xd is not None else 1)
    line = {"case": name, "K": K, "nmods": nm, "r": r,
            "a_vs_b_relerr": float((outs[VA][0].float() - outs[VB][0].float()).norm() / outs[VA][0].float().norm()),
            "xd_equal": bool(torch.equal(outs[VA][1], outs[VB][1])) if xd is not None else None}
    for v in (VA, VB):
        t = sorted(res[v])[2]
        line[f"v{v}"] = {"us": round(t * 1e3, 1), "GBps": round(nbytes / t / 1e6, 1)}
    print(json.dumps(line), flush=True)
