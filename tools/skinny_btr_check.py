"""Outputs of the skinny LoRA products for fixed inputs (ablation build), saved for a bit-for-bit comparison
of two library variants run in separate processes: python tools/skinny_btr_check.py OUT.pt [--compare A.pt B.pt]"""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    bad = {k: int((a[k] != b[k]).sum()) for k in a}
    print("mismatching elements:", bad)
    sys.exit(1 if any(bad.values()) else 0)

from ospo_amd import ops  # noqa: E402

M, F = 4800, 11008
res = {}
torch.manual_seed(0)
for name, K, nt in (("qkv", 4096, 3), ("o", 4096, 1), ("gu", 4096, 2), ("m37", 1344, 4)):
    Mx = M if name != "m37" else 37
    x = torch.randn(Mx, K, device="cuda").bfloat16()
    bt = (torch.randn(16 * nt - (3 if name == "m37" else 0), K, device="cuda") * 0.05).bfloat16()
    ws = ops.lora_skinny_ws(Mx, K, 8)
    bits = torch.zeros((Mx * K + 7) // 8, dtype=torch.uint8, device="cuda")
    out = torch.zeros(Mx, 64, device="cuda", dtype=torch.bfloat16)
    ops.lora_skinny(x, bt, out, Mx, Mx, K, nt, 0, 2.0, ws=ws, dropout=(7, 0.05), keep_bits=bits)
    res[name] = out.cpu()
    res[name + "_bits"] = bits.cpu()
    out2 = torch.zeros(Mx, 64, device="cuda", dtype=torch.bfloat16)
    ops.lora_skinny(x, bt, out2, Mx, Mx, K, nt, 0, 2.0, ws=ws)
    res[name + "_nodrop"] = out2.cpu()
gu = torch.randn(M, 2 * F, device="cuda").bfloat16()
h = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
bd = (torch.randn(16, F, device="cuda") * 0.05).bfloat16()
ws = ops.lora_skinny_ws(M, F, 8)
bits = torch.zeros(M * F // 8, dtype=torch.uint8, device="cuda")
out = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
ops.swiglu_fwd_lora_down(gu, h, bd, out, M, M, F, 1, 2.0, ws=ws, dropout=(7, 0.05), keep_bits=bits)
res["ud"], res["ud_h"], res["ud_bits"] = out.cpu(), h.cpu(), bits.cpu()
torch.save(res, sys.argv[1])
print("saved", sys.argv[1])
