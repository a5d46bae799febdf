"""SwiGLU + u_d (ospo_swiglu_fwd_lora_down, dropout + keep bits) at several workgroup targets (ablation build,
ospo_set_skinny_variant(100 + W)); alternating two inputs.  JSON line."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402


def med(f, it=20):
    def timeit():
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            f()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / it * 1e3
    return round(sorted(timeit() for _ in range(3))[1], 1)


M, F = 4800, 11008
gu = [torch.randn(M, 2 * F, device="cuda").bfloat16() for _ in range(2)]
h = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
bt = (torch.randn(16, F, device="cuda") * 0.05).bfloat16()
ws = torch.zeros(4 * ops.lora_skinny_ws(M, F, 8).numel(), device="cuda")
bits = torch.zeros(M * F // 8, dtype=torch.uint8, device="cuda")
out = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
line = {"case": "swiglu_u_d drop+bits"}
for w in (512, 768, 1024, 1536, 2048):
    call("ospo_set_skinny_variant", 100 + w)
    i = [0]

    def f():
        i[0] ^= 1
        ops.swiglu_fwd_lora_down(gu[i[0]], h, bt, out, M, M, F, 1, 2.0, ws=ws, dropout=(7, 0.05), keep_bits=bits)
    line[f"w{w}"] = med(f)
call("ospo_set_skinny_variant", 4)
print(json.dumps(line), flush=True)
