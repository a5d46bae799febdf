"""Where the forward LoRA u products' time goes (ablation build): u_qkv / u_o / the SwiGLU-fused u_d at the
step shape, without dropout, with dropout, with dropout + keep bits; a torch read-only reduction of the same
activation for the achievable stream rate; workgroup-target sweep (variant 100 + W).  JSON lines."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

M = 4800


def timeit(f, it=20):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def med(f):
    return round(sorted(timeit(f) for _ in range(3))[1], 1)


torch.manual_seed(0)
for name, K, nt in (("u_qkv", 4096, 3), ("u_o", 4096, 1)):
    xs = [torch.randn(M, K, device="cuda").bfloat16() for _ in range(2)]
    bt = (torch.randn(16 * nt, K, device="cuda") * 0.05).bfloat16()
    ws = torch.zeros(2 * ops.lora_skinny_ws(M, K, 8).numel(), device="cuda")  # room for the 2048-workgroup split
    bits = torch.zeros(M * K // 8, dtype=torch.uint8, device="cuda")
    out = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
    line = {"case": name, "MB": round(M * K * 2 / 1e6, 1)}
    for w in (0, 256, 512, 1024, 2048):
        call("ospo_set_skinny_variant", 4 if w == 0 else 100 + w)
        for tag, kw in (("nodrop", {}), ("drop", {"dropout": (7, 0.05)}), ("drop_bits", {"dropout": (7, 0.05), "keep_bits": bits})):
            if w not in (0, 512) and tag != "drop_bits":
                continue
            i = [0]

            def f():
                i[0] ^= 1
                ops.lora_skinny(xs[i[0]], bt, out, M, M, K, nt, 0, 2.0, ws=ws, **kw)
            line[f"{tag}_w{w}"] = med(f)
    call("ospo_set_skinny_variant", 4)
    line["torch_sum_read_us"] = med(lambda: xs[0].sum(1, dtype=torch.float32))
    print(json.dumps(line), flush=True)
F = 11008
gu = [torch.randn(M, 2 * F, device="cuda").bfloat16() for _ in range(2)]
h = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
bt = (torch.randn(16, F, device="cuda") * 0.05).bfloat16()
ws = ops.lora_skinny_ws(M, F, 8)
bits = torch.zeros(M * F // 8, dtype=torch.uint8, device="cuda")
out = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
line = {"case": "swiglu_u_d", "MB_read": round(M * 2 * F * 2 / 1e6, 1), "MB_write": round(M * F * 2 / 1e6, 1)}
for tag, kw in (("nodrop", {}), ("drop", {"dropout": (7, 0.05)}), ("drop_bits", {"dropout": (7, 0.05), "keep_bits": bits})):
    i = [0]

    def f():
        i[0] ^= 1
        ops.swiglu_fwd_lora_down(gu[i[0]], h, bt, out, M, M, F, 1, 2.0, ws=ws, **kw)
    line[tag] = med(f)
i = [0]


def sw():
    i[0] ^= 1
    ops.swiglu_fwd(gu[i[0]], h)
line["swiglu_fwd_alone"] = med(sw)
line["torch_copy_gu_us"] = med(lambda: gu[1].copy_(gu[0]))
print(json.dumps(line), flush=True)
