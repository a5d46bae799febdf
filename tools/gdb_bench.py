"""Time the fused LoRA backward stream (ospo_lora_gdb: g = s dy.B and dB += dy^T u) on the step's
four groups (M = 4800; q|k|v, o, gate|up, down) and report dy's read rate."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops

M = 4800
GROUPS = [("qkv", 3, 4096), ("o", 1, 4096), ("gu", 2, 11008), ("down", 1, 4096)]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    out = {}
    for name, nm, Nmod in GROUPS:
        dy = torch.randn(M, nm * Nmod, device="cuda").bfloat16()
        bt = (torch.randn(nm * 16, Nmod, device="cuda") * 0.02).bfloat16()
        Rp = 64 if nm * 16 <= 64 else 128
        u = torch.randn(M, Rp, device="cuda").bfloat16()
        g = torch.empty(M, Rp, device="cuda", dtype=torch.bfloat16)
        dB = torch.zeros(nm * Nmod, 16, device="cuda")
        ws = ops.lora_gdb_ws(M, nm, Nmod, "cuda")
        us = timeit(lambda: ops.lora_gdb(dy, bt, u, g, dB, M, M, nm, Nmod, 2.0, ws))
        out[name] = {"us": round(us, 1), "dy_TBps": round(dy.numel() * 2 / us / 1e6, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
