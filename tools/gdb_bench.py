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


def run(r):
    out = {}
    for name, nm, Nmod in GROUPS:
        dy = torch.randn(M, nm * Nmod, device="cuda").bfloat16()
        bt = (torch.randn(nm * r, Nmod, device="cuda") * 0.02).bfloat16()
        Rp = 64 if nm * r <= 64 else 128
        u = torch.randn(M, Rp, device="cuda").bfloat16()
        g = torch.empty(M, Rp, device="cuda", dtype=torch.bfloat16)
        dB = torch.zeros(nm * Nmod, r, device="cuda")
        ws = ops.lora_gdb_ws(M, nm, Nmod, "cuda", r=r)
        us = timeit(lambda: ops.lora_gdb(dy, bt, u, g, dB, M, M, nm, Nmod, 2.0, ws, r=r))
        out[name] = {"us": round(us, 1), "dy_TBps": round(dy.numel() * 2 / us / 1e6, 2)}
        del dy, u, g, dB, ws
    return out


def main():
    # argv: r (16 / 32), then the ablation variants to interleave (comma-separated env names, "" = default)
    r = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    variants = sys.argv[2].split(",") if len(sys.argv) > 2 else [""]
    for rep in range(2):
        for v in variants:
            for k in ("OSPO_GDB_NS6", "OSPO_GDB_NS2", "OSPO_GDB_NS3", "OSPO_GDB_RSB4", "OSPO_NT_GDB", "OSPO_GDB_MINWG", "OSPO_GDB_RSB8", "OSPO_GDB_RED8", "OSPO_GDB_RED16"):
                os.environ.pop(k, None)
            for k in filter(None, v.split("+")):
                os.environ[k] = "1"
            print(json.dumps({"r": r, "variant": v or "default", "rep": rep, **run(r)}), flush=True)


if __name__ == "__main__":
    main()
