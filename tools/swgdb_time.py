"""ospo_swiglu_lora_gdb against the two launches it replaces (ospo_swiglu_bwd + ospo_lora_gdb over dgu) at the
step's gate|up shape (M = 4800, F = 11008), interleaved, HIP events.  Run on the GPU box:
python tools/swgdb_time.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402


def main():
    torch.manual_seed(0)
    M, F, r = 4800, 11008, 16
    dev = "cuda"
    dh = torch.randn(M, F, device=dev).bfloat16()
    gu = torch.randn(M, 2 * F, device=dev).bfloat16()
    dgu = torch.empty(M, 2 * F, device=dev, dtype=torch.bfloat16)
    bt = torch.randn(2 * r, F, device=dev).bfloat16()
    u = torch.randn(M, 64, device=dev).bfloat16()
    out = torch.empty(M, 64, device=dev, dtype=torch.bfloat16)
    dB = torch.zeros(2 * F, r, device=dev)
    ws = ops.lora_gdb_ws(M, 2, F, dev)

    def two():
        ops.swiglu_bwd(dh, gu, dgu)
        ops.lora_gdb(dgu, bt, u, out, dB, M, M, 2, F, 1.0, ws=ws)

    def swiglu_only():
        ops.swiglu_bwd(dh, gu, dgu)

    def gdb_only():
        ops.lora_gdb(dgu, bt, u, out, dB, M, M, 2, F, 1.0, ws=ws)

    def fused():
        ops.swiglu_lora_gdb(dh, gu, dgu, bt, u, out, dB, M, M, 1.0, ws=ws)

    two()
    torch.cuda.synchronize()
    ref_out, ref_dgu = out.clone(), dgu.clone()
    fused()
    torch.cuda.synchronize()
    check = {"dgu_equal": bool(torch.equal(dgu, ref_dgu)), "g_equal": bool(torch.equal(out, ref_out)),
             "g_max_rel": float(((out.float() - ref_out.float()).abs().max() / ref_out.float().abs().max()))}
    fns = {"two_launches": two, "swiglu_bwd": swiglu_only, "lora_gdb": gdb_only, "fused": fused}
    res = {k: [] for k in fns}
    for _ in range(7):
        for k, fn in fns.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 20 * 1e3)
    byts = (M * F * 3 + M * 2 * F) * 2  # dh, gate, up read + dgu written
    line = {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}
    line["fused_hbm_gbs"] = round(byts / line["fused"] / 1e3, 1)
    print(json.dumps({"variant": os.environ.get("OSPO_SWGDB", "0"), "shape": [M, F], "us": line, **check}), flush=True)


if __name__ == "__main__":
    main()
