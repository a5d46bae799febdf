"""Time the skinny LoRA products (ospo_lora_skinny) on the SimPO step's shapes, per kernel variant
(ablation build: 3 = v2, 4 = v3 LDS-line streaming, 100 + W = v3 with W target workgroups), and report
achieved HBM GB/s over the streamed activation (the algorithmic bytes) and the error against fp32."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops
from ospo_amd import dropout as Dm
from ospo_amd._lib import call

M = int(os.environ.get("SB_M", "4800"))
VARIANTS = [int(v) for v in os.environ.get("SB_VARIANTS", "3,4").split(",")]
CASES = [  # name, K (row length of the activation), n_tiles, a_koff (0 = dense), Kred, dropout
    ("u_qkv", 4096, 3, 0, 4096, True), ("u_o", 4096, 1, 0, 4096, True), ("u_gu", 4096, 2, 0, 4096, True),
    ("u_d", 11008, 1, 0, 11008, True),
    ("g_qkv", 12288, 3, 4096, 4096, False), ("g_o", 4096, 1, 0, 4096, False), ("g_gu", 22016, 2, 11008, 11008, False),
    ("g_d", 4096, 1, 0, 4096, False),
]


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


def main():
    torch.manual_seed(0)
    for name, K, nt, koff, kred, drop in CASES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        bt = (torch.randn(16 * nt, kred, device="cuda") * 0.05).bfloat16()
        ws = ops.lora_skinny_ws(M, kred, 8)
        dr = (12345, 0.05) if drop else None
        if koff:
            ref = torch.cat([x[:, j * koff:j * koff + kred].float() @ bt[16 * j:16 * (j + 1)].float().T
                             for j in range(nt)], 1) * 2.0
        else:
            xa = x.float()
            if drop:
                keep = torch.from_numpy(Dm.keep_mask(M, K, 12345, 0.05)).to("cuda")
                xa = torch.where(keep, (x.float() / 0.95).bfloat16().float(), torch.zeros((), device="cuda"))
            ref = xa @ bt.float().T * 2.0
        line = {"case": name}
        for v in VARIANTS:
            call("ospo_set_skinny_variant", v)
            out = torch.full((M, 64), float("nan"), device="cuda", dtype=torch.bfloat16)
            f = lambda: ops.lora_skinny(x, bt, out, M, M, kred, nt, koff, 2.0, ws=ws, dropout=dr)
            us = sorted(timeit(f) for _ in range(3))[1]
            err = float((out[:, :16 * nt].float() - ref).norm() / ref.norm())
            pad_ok = bool((out[:, 16 * nt:] == 0).all())
            line[f"v{v}"] = {"us": round(us, 1), "GBps": round(M * (kred * (nt if koff else 1)) * 2 / us / 1e3, 1),
                             "relerr": round(err, 6), "pad_zero": pad_ok}
        call("ospo_set_skinny_variant", 4)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
