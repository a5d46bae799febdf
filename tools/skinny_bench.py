"""Time the skinny LoRA products (ospo_lora_skinny) on the SimPO step's shapes and
report achieved HBM GB/s over the streamed activation (the algorithmic bytes)."""
import json
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops

M = 4800
CASES = [  # name, K (row length of the activation), n_tiles, a_koff (0 = dense), Kred
    ("u_qkv", 4096, 3, 0, 4096), ("u_o", 4096, 1, 0, 4096), ("u_gu", 4096, 2, 0, 4096), ("u_d", 11008, 1, 0, 11008),
    ("g_qkv", 12288, 3, 4096, 4096), ("g_o", 4096, 1, 0, 4096), ("g_gu", 22016, 2, 11008, 11008),
    ("g_d", 4096, 1, 0, 4096),
]


def main():
    for name, K, nt, koff, kred in CASES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        bt = torch.randn(16 * nt, kred, device="cuda").bfloat16()
        out = torch.empty(M, 64, device="cuda", dtype=torch.bfloat16)
        ws = ops.lora_skinny_ws(M, kred, nt)
        f = lambda: ops.lora_skinny(x, bt, out, M, M, kred, nt, koff, 2.0, ws=ws)
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(json.dumps({"case": name, "us": round(us, 1), "GBps": round(M * K * 2 / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
