"""PMC probe target: u_qkv (dropout + keep bits) and the SwiGLU + u_d product, 20 launches each, product
library (run under rocprofv3 --pmc; see DESIGN.md section 5 'Forward LoRA u products')."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

M, K, F = 4800, 4096, 11008
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda").bfloat16()
bt = (torch.randn(48, K, device="cuda") * 0.05).bfloat16()
ws = ops.lora_skinny_ws(M, F, 8)
bits = torch.zeros(M * F // 8, dtype=torch.uint8, device="cuda")
out = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
for _ in range(20):
    ops.lora_skinny(x, bt, out, M, M, K, 3, 0, 2.0, ws=ws, dropout=(7, 0.05), keep_bits=bits)
gu = torch.randn(M, 2 * F, device="cuda").bfloat16()
h = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
bd = (torch.randn(16, F, device="cuda") * 0.05).bfloat16()
for _ in range(20):
    ops.swiglu_fwd_lora_down(gu, h, bd, out, M, M, F, 1, 2.0, ws=ws, dropout=(7, 0.05), keep_bits=bits)
for _ in range(20):
    ops.swiglu_fwd(gu, h)
torch.cuda.synchronize()
print("done")
