"""Time the attention kernels on the step's shape (S = 8 sequences, T = 600, 32 heads,
head_dim 128): forward, and backward (dQ + dK/dV, RoPE-fused).  OSPO_ATTN_WAVES=4|8
selects the workgroup size (read once per process)."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))  # A/B knobs: the ablation build
import json
import math
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops

S, T, H, hd = 8, 600, 32, 128


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
    D = H * hd
    rows = S * T
    qkv = (torch.randn(rows, 3 * D, device="cuda")).bfloat16()
    o = torch.empty(rows, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(S * H * T, device="cuda")
    delta = torch.empty(S * H * T, device="cuda")
    do = torch.randn(rows, D, device="cuda").bfloat16()
    dqkv = torch.empty(rows, 3 * D, device="cuda", dtype=torch.bfloat16)
    cos, sin = ops.rope_tables(T, hd, 1e4, "cuda")
    sc = 1 / math.sqrt(hd)
    f = timeit(lambda: ops.flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, sc))
    b = timeit(lambda: ops.flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, None, dqkv, S, T, H, hd, sc,
                                          rope_cos=cos, rope_sin=sin))
    ws = ops.flash_attn_bwd_ws(S, T, H, "cuda")
    b5 = timeit(lambda: ops.flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, ws, dqkv, S, T, H, hd, sc,
                                           rope_cos=cos, rope_sin=sin))
    fl = 4 * S * H * hd * T * (T + 1) / 2  # QK^T + PV, causal: the algorithmic forward
    print(json.dumps({"waves": os.environ.get("OSPO_ATTN_WAVES", "8"), "fwd_us": round(f, 1),
                      "bwd7_us": round(b, 1), "bwd5_us": round(b5, 1), "fwd_tflops": round(fl / f / 1e6, 1),
                      "bwd7_alg_tflops": round(2 * fl / b / 1e6, 1), "bwd5_alg_tflops": round(2 * fl / b5 / 1e6, 1),
                      "bwd5_frac_of_2500": round(2 * fl / b5 / 1e6 / 2500, 4)}))


if __name__ == "__main__":
    main()
