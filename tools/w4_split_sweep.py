"""Split-K tail sweep for the w4 GEMM on the step shapes: the library's cost model (split 0) against pinned
tail splits 1..8 (ops.gemm_nt split=), interleaved, HIP events, medians.  The model's constants were fitted
on the SP8 kernel (T = 1.9 us per K-tile); this checks them on the w4 loop.  Run on the GPU box:
python tools/w4_split_sweep.py  (SWEEP_M=9600: config 3's per-GPU batch, 8 pairs; round 5)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

M = int(os.environ.get("SWEEP_M", "4800"))
MG = M // 600 * 576  # gen_head rows: the 576 image positions of each sequence
SHAPES = [("qkv_fwd", M, 12288, 4096, 64), ("o_fwd", M, 4096, 4096, 64), ("gu_fwd", M, 22016, 4096, 64),
          ("down_fwd", M, 4096, 11008, 64), ("down_dx", M, 11008, 4096, 64), ("gu_dx", M, 4096, 22016, 64),
          ("qkv_dx", M, 4096, 12288, 64), ("gh2_fwd", MG, 16384, 4096, 0), ("gh2_dx", MG, 4096, 16384, 0)]
SPLITS = [0, 1, 2, 3, 4, 5, 6, 8]


def main():
    torch.manual_seed(0)
    dev = "cuda"
    out_all = {}
    for name, m, n, k, k2 in SHAPES:
        a = (torch.rand(m, k, device=dev) * 2 - 1).bfloat16()
        b = (torch.rand(n, k, device=dev) * 2 - 1).bfloat16()
        a2 = (torch.rand(m, k2, device=dev) * 2 - 1).bfloat16() if k2 else None
        b2 = (torch.rand(n, k2, device=dev) * 2 - 1).bfloat16() if k2 else None
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        drop = name.endswith("_dx") and k2
        bits = torch.randint(0, 256, (m * n // 8,), device=dev, dtype=torch.uint8) if drop else None
        res = {s: [] for s in SPLITS}

        def fn(s):
            if drop:
                ops.gemm_nt(a, b, out, a2=a2, b2=b2, dropout=(5, 0.05), keep_bits=bits, split=s)
            else:
                ops.gemm_nt(a, b, out, a2=a2, b2=b2, split=s)
        for _ in range(5):
            for s in SPLITS:
                fn(s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn(s)
                e1.record()
                torch.cuda.synchronize()
                res[s].append(e0.elapsed_time(e1) / 10 * 1e3)
        med = {s: round(sorted(v)[2], 1) for s, v in res.items()}
        best = min((v, s) for s, v in med.items() if s)
        line = {"shape": name, "us": med, "model_us": med[0], "best_pinned": best[1], "best_us": best[0],
                "model_minus_best_us": round(med[0] - best[0], 1)}
        out_all[name] = line
        print(json.dumps(line), flush=True)
    tot = sum(v["model_minus_best_us"] for v in out_all.values())
    print(json.dumps({"sum_model_minus_best_us_per_shape_set": round(tot, 1)}), flush=True)


if __name__ == "__main__":
    main()
