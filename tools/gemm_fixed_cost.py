"""Per-tile fixed cost of the 256x256 GEMM: time one full round (256 tiles) and two rounds at
several K, fit t = fixed + K-tiles * slope (least squares).  Prints one JSON line per grid."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops

KS = [1024, 2048, 4096, 8192, 16384]


def timeit(fn, it=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    torch.manual_seed(0)
    for M, N in ((4096, 4096), (8192, 4096), (4096, 8192)):
        ts = []
        for K in KS:
            a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ref = torch.empty_like(out)
            t = sorted(timeit(lambda: ops.gemm_nt(a, b, out)) for _ in range(5))[2]
            tb = sorted(timeit(lambda: torch.matmul(a, b.t(), out=ref)) for _ in range(5))[2]
            ts.append((K // 64, t, tb))
        x = np.array([k for k, _, _ in ts], float)
        y = np.array([t for _, t, _ in ts])
        slope, fixed = np.polyfit(x, y, 1)
        print(json.dumps({"M": M, "N": N, "tiles": (M // 256) * (N // 256), "us": [round(t, 1) for _, t, _ in ts],
                          "hipblaslt_us": [round(t, 1) for _, _, t in ts], "K": KS,
                          "fixed_us": round(fixed, 2), "us_per_ktile": round(slope, 3),
                          "tflops_at_16k": round(2.0 * M * N * KS[-1] / ts[-1][1] / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
