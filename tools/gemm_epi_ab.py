"""Plain-epilogue store variants of the w4 GEMM (verdict r4 item 3c), same process, interleaved, on the step's
GEMM shapes.  OSPO_GEMM_EPI (ablation build, read per launch): 0 = the product epilogue (4 LDS reads in flight
per batch; round 5: staged inside the last K-tile), 1 = 8 in flight, 2 = non-temporal stores, 3 = both, 4 = 16 in
flight, 9 = the round-4 staging after the K loop (w4_stage_bf16).  Only launches whose
epilogue is plain (no residual, no RoPE) change; every variant must write the same bytes.  Prints one JSON
line per shape: median us per variant and bit-identity."""
import os as _os
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

M = int(os.environ.get("SWEEP_M", "4800"))
MG = M // 600 * 576
SHAPES = [("gu_fwd", M, 22016, 4096, 64), ("down_dx", M, 11008, 4096, 64), ("gu_dx", M, 4096, 22016, 64),
          ("qkv_dx", M, 4096, 12288, 64), ("o_dx", M, 4096, 4096, 64), ("gh2_fwd", MG, 16384, 4096, 0),
          ("sq4096", 4096, 4096, 4096, 0)]
VARS = [int(v) for v in os.environ.get("AB_EPI", "0 9 1 2 3 4").split()]


def main():
    torch.manual_seed(0)
    dev = "cuda"
    for name, m, n, k, k2 in SHAPES:
        ops_ = []
        for rep in range(2):  # two operand sets alternate: no launch re-reads the last one's from the MALL
            a = (torch.rand(m, k, device=dev) * 2 - 1).bfloat16()
            b = (torch.rand(n, k, device=dev) * 2 - 1).bfloat16()
            a2 = (torch.rand(m, k2, device=dev) * 2 - 1).bfloat16() if k2 else None
            b2 = (torch.rand(n, k2, device=dev) * 2 - 1).bfloat16() if k2 else None
            ops_.append((a, b, a2, b2))
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        drop = name.endswith("_dx") and k2
        bits = torch.randint(0, 256, (m * n // 8,), device=dev, dtype=torch.uint8) if drop else None

        def fn(i):
            a, b, a2, b2 = ops_[i & 1]
            if drop:
                ops.gemm_nt(a, b, out, a2=a2, b2=b2, dropout=(5, 0.05), keep_bits=bits)
            else:
                ops.gemm_nt(a, b, out, a2=a2, b2=b2)
        os.environ["OSPO_GEMM_EPI"] = "0"
        fn(0)
        ref = out.clone()
        res = {v: [] for v in VARS}
        same = {v: True for v in VARS}
        for _ in range(5):
            for v in VARS:
                os.environ["OSPO_GEMM_EPI"] = str(v)
                fn(0)
                same[v] &= bool(torch.equal(out, ref))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(10):
                    fn(i)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / 10 * 1e3)
        os.environ["OSPO_GEMM_EPI"] = "0"
        print(json.dumps({"shape": name, "us": {v: round(statistics.median(t), 1) for v, t in res.items()},
                          "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
