"""Split-count sweep of the decode GEMV on MFMA-tiled weights (ablation build: ospo_set_gemv_splits),
R = 32, the 7B decode shapes; two weight copies alternate so no launch re-reads a weight from the MALL.
Prints one JSON line per shape: us per split count (0 = the product heuristic)."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402
from tools.t2i_tiled_ab import SHAPES, timeit  # noqa: E402

R = 32
for name, N, K in SHAPES + [("gh1", 4096, 4096)]:
    x = torch.randn(R, K, device="cuda").bfloat16()
    wt = [ops.tile_decode_weight((torch.randn(N, K, device="cuda") * 0.02).bfloat16()) for _ in range(2)]
    out = torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(max(ops.decode_gemv_ws(R, N, K, "cuda").numel(), 16 * R * N * 4 // 4 + 16), device="cuda")
    res = {}
    for _ in range(3):
        for s in (0, 1, 2, 4, 8, 16):
            if s > 0 and s > K // 512:
                continue
            call("ospo_set_gemv_splits", s)

            def f():
                ops.decode_gemv(x, wt[0], out, ws=ws)
                ops.decode_gemv(x, wt[1], out, ws=ws)
            res.setdefault(s, []).append(timeit(f) / 2 * 1e3)
    call("ospo_set_gemv_splits", 0)
    print(json.dumps({"shape": name, "N": N, "K": K, "us": {str(k): round(sorted(v)[1], 2) for k, v in res.items()}}),
          flush=True)
