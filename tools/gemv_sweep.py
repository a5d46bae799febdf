"""Sweep the decode GEMV's schedule (v2: 64 rows / v3: 128 rows per workgroup) x K-split count on
the 7B decode shapes (R = 32), one process, interleaved rounds.  Prints the best per shape."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))  # A/B knobs: the ablation build
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

R = 32
SHAPES = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gu", 22016, 4096), ("down", 4096, 11008), ("gh2", 16384, 4096)]
SPLITS = [0, 1, 2, 3, 4, 6, 8, 11, 16]


def timeit(fn, it=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


torch.manual_seed(0)
for name, N, K in SHAPES:
    x = torch.randn(R, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    out = torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
    ws = ops.decode_gemv_ws(R, N, K, "cuda")
    ws = torch.zeros(max(ws.numel(), 16 * (N // 16) * 2 * 64 * 4 + 64), device="cuda")
    res = {}
    for _ in range(3):
        for v in (2, 3):
            for sp in SPLITS:
                call("ospo_set_gemv_variant", v)
                call("ospo_set_gemv_splits", sp)
                res.setdefault((v, sp), []).append(timeit(lambda: ops.decode_gemv(x, w, out, ws=ws)))
    call("ospo_set_gemv_variant", 2)
    call("ospo_set_gemv_splits", 0)
    med = {k: sorted(t)[1] for k, t in res.items()}
    best = min(med, key=med.get)
    print(json.dumps({"shape": name, "N": N, "K": K, "best": {"variant": best[0], "splits": best[1], "us": round(med[best], 1)},
                      "auto_v2_us": round(med[(2, 0)], 1), "auto_v3_us": round(med[(3, 0)], 1),
                      "all": {f"v{v}s{sp}": round(t, 1) for (v, sp), t in sorted(med.items())}}), flush=True)
