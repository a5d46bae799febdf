"""A/B of the decode GEMV schedules (ospo_set_gemv_variant 1 / 2 / 3, GV_VARIANTS) on the 7B decode shapes, R = 32
rows, interleaved rounds in one process.  Prints GB/s of weight streaming per shape."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))  # A/B knobs: the ablation build
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

R = int(os.environ.get("GV_R", "32"))
VARIANTS = [int(v) for v in os.environ.get("GV_VARIANTS", "2,3").split(",")]
SHAPES = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gu", 22016, 4096), ("down", 4096, 11008), ("gh1", 4096, 4096),
          ("gh2", 16384, 4096)]


def timeit(fn, it=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


torch.manual_seed(0)
for name, N, K in SHAPES:
    x = torch.randn(R, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    out = torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
    ws = ops.decode_gemv_ws(R, N, K, "cuda")
    res = {v: [] for v in VARIANTS}
    outs = {}
    for _ in range(5):
        for v in VARIANTS:
            call("ospo_set_gemv_variant", v)
            res[v].append(timeit(lambda: ops.decode_gemv(x, w, out, ws=ws)))
    for v in VARIANTS:
        call("ospo_set_gemv_variant", v)
        ops.decode_gemv(x, w, out, ws=ws)
        outs[v] = out.clone()
    call("ospo_set_gemv_variant", 3)
    ref = x.float() @ w.float().T
    line = {"shape": name, "N": N, "K": K, "R": R}
    for v in VARIANTS:
        t = sorted(res[v])[2]
        line[f"v{v}"] = {"us": round(t * 1e3, 1), "GBps": round(N * K * 2 / t / 1e6, 1),
                         "relerr": float((outs[v].float() - ref).norm() / ref.norm())}
    print(json.dumps(line), flush=True)
