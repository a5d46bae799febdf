"""Where the SP8 GEMM's K-tile time goes: s_memtime stamps of one steady K-tile (local tile 8) in every
wave (ablation build, variant 29).  Per wave and per phase p: k0 R start, k1 after the barrier (M start),
k2 after lgkmcnt(0), k3 after the MFMA cluster issue, k4 after g0's vmcnt waits (before the barrier)."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import sys
import torch
import numpy as np

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops
from ospo_amd._lib import call

SHAPES = [("qkv_fwd", 4800, 12288, 4096, 64), ("gu_dx", 4800, 4096, 22016, 64), ("o_fwd", 4800, 4096, 4096, 64)]


def main():
    torch.manual_seed(0)
    for name, m, n, k, k2 in SHAPES:
        a = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
        a2 = (torch.rand(m, k2, device="cuda") * 2 - 1).bfloat16()
        b2 = (torch.rand(n, k2, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        grid = ((m + 255) // 256) * (n // 256)
        dbg = torch.zeros(grid * 8 * 16, dtype=torch.int32, device="cuda")
        call("ospo_gemm_set_debug_buffer", dbg.data_ptr())
        call("ospo_set_gemm_variant", 29)
        for _ in range(20):
            ops.gemm_nt(a, b, out, a2=a2, b2=b2)
        torch.cuda.synchronize()
        call("ospo_set_gemm_variant", 0)
        st = dbg.cpu().numpy().view(np.uint32).astype(np.int64).reshape(grid, 8, 16)[:, :, :10].reshape(grid, 8, 2, 5)
        res = {"shape": name}
        for gname, ws in (("g0", slice(0, 4)), ("g1", slice(4, 8))):
            s = st[:, ws]  # [grid, 4, 2, 5]
            d = {}
            for p in range(2):
                d[f"p{p}_R+bar"] = float(np.median(s[:, :, p, 1] - s[:, :, p, 0]))
                d[f"p{p}_lgkm"] = float(np.median(s[:, :, p, 2] - s[:, :, p, 1]))
                d[f"p{p}_mfma"] = float(np.median(s[:, :, p, 3] - s[:, :, p, 2]))
                d[f"p{p}_vmw"] = float(np.median(s[:, :, p, 4] - s[:, :, p, 3]))
            d["bar_after_M0"] = float(np.median(s[:, :, 1, 0] - s[:, :, 0, 4]))
            d["tile_span_k0p0_to_k4p1"] = float(np.median(s[:, :, 1, 4] - s[:, :, 0, 0]))
            res[gname] = d
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
