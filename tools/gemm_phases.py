"""Where a 256x256 GEMM launch's time goes outside the K loop: s_memrealtime (100 MHz) stamps per workgroup
(ablation build, variant 30): entry, after the prologue, after the K loop, after the accumulators are
staged in LDS, after the epilogue stores are issued, after they complete.  No split-K tail (one launch)."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import sys
import numpy as np
import torch

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops
from ospo_amd._lib import call

SHAPES = [("1round_K4096", 4096, 4096, 4096, 0), ("2round_K4096", 8192, 4096, 4096, 0), ("qkv_fwd", 4800, 12288, 4096, 64),
          ("1round_K1024", 4096, 4096, 1024, 0)]


def main():
    torch.manual_seed(0)
    for name, m, n, k, k2 in SHAPES:
        a = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
        a2 = (torch.rand(m, k2, device="cuda") * 2 - 1).bfloat16() if k2 else None
        b2 = (torch.rand(n, k2, device="cuda") * 2 - 1).bfloat16() if k2 else None
        res = torch.rand(m, n, device="cuda").bfloat16()
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        grid = ((m + 255) // 256) * (n // 256)
        dbg = torch.zeros(grid * 8 * 2, dtype=torch.int32, device="cuda")
        call("ospo_gemm_set_debug_buffer", dbg.data_ptr())
        call("ospo_set_gemm_variant", 30)
        line = {"shape": name, "grid": grid}
        for resid in (False, True):
            for _ in range(10):
                ops.gemm_nt(a, b, out, a2=a2, b2=b2, residual=res if resid else None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            ops.gemm_nt(a, b, out, a2=a2, b2=b2, residual=res if resid else None)
            e1.record()
            torch.cuda.synchronize()
            st = dbg.cpu().numpy().view(np.int64).reshape(grid, 8)[:, :6].astype(np.float64) * 0.01  # us
            t0 = st[:, 0].min()
            st -= t0
            d = {"event_us": round(e0.elapsed_time(e1) * 1e3, 1),
                 "span_us": round(st[:, 5].max(), 1),
                 "entry_p50_max": [round(np.median(st[:, 0]), 2), round(st[:, 0].max(), 2)],
                 "prologue_p50": round(np.median(st[:, 1] - st[:, 0]), 2),
                 "loop_p50": round(np.median(st[:, 2] - st[:, 1]), 2),
                 "acc_to_lds_p50": round(np.median(st[:, 3] - st[:, 2]), 2),
                 "epi_issue_p50": round(np.median(st[:, 4] - st[:, 3]), 2),
                 "store_drain_p50": round(np.median(st[:, 5] - st[:, 4]), 2),
                 "wg_total_p50": round(np.median(st[:, 5] - st[:, 0]), 2),
                 "loop_end_min_max": [round(st[:, 2].min(), 2), round(st[:, 2].max(), 2)]}
            if grid > 256:
                later = st[256:, 0]
                d["round2_entry_min_p50"] = [round(later.min(), 2), round(np.median(later), 2)]
            line["res" if resid else "plain"] = d
        call("ospo_set_gemm_variant", 0)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
