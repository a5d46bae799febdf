"""Where a w4 GEMM workgroup's time goes, and the clock the chip holds under it: s_memtime (core clock)
and s_memrealtime (100 MHz) stamps per workgroup (ablation variant 42): entry, program start, program end,
epilogue stores drained.  In-kernel clock = d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md
'DVFS give-back' item 6), after >= 2 s of back-to-back launches on random data.
Round 5 (verdict r4 item 3b): W4_DATA=zero runs the same launches on all-zero operands, so the clock on random
vs zero data separates MFMA data energy from the staging traffic (which is the same for both)."""
import os as _os
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

SHAPES = [("sq4096", 4096, 4096, 4096, 0), ("qkv_fwd", 4800, 12288, 4096, 64), ("down_fwd", 4800, 4096, 11008, 64)]


def main():
    torch.manual_seed(0)
    for name, m, n, k, k2 in SHAPES:
        zero = _os.environ.get("W4_DATA", "random") == "zero"
        fill = (lambda r, c: torch.zeros(r, c, device="cuda", dtype=torch.bfloat16)) if zero else \
            (lambda r, c: (torch.rand(r, c, device="cuda") * 2 - 1).bfloat16())
        a = fill(m, k)
        b = fill(n, k)
        a2 = fill(m, k2) if k2 else None
        b2 = fill(n, k2) if k2 else None
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        grid = ((m + 255) // 256) * (n // 256) * 8  # generous: split-K pieces included
        dbg = torch.zeros(grid * 8, dtype=torch.int64, device="cuda")
        call("ospo_gemm_set_debug_buffer", dbg.data_ptr())
        call("ospo_set_gemm_variant", 42)
        t0 = time.time()
        while time.time() - t0 < 2.0:
            for _ in range(20):
                ops.gemm_nt(a, b, out, a2=a2, b2=b2, split=1)
            torch.cuda.synchronize()
        dbg.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.gemm_nt(a, b, out, a2=a2, b2=b2, split=1)
        e1.record()
        torch.cuda.synchronize()
        call("ospo_set_gemm_variant", 0)
        st = dbg.cpu().numpy().reshape(-1, 8)
        st = st[st[:, 1] != 0].astype(np.float64)
        rt = st[:, [1, 2, 4, 5, 6, 7]] * 0.01  # realtime us: entry, prog start, prog end, staged, issued, drained
        clk = (st[:, 3] - st[:, 0]) / (rt[:, 2] - rt[:, 1]) / 1e3  # GHz over the program
        ntile = (k + k2) // 64
        loop_us = rt[:, 2] - rt[:, 1]
        r0 = rt[:, 0].min()
        med = lambda x: round(float(np.median(x)), 2)  # noqa: E731
        line = {"shape": name, "data": "zero" if zero else "random", "wgs": int(len(st)), "event_us": round(e0.elapsed_time(e1) * 1e3, 1),
                "span_us": round(rt[:, 5].max() - r0, 1),
                "clock_ghz_p10_p50_p90": [round(float(np.percentile(clk, q)), 3) for q in (10, 50, 90)],
                "setup_us_p50": med(rt[:, 1] - rt[:, 0]),
                "program_us_p50": med(loop_us),
                "per_ktile_us_p50": round(float(np.median(loop_us)) / ntile, 4),
                "per_ktile_cycles_p50": round(float(np.median((st[:, 3] - st[:, 0]) / ntile)), 1),
                "stage_us_p50": med(rt[:, 3] - rt[:, 2]), "store_issue_us_p50": med(rt[:, 4] - rt[:, 3]),
                "store_drain_us_p50": med(rt[:, 5] - rt[:, 4]),
                "wg_total_us_p50": med(rt[:, 5] - rt[:, 0]),
                "entry_spread_us": round(float(np.percentile(rt[:, 0] - r0, 90)), 2),
                "prog_end_spread_us_p10_p90": [round(float(np.percentile(rt[:, 2] - r0, q)), 2) for q in (10, 90)]}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
