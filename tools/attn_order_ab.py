"""Workgroup order of the attention backward kernels (verdict r4 item 2a), same process, interleaved.

OSPO_ATTN_ORDER (ablation build, read per call) selects group_major's mode for the dK/dV and dQ kernels,
OSPO_ATTN_ORDER_DQ the dQ kernel's alone: 0 block-major (heaviest first chip-wide, the default), 1 group-major,
g >= 2 banded (each XCD walks bands of g groups, heaviest first within a band).  The step's shape: S = 8
sequences, T = 600, 32 heads, RoPE fused; two input sets alternate so no launch re-reads the previous one's
operands from the Infinity Cache.  Every order must give bit-identical dq|dk|dv (the order moves no
arithmetic).  Prints one JSON line per (dkdv order, dq order): median us of the whole 5-product backward."""
import os as _os
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

S, T, H, hd = int(os.environ.get("AB_S", "8")), 600, 32, 128
ORDERS = [tuple(int(x) for x in c.split(",")) for c in
          os.environ.get("AB_ORDERS", "0,0 1,1 2,0 4,0 8,0 4,4 2,2").split()]


def main():
    D = H * hd
    rows = S * T
    sets = []
    for k in range(2):
        g = torch.Generator(device="cuda").manual_seed(k)
        qkv = torch.randn(rows, 3 * D, device="cuda", generator=g).bfloat16()
        do = torch.randn(rows, D, device="cuda", generator=g).bfloat16()
        o = torch.empty(rows, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(S * H * T, device="cuda")
        sets.append((qkv, do, o, lse))
    cos, sin = ops.rope_tables(T, hd, 1e4, "cuda")
    sc = 1 / math.sqrt(hd)
    delta = torch.empty(S * H * T, device="cuda")
    ws = ops.flash_attn_bwd_ws(S, T, H, "cuda")
    dqkv = torch.empty(rows, 3 * D, device="cuda", dtype=torch.bfloat16)
    for qkv, do, o, lse in sets:
        ops.flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, sc)

    def bwd(k):
        qkv, do, o, lse = sets[k]
        ops.flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, ws, dqkv, S, T, H, hd, sc, rope_cos=cos, rope_sin=sin)

    def set_order(od, oq):
        os.environ["OSPO_ATTN_ORDER"] = str(od)
        os.environ["OSPO_ATTN_ORDER_DQ"] = str(oq)

    ref = []
    set_order(0, 0)
    for k in range(2):
        bwd(k)
        ref.append(dqkv.clone())
    times = {c: [] for c in ORDERS}
    same = {c: True for c in ORDERS}
    for rnd in range(6):
        for c in ORDERS:
            set_order(*c)
            for k in range(2):
                bwd(k)
                same[c] &= bool(torch.equal(dqkv, ref[k]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for it in range(10):
                bwd(it & 1)
            e1.record()
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / 10 * 1e3)
    for c in ORDERS:
        print(json.dumps({"order_dkdv": c[0], "order_dq": c[1], "bwd5_us_median": round(statistics.median(times[c]), 1),
                          "bwd5_us": [round(t, 1) for t in times[c]], "bit_identical": same[c]}), flush=True)

    # the forward (attn_fwd2_kernel): OSPO_ATTN_ORDER_FWD 0 = (head, sequence, block) grid, g >= 2 banded
    def fwd(k):
        qkv, do, o, lse = sets[k]
        ops.flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, sc)

    os.environ["OSPO_ATTN_ORDER_FWD"] = "0"
    fref = []
    for k in range(2):
        fwd(k)
        fref.append((sets[k][2].clone(), sets[k][3].clone()))
    forders = [int(x) for x in os.environ.get("AB_FWD_ORDERS", "0 2 4 8 16").split()]
    ft = {c: [] for c in forders}
    fsame = {c: True for c in forders}
    for rnd in range(6):
        for c in forders:
            os.environ["OSPO_ATTN_ORDER_FWD"] = str(c)
            for k in range(2):
                fwd(k)
                fsame[c] &= bool(torch.equal(sets[k][2], fref[k][0]) and torch.equal(sets[k][3], fref[k][1]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for it in range(10):
                fwd(it & 1)
            e1.record()
            torch.cuda.synchronize()
            ft[c].append(e0.elapsed_time(e1) / 10 * 1e3)
    for c in forders:
        print(json.dumps({"order_fwd": c, "fwd_us_median": round(statistics.median(ft[c]), 1),
                          "fwd_us": [round(t, 1) for t in ft[c]], "bit_identical": fsame[c]}), flush=True)

    # round 5: the O rescale skipped where no row's running max moved (default) vs every tile (OSPO_ATTN_FWD2_DBG=5)
    os.environ["OSPO_ATTN_ORDER_FWD"] = "0"
    rt = {"skip": [], "always": []}
    rsame = True
    for rnd in range(6):
        for v in ("skip", "always"):
            if v == "always":
                os.environ["OSPO_ATTN_FWD2_DBG"] = "5"
            else:
                os.environ.pop("OSPO_ATTN_FWD2_DBG", None)
            for k in range(2):
                fwd(k)
                rsame &= bool(torch.equal(sets[k][2], fref[k][0]) and torch.equal(sets[k][3], fref[k][1]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for it in range(10):
                fwd(it & 1)
            e1.record()
            torch.cuda.synchronize()
            rt[v].append(e0.elapsed_time(e1) / 10 * 1e3)
    os.environ.pop("OSPO_ATTN_FWD2_DBG", None)
    print(json.dumps({"fwd_rescale": {v: round(statistics.median(t), 1) for v, t in rt.items()},
                      "bit_identical": rsame}), flush=True)


if __name__ == "__main__":
    main()
