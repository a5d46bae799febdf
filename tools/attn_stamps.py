"""Phase stamps of the pipelined dK/dV kernel at the step shape (ablation build): per-tile cycles of
the first LDS wait, the S/dP + softmax sub-phases, the dV/dK sub-phases, the vmcnt drain and the
barrier, averaged over waves (s_memtime counts at the constant 100 MHz x ... reference: see output)."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import ctypes
import json
import math
import sys
import torch

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops, _lib

S, T, H, hd = 8, 600, 32, 128


def main():
    D = H * hd
    rows = S * T
    qkv = torch.randn(rows, 3 * D, device="cuda").bfloat16()
    o = torch.empty(rows, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(S * H * T, device="cuda")
    delta = torch.empty(S * H * T, device="cuda")
    do = torch.randn(rows, D, device="cuda").bfloat16()
    dqkv = torch.empty(rows, 3 * D, device="cuda", dtype=torch.bfloat16)
    cos, sin = ops.rope_tables(T, hd, 1e4, "cuda")
    sc = 1 / math.sqrt(hd)
    ws = ops.flash_attn_bwd_ws(S, T, H, "cuda")
    ops.flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, sc)
    nkb = (T + 63) // 64
    buf2 = torch.zeros(2 * nkb * S * H * 4 * 8, dtype=torch.int64, device="cuda")
    buf = buf2[: nkb * S * H * 4 * 8]
    lib = _lib.lib()
    lib.ospo_attn_set_stamps(ctypes.c_void_p(buf2.data_ptr()))
    for _ in range(3):
        ops.flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, ws, dqkv, S, T, H, hd, sc, rope_cos=cos, rope_sin=sin)
    torch.cuda.synchronize()
    lib.ospo_attn_set_stamps(ctypes.c_void_p(0))
    st = buf.view(nkb, S * H * 4, 8).double()
    tiles = ((buf.view(nkb, S * H * 4, 8)[..., 7] >> 20) & 0xFF).double()
    rt = ((buf.view(-1, 8)[:, 7] >> 32) & 0xFFFFFFFF) - (buf.view(-1, 8)[:, 6] & 0xFFFFFFFF)
    tot = (buf.view(-1, 8)[:, 5] & 0xFFFFFFFF).double()
    pro = (buf.view(-1, 8)[:, 5] >> 32).double()
    loop = buf.view(-1, 8)[:, :5].double().sum(1)
    out = {}
    names = ["first_wait", "sdp_softmax", "dvdk", "vmcnt", "barrier"]
    for i, nm in enumerate(names):
        out[nm + "_per_tile"] = round(float(st[..., i].sum() / tiles.sum()), 1)
    out["stage_issue_per_tile"] = round(float(buf2[nkb * S * H * 4 * 8:].view(-1, 8)[:, 6].double().sum() / tiles.sum()), 1)
    out["memtime_ticks_per_us"] = round(float(tot.sum() / (rt.double().sum() / 100.0)), 1)
    out["loop_share_of_wg"] = round(float(loop.sum() / tot.sum()), 3)
    out["prologue_share_of_wg"] = round(float(pro.sum() / tot.sum()), 3)
    out["prologue_us_mean"] = round(float(pro.mean()) / 2046.5, 2)
    out["per_kb_total_per_tile"] = [round(float(st[k, :, :5].sum() / tiles[k].sum()), 1) for k in range(nkb)]
    print(json.dumps(out))
    print(json.dumps(occupancy(buf, nkb)))




def occupancy(buf, nkb):
    """WG residency per CU from the start / end realtime stamps (100 MHz) and HW_ID / XCC_ID."""
    import collections
    st = buf.view(-1, 8).cpu()
    wave0 = st[::4]
    start = wave0[:, 6] & 0xFFFFFFFF
    end = (wave0[:, 7] >> 32) & 0xFFFFFFFF
    hw = wave0[:, 7] & 0xFFFF
    xcc = (wave0[:, 7] >> 16) & 0xF
    cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 3) << 5) | (xcc << 7)
    t0 = int(start.min())
    per_cu = collections.defaultdict(list)
    for i in range(len(start)):
        per_cu[int(cu[i])].append((int(start[i]) - t0, int(end[i]) - t0))
    # max concurrent WGs on a CU, and the CU-busy fraction
    maxc, total = 0, int(end.max()) - t0
    for iv in per_cu.values():
        ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv])
        c = 0
        for _, d in ev:
            c += d
            maxc = max(maxc, c)
    dur = (end - start).double()
    return {"cus_seen": len(per_cu), "max_wg_per_cu": maxc, "span_us": total / 100.0,
            "wg_us_mean": round(float(dur.mean()) / 100.0, 2), "wg_us_max": round(float(dur.max()) / 100.0, 2)}


if __name__ == "__main__":
    main()
