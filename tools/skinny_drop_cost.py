"""What the dropout costs the forward's u products at the step shape (M 4800, K 4096; round 6):
ospo_lora_skinny with dropout + keep-bit output (the engine's call), with dropout and no bits, and without dropout,
for the 3 / 2 / 1-tile products (q|k|v, gate|up, o), medians of 3 x 20 launches (HIP events), inputs alternated
between two copies so nothing is re-read from the Infinity Cache.  Product library."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

M, K = 4800, 4096


def timeit(f, it=20):
    for i in range(4):
        f(i & 1)
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(it):
            f(i & 1)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / it * 1e3)
    return sorted(ts)[1]


def main():
    torch.manual_seed(0)
    xs = [torch.randn(M, K, device="cuda").bfloat16() for _ in range(2)]
    bits = torch.empty(M * K // 8, dtype=torch.uint8, device="cuda")
    out = {}
    for nt in (3, 2, 1):
        bt = (torch.randn(16 * nt, K, device="cuda") * 0.05).bfloat16()
        ws = ops.lora_skinny_ws(M, K, nt)
        o = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
        res = {}
        for tag, dr, kb in (("drop_bits", (12345, 0.05), bits), ("drop", (12345, 0.05), None), ("plain", None, None)):
            f = lambda i: ops.lora_skinny(xs[i], bt, o, M, M, K, nt, 0, 2.0, b_rows=16 * nt, ws=ws,  # noqa: E731
                                          dropout=dr, keep_bits=kb)
            res[tag] = round(timeit(f), 1)
        res["GBps_plain"] = round(M * K * 2 / res["plain"] / 1e3, 0)
        out[f"nt{nt}"] = res
    # a pure stream of the same bytes for scale: x.sum() over bf16 (torch)
    ts = timeit(lambda i: xs[i].sum())
    out["torch_sum_39MB_us"] = round(ts, 1)
    print(json.dumps({"skinny_u_dropout_cost_us": out}), flush=True)


if __name__ == "__main__":
    main()
