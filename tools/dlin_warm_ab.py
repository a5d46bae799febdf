"""Decode Linear (ospo_decode_linear, R = 32 rows, the T2I step's shapes) with its weight cold in HBM vs warm in the
256 MB Infinity Cache (MALL): does a weight prefetch ahead of its launch pay?  Cold = every launch reads another
copy of the weight (copies summing to > 1 GB, so no launch finds its weight in the MALL); warm = the same copy
launched back to back.  Prints one JSON line per shape: us per launch, TB/s on the weight bytes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

R = 32
SHAPES = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008)]


def main():
    torch.manual_seed(0)
    dev = "cuda"
    x = (torch.randn(R, 11008, device=dev) * 0.5).bfloat16()
    for name, N, K in SHAPES:
        wbytes = N * K * 2
        ncopy = max(2, -(-(1 << 30) // wbytes))
        ws_ = [ops.tile_decode_weight((torch.rand(N, K, device=dev) * 0.02 - 0.01).bfloat16()) for _ in range(ncopy)]
        out = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
        ws = ops.decode_linear_ws(R, N, K, dev)
        xk = x[:, :K].contiguous()

        def run(i):
            ops.decode_linear(xk, ws_[i % ncopy], out, ws)

        def timed(seq):
            for i in seq[:4]:
                run(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in seq:
                run(i)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / len(seq) * 1e3

        res = {}
        for rep in range(3):
            res.setdefault("cold", []).append(timed(list(range(4 * ncopy))))
            res.setdefault("warm", []).append(timed([0] * (4 * ncopy)))
        cold, warm = min(res["cold"]), min(res["warm"])
        print(json.dumps({"shape": name, "N": N, "K": K, "weight_MB": round(wbytes / 1e6, 1), "copies": ncopy,
                          "cold_us": round(cold, 2), "warm_us": round(warm, 2),
                          "cold_TBps": round(wbytes / cold / 1e6, 2), "warm_TBps": round(wbytes / warm / 1e6, 2)}),
              flush=True)
        del ws_


if __name__ == "__main__":
    main()
