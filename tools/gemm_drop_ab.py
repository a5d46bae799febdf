"""The dX GEMMs' LoRA-dropout epilogue in isolation (step shapes, 4 pairs): no dropout vs the mask re-hashed
(64 hashes per lane per tile) vs the mask read from the forward's keep bits (staged with tile 0), interleaved
rounds in one process.  One JSON line per shape: median ms per variant and bit-equality of hash vs bits."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

M = 4800
SHAPES = [("down_dx", 11008, 4096), ("gu_dx", 4096, 22016), ("qkv_dx", 4096, 12288), ("o_dx", 4096, 4096)]
ROUNDS, ITERS = 5, 10
DROP = (4321, 0.05)


def timeit(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(ITERS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / ITERS


def main():
    torch.manual_seed(0)
    for name, n, k in SHAPES:
        a = (torch.rand(M, k, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
        a2 = (torch.rand(M, 64, device="cuda") * 2 - 1).bfloat16()
        b2 = (torch.rand(n, 64, device="cuda") * 2 - 1).bfloat16()
        x = torch.randn(M, n, device="cuda").bfloat16()
        bits = torch.zeros(M * n // 8, device="cuda", dtype=torch.uint8)
        ops.lora_skinny(x, torch.zeros(64, n, device="cuda").bfloat16(), torch.empty(M, 64, device="cuda").bfloat16(),
                        M, M, n, 1, 0, 1.0, b_rows=16, dropout=DROP, keep_bits=bits)
        outs = {v: torch.empty(M, n, device="cuda", dtype=torch.bfloat16) for v in ("nodrop", "hash", "bits")}
        fns = {"nodrop": lambda: ops.gemm_nt(a, b, outs["nodrop"], a2=a2, b2=b2),
               "hash": lambda: ops.gemm_nt(a, b, outs["hash"], a2=a2, b2=b2, dropout=DROP),
               "bits": lambda: ops.gemm_nt(a, b, outs["bits"], a2=a2, b2=b2, dropout=DROP, keep_bits=bits)}
        times = {v: [] for v in fns}
        for _ in range(ROUNDS):
            for v, fn in fns.items():
                times[v].append(timeit(fn))
        line = {"shape": name, "M": M, "N": n, "K": k, "bits_equal_hash": bool(torch.equal(outs["hash"], outs["bits"]))}
        for v, ts in times.items():
            line[v] = round(sorted(ts)[len(ts) // 2], 4)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
