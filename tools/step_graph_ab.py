"""Launch gaps of the eager training step: the bench's config-2 step (30 layers, 4 pairs, r = 16) timed eager
against the same step captured once in a hipGraph and replayed (A/B tool, not a product path: a replay repeats
the captured host scalars -- AdamW step count, dropout seeds -- so its updates are not a valid trajectory).
Prints one JSON line: ms per step eager / replayed, and the difference per kernel launch."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ospo_amd.simpo import SimPOConfig, SimPOLossBuffers, train_step  # noqa: E402


def main():
    dev = torch.device("cuda")
    layers = int(os.environ.get("LAYERS", "30"))
    dims, eng, batches, weights = bench.simpo_setup(layers=layers, device=dev)
    del weights
    torch.cuda.empty_cache()
    cfg, buf = SimPOConfig(), SimPOLossBuffers(4, dev)

    def step(i):
        return train_step(eng, *batches[i % 4], cfg, buf)

    def timed(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    for i in range(3):
        step(i)
    eager = [timed(step, 8) for _ in range(2)]
    print(json.dumps({"eager_ms": eager}), flush=True)
    # capture on a side stream, as torch.cuda.graph does (warm-up done above)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step(0)
    torch.cuda.synchronize()
    rep = [timed(lambda i: g.replay(), 8) for _ in range(2)]
    eager2 = [timed(step, 8) for _ in range(2)]
    e, r = min(eager + eager2), min(rep)
    print(json.dumps({"layers": layers, "eager_ms": [round(x, 2) for x in eager + eager2],
                      "graph_ms": [round(x, 2) for x in rep], "gain_pct": round((e - r) / e * 100, 2)}), flush=True)


if __name__ == "__main__":
    main()
