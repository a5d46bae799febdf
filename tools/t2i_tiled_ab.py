"""A/B of the decode weight layouts (row-major vs the MFMA-tiled layout of ops.tile_decode_weight).

1. Per GEMV shape of the 7B decode step (R = 32): median of interleaved rounds, weight GB/s.
2. The whole decode step (hipGraph of one step at mid-image, 7B, 16 prompts x (cond, uncond)):
   one graph per layout, replays interleaved, per-step time and weight+KV GB/s.
Prints JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

R = 32
SHAPES = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gu", 22016, 4096), ("down", 4096, 11008), ("gh2", 16384, 4096)]


def timeit(fn, it=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def shapes():
    torch.manual_seed(0)
    for name, N, K in SHAPES:
        x = torch.randn(R, K, device="cuda").bfloat16()
        # two copies of each layout so back-to-back launches do not re-read one weight from the 256 MB MALL
        ws_ = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(2)]
        wt_ = [ops.tile_decode_weight(w) for w in ws_]
        out = torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
        gws = ops.decode_gemv_ws(R, N, K, "cuda")
        res = {"row": [], "tiled": []}
        for _ in range(5):
            for k, ww in (("row", ws_), ("tiled", wt_)):
                def f(ww=ww):
                    ops.decode_gemv(x, ww[0], out, ws=gws)
                    ops.decode_gemv(x, ww[1], out, ws=gws)
                res[k].append(timeit(f) / 2)
        line = {"shape": name, "N": N, "K": K, "R": R}
        for k in res:
            t = sorted(res[k])[2]
            line[k] = {"us": round(t * 1e3, 2), "GBps": round(N * K * 2 / t / 1e6, 1)}
        print(json.dumps(line), flush=True)
        del ws_, wt_


def step():
    from ospo_amd.engine import JANUS_PRO_7B, synthetic_weights
    from ospo_amd.generate import T2IGenerator
    dev = torch.device("cuda", 0)
    dims = JANUS_PRO_7B
    B, N, Lp = 16, 576, 48
    w = synthetic_weights(dims, dev, seed=0, lora_seed=1)
    gen = T2IGenerator(dims, w, device=dev, max_batch=B, max_prompt_len=Lp, n_img_tokens=N)
    del w
    torch.cuda.empty_cache()
    tiled = [{k: lw[k + "_d"] for k in ("qkv", "o", "gu", "down")} for lw in gen.layers]
    heads = (gen.gh_w1_d, gen.gh_w2_d, gen.al_w2_d)

    def set_layout(t):
        for lw, tl in zip(gen.layers, tiled):
            for k in ("qkv", "o", "gu", "down"):
                lw[k + "_d"] = tl[k] if t else lw[k]
        gen.gh_w1_d, gen.gh_w2_d, gen.al_w2_d = heads if t else (gen.gh_w1, gen.gh_w2, gen.al_w2)

    graphs = {}
    s = torch.cuda.Stream()
    for name, t in (("row", False), ("tiled", True)):
        set_layout(t)
        gen.pos.fill_(Lp + N // 2)
        gen.step.fill_(N)  # the sampler writes no token past the image (step >= n)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            gen._decode_step(2 * B)  # warm-up outside capture
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            gen._decode_step(2 * B)
        graphs[name] = gr
    res = {"row": [], "tiled": []}
    for _ in range(5):
        for name, gr in graphs.items():
            gen.pos.fill_(Lp + N // 2)
            gen.step.fill_(N)
            torch.cuda.synchronize()
            res[name].append(timeit(gr.replay, it=20))
    wbytes = sum(lw[k].numel() * 2 for lw in gen.layers for k in ("qkv", "o", "gu", "down"))
    wbytes += (gen.gh_w1.numel() + gen.gh_w2.numel() + gen.al_w2.numel()) * 2
    kv = dims.n_layers * 2 * 2 * B * dims.n_heads * (Lp + N // 2 + 10) * 128 * 2
    line = {"workload": "7B decode step, 32 rows, pos ~ Lp + 298", "weight_bytes": wbytes, "kv_bytes": kv}
    for name in res:
        t = sorted(res[name])[2]
        line[name] = {"us": round(t * 1e3, 1), "GBps": round((wbytes + kv) / t / 1e6, 1)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "shapes"):
        shapes()
    if which in ("all", "step"):
        step()
