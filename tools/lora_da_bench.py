"""dA of the four LoRA groups of one layer (Janus-Pro-7B, 4 pairs, T = 600: Mk = 4800 tokens, r = 16,
dropout 0.05) in isolation: the f32-atomic 64 x 64 tile product the engine ran through round 2
(ospo_gemm_f32acc_bdrop, 8 / 4 K splits) against the one-stream ospo_lora_da at several split counts,
interleaved rounds in one process.  One JSON line per (group, variant) with the median time and the rate
on the x stream (the algorithmic bytes: Mk x Kin bf16); a final line per variant with the layer sum."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

Mk, D, F, r, Rp = 4800, 4096, 11008, 16, 64
GROUPS = [("qkv", 3, D), ("o", 1, D), ("gu", 2, D), ("down", 1, F)]  # name, modules, Kin
SPLITS = [int(v) for v in os.environ.get("DA_SPLITS", "0,4,8,16").split(",")]
DROP = (1234, 0.05) if os.environ.get("DA_DROP", "1") == "1" else None
ROUNDS, ITERS = 5, 20


def timeit(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(ITERS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / ITERS * 1e3


def main():
    torch.manual_seed(0)
    tot = {}
    for name, nm, kin in GROUPS:
        used = nm * r
        g = (torch.randn(Mk, Rp, device="cuda") * 0.1).bfloat16()
        g[:, used:] = 0
        x = torch.randn(Mk, kin, device="cuda").bfloat16()
        out = torch.zeros(used, kin, device="cuda")
        variants = {"tiles": lambda: ops.gemm_f32acc(g[:, :used], x, out, a_kmajor=True, b_kmajor=True,
                                                      k_splits=4 if kin > 8192 else 8, b_dropout=DROP)}
        for sp in SPLITS:
            variants[f"stream_s{sp}"] = (lambda sp=sp: ops.lora_da(x, g, out, s_cols=used, splits=sp, dropout=DROP))
        if DROP:  # the mask from the forward's keep bits instead of re-hashed
            bits = torch.zeros(Mk * kin // 8, device="cuda", dtype=torch.uint8)
            ops.lora_skinny(x, torch.zeros(64, kin, device="cuda").bfloat16(), torch.empty(Mk, 64, device="cuda").bfloat16(),
                            Mk, Mk, kin, 1, 0, 1.0, b_rows=16, dropout=DROP, keep_bits=bits)
            for sp in SPLITS:
                variants[f"bits_s{sp}"] = (lambda sp=sp, bits=bits: ops.lora_da(x, g, out, s_cols=used, splits=sp,
                                                                                 dropout=DROP, keep_bits=bits))
        times = {k: [] for k in variants}
        for _ in range(ROUNDS):
            for k, fn in variants.items():
                times[k].append(timeit(fn))
        # agreement of the two products (fp32 atomics: reassociation only)
        a = torch.zeros_like(out)
        b = torch.zeros_like(out)
        ops.gemm_f32acc(g[:, :used], x, a, a_kmajor=True, b_kmajor=True, k_splits=1, b_dropout=DROP)
        ops.lora_da(x, g, b, s_cols=used, splits=1, dropout=DROP)
        torch.cuda.synchronize()
        same = bool(torch.equal(a, b))
        for k, ts in times.items():
            us = sorted(ts)[len(ts) // 2]
            tot[k] = tot.get(k, 0.0) + us
            print(json.dumps({"group": name, "variant": k, "us": round(us, 2),
                              "GBps_x": round(Mk * kin * 2 / us / 1e3, 1), "bit_equal_1split": same}), flush=True)
    for k, us in tot.items():
        print(json.dumps({"variant": k, "per_layer_us": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
