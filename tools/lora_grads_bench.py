"""A/B the LoRA weight-gradient products (dA = g^T x, dB = dy^T u) on one layer's
shapes (Janus-Pro-7B, 4 pairs, T = 600): legacy (Rp rows, 9/4 splits, big tiles) vs
current (used rows, 8 splits, grid-aware tiles).  Run twice: with and without
OSPO_F32ACC_LEGACY=1 (the C tile rule is read once per process)."""
import json
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops

Mk, D, F, r, Rp = 4800, 4096, 11008, 16, 64
GROUPS = [("qkv", 3, D, D), ("o", 1, D, D), ("gu", 2, D, F), ("down", 1, F, D)]  # name, nmods, Kin, Nmod
legacy = os.environ.get("OSPO_F32ACC_LEGACY") is not None
STREAM = int(os.environ.get("OSPO_WGRAD_WGS", "0"))  # > 0: ospo_lora_wgrad with ~this many workgroups per product


def main():
    torch.manual_seed(0)
    tot = 0.0
    for name, nm, kin, nmod in GROUPS:
        g = (torch.randn(Mk, Rp, device="cuda") * 0.1).bfloat16()
        x = torch.randn(Mk, kin, device="cuda").bfloat16()
        dy = torch.randn(Mk, nm * nmod, device="cuda").bfloat16()
        u = (torch.randn(Mk, Rp, device="cuda") * 0.1).bfloat16()
        used = nm * r
        dA = torch.zeros(Rp if legacy else used, kin, device="cuda")
        dB = torch.zeros(nm * nmod, r, device="cuda")

        def splits(n):
            return max(1, min(Mk // 64 // 4, round(STREAM / max(1, n // 256))))

        def run():
            if STREAM:
                ops.lora_wgrad(x, g, dA, mode=0, s_cols=used, splits=splits(kin))
                ops.lora_wgrad(dy, u, dB, mode=1, s_cols=used, splits=splits(nm * nmod), nmod=nmod, r=r)
            elif legacy:
                ops.gemm_f32acc(g, x, dA, a_kmajor=True, b_kmajor=True, k_splits=min(Mk // 512, 16))
                ops.gemm_f32acc(dy, u, dB, a_kmajor=True, b_kmajor=True, k_splits=min(Mk // 1024, 8), diag=(nmod, r))
            else:
                ops.gemm_f32acc(g[:, :used], x, dA, a_kmajor=True, b_kmajor=True, k_splits=8)
                ops.gemm_f32acc(dy, u, dB, a_kmajor=True, b_kmajor=True, k_splits=8, diag=(nmod, r))
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        tot += us
        gb = Mk * (kin + nm * nmod) * 2 / 1e9
        print(json.dumps({"group": name, "legacy": legacy, "stream_wgs": STREAM, "dA+dB_us": round(us, 1),
                          "GBps": round(gb / us * 1e6, 1)}), flush=True)
    print(json.dumps({"legacy": legacy, "stream_wgs": STREAM, "per_layer_us": round(tot, 1)}), flush=True)


if __name__ == "__main__":
    main()
