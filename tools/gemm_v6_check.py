"""Persistent GEMM (v6, ablation variant 32, rejected) against the one-unit-per-workgroup SP8 kernel (v5, the
default schedule) on the SimPO step's shapes: bit-equality for every epilogue (plain, bias + residual, RoPE,
dropout-masked extension, pinned split-K tails) and interleaved timings.  Ablation build only.
One JSON line per case; exits 1 if any case differs."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

M = int(os.environ.get("GB_M", "4800"))
QUICK = os.environ.get("GB_QUICK", "0") == "1"
CASES = [  # name, M, N, K, K2, epilogue
    ("qkv_fwd_rope", M, 12288, 4096, 64, "rope"), ("o_fwd_res", M, 4096, 4096, 64, "res"),
    ("gu_fwd", M, 22016, 4096, 64, "plain"), ("down_fwd_res", M, 4096, 11008, 64, "res"),
    ("down_dx_drop", M, 11008, 4096, 64, "drop"), ("gu_dx_drop", M, 4096, 22016, 64, "drop"),
    ("qkv_dx_drop", M, 4096, 12288, 64, "drop"), ("gh2_fwd", 4608, 16384, 4096, 0, "plain"),
    ("gh2_dx", 4608, 4096, 16384, 0, "plain"), ("o_fwd_bias", M, 4096, 4096, 64, "bias"),
    ("split_tail", 1280, 3840, 4096, 64, "split4"), ("split_tail_drop", 1280, 3840, 4096, 64, "drop_split2"),
    ("ragged_m", 1000, 1024, 512, 64, "res"), ("tiny_k", 520, 768, 128, 0, "rope"),
]
ROUNDS, ITERS = (1, 2) if QUICK else (5, 10)


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
    bad = 0
    rope_tab = ops.rope_tables(600, 128, 1e4, "cuda")
    for name, m, n, k, k2, epi in CASES:
        a = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
        a2 = (torch.rand(m, k2, device="cuda") * 2 - 1).bfloat16() if k2 else None
        b2 = (torch.rand(n, k2, device="cuda") * 2 - 1).bfloat16() if k2 else None
        ex = {}
        if epi in ("res", "bias"):
            ex["bias"] = (torch.rand(n, device="cuda") - 0.5).bfloat16()
            if epi == "res":
                ex["residual"] = (torch.rand(m, n, device="cuda") - 0.5).bfloat16()
            ex["alpha"] = 0.75
        elif epi == "rope":
            ex["rope"] = (rope_tab[0], rope_tab[1], 600, (2 * n // 3) // 128 * 128)  # the q | k columns
        elif epi.startswith("drop"):
            ex["dropout"] = (77, 0.05)
        if "split" in epi:
            ex["split"] = int(epi[-1])
        outs, times = {}, {}
        for v in (0, 32):
            call("ospo_set_gemm_variant", v)
            o = torch.full((m, n), float("nan"), device="cuda", dtype=torch.bfloat16)
            ops.gemm_nt(a, b, o, a2=a2, b2=b2, **ex)
            torch.cuda.synchronize()
            outs[v] = o
        for _ in range(ROUNDS):
            for v in (0, 32):
                call("ospo_set_gemm_variant", v)
                o = outs[v]
                times.setdefault(v, []).append(timeit(lambda: ops.gemm_nt(a, b, o, a2=a2, b2=b2, **ex)))
        call("ospo_set_gemm_variant", 0)
        same = bool(torch.equal(outs[32], outs[0]))
        finite = bool(torch.isfinite(outs[32].float()).all())
        bad += (not same) or (not finite)
        fl = 2.0 * m * n * k
        line = {"case": name, "M": m, "N": n, "K": k, "K2": k2, "epi": epi, "bit_equal_v5": same, "finite": finite}
        if not same:
            d = (outs[32].float() - outs[0].float()).abs()
            idx = torch.nonzero(d > 0)
            line["n_diff"] = int(idx.shape[0])
            line["first_diff"] = idx[:4].tolist()
        for v, lab in ((0, "v5"), (32, "v6")):
            t = sorted(times[v])[len(times[v]) // 2]
            line[lab] = {"ms": round(t, 4), "tflops": round(fl / t / 1e9, 1)}
        print(json.dumps(line), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
