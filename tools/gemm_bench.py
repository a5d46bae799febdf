"""A/B the NT GEMM variants on the SimPO step's exact shapes (M = 2B*T = 4800 rows at 4
pairs, LoRA K-extension of 64) against torch.matmul (hipBLASLt), interleaved rounds in
one process (cdna_hip_programming.md rule 24).  Prints one JSON line per shape."""
import os as _os; _os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ospo_amd", "libospo_hip_ablation.so"))  # A/B knobs: the ablation build
import json
import sys
import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops
from ospo_amd._lib import call

M = int(os.environ.get("GB_M", "4800"))
SHAPES = [  # name, M, N, K, K2
    ("qkv_fwd", M, 12288, 4096, 64), ("o_fwd", M, 4096, 4096, 64), ("gu_fwd", M, 22016, 4096, 64),
    ("down_fwd", M, 4096, 11008, 64), ("down_dx", M, 11008, 4096, 64), ("gu_dx", M, 4096, 22016, 64),
    ("qkv_dx", M, 4096, 12288, 64), ("gh2_fwd", 4608, 16384, 4096, 0), ("gh2_dx", 4608, 4096, 16384, 0),
]
VARIANTS = [int(v) for v in os.environ.get("GB_VARIANTS", "0,1").split(",") if v != ""]
MX8 = os.environ.get("GB_MX8", "0") == "1"  # also time the block-scaled fp8 GEMM (+ its A quantization)
SPLITS = [int(v) for v in os.environ.get("GB_SPLITS", "").split(",") if v != ""]  # forced tail splits (v0)
DROP = os.environ.get("GB_DROP", "0") == "1"
RES = os.environ.get("GB_RES", "0") == "1"
ROPE = os.environ.get("GB_ROPE", "0") == "1"  # also time qkv_fwd with the RoPE epilogue (T = 600, q|k columns)  # bias + residual epilogue on every variant (bit-equality covers it)  # also time the dropout-masked extension form (the dX GEMMs)
ROUNDS, ITERS = 5, 10


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
    for name, m, n, k, k2 in SHAPES:
        a = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
        a2 = (torch.rand(m, k2, device="cuda") * 2 - 1).bfloat16() if k2 else None
        b2 = (torch.rand(n, k2, device="cuda") * 2 - 1).bfloat16() if k2 else None
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        ref = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        ex = {"bias": (torch.rand(n, device="cuda") - 0.5).bfloat16(),
              "residual": (torch.rand(m, n, device="cuda") - 0.5).bfloat16()} if RES else {}
        res = {f"v{v}": [] for v in VARIANTS}
        res["hipblaslt"] = []
        for sp in SPLITS:
            res[f"split{sp}"] = []
        if MX8:
            a8, b8 = ops.MX8.of(a), ops.MX8.of(b)
            res["mx8_quantA"] = []
            for v in VARIANTS:
                res[f"mx8_v{v}"] = []
        for _ in range(ROUNDS):
            if MX8:
                for v in VARIANTS:
                    call("ospo_set_gemm_variant", v)
                    res[f"mx8_v{v}"].append(timeit(lambda: ops.gemm_nt_mx8(a8, b8, out, a2=a2, b2=b2)))
                res["mx8_quantA"].append(timeit(lambda: ops.quant_mx8(a, a8)))
            for v in VARIANTS:
                call("ospo_set_gemm_variant", v)
                res[f"v{v}"].append(timeit(lambda: ops.gemm_nt(a, b, out, a2=a2, b2=b2, **ex)))
            res["hipblaslt"].append(timeit(lambda: torch.matmul(a, b.t(), out=ref)))
            if ROPE and name == "qkv_fwd":
                if "rope_tab" not in locals():
                    rope_tab = ops.rope_tables(600, 128, 1e4, "cuda")
                call("ospo_set_gemm_variant", 0)
                res.setdefault("v0_rope", []).append(timeit(lambda: ops.gemm_nt(a, b, out, a2=a2, b2=b2, rope=(rope_tab[0], rope_tab[1], 600, 8192))))
            if DROP and k2:
                call("ospo_set_gemm_variant", 0)
                res.setdefault("v0_dropout", []).append(timeit(lambda: ops.gemm_nt(a, b, out, a2=a2, b2=b2, dropout=(77, 0.05))))
            for sp in SPLITS:
                res[f"split{sp}"].append(timeit(lambda: ops.gemm_nt(a, b, out, a2=a2, b2=b2, split=sp)))
        exp = a.float() @ b.float().t() + (a2.float() @ b2.float().t() if k2 else 0)
        errs, same = {}, {}
        call("ospo_set_gemm_variant", 0)
        ops.gemm_nt(a, b, ref, a2=a2, b2=b2, **ex)
        for v in VARIANTS:
            call("ospo_set_gemm_variant", v)
            out.zero_()
            ops.gemm_nt(a, b, out, a2=a2, b2=b2, **ex)
            errs[f"v{v}"] = float((out.float() - exp).norm() / exp.norm())
            same[f"v{v}"] = bool(torch.equal(out, ref))
        call("ospo_set_gemm_variant", 0)
        del exp
        fl = 2.0 * m * n * k
        line = {"shape": name, "M": m, "N": n, "K": k, "K2": k2, "tile": ops.gemm_nt_tile(m, n), "relerr": errs, "bit_equal_v0": same}
        for kk, ts in res.items():
            t = sorted(ts)[len(ts) // 2]
            line[kk] = {"ms": round(t, 4), "tflops": round(fl / t / 1e9, 1)}
            if kk == "mx8_quantA":
                line[kk] = {"ms": round(t, 4), "GBps": round(3.0 * m * k / t / 1e6, 1)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
