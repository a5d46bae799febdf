"""The MXFP8 w4 GEMM (gemm_nt_w4_kernel<.., MX = true>, ablation variant 52; the library keeps SP8 for MX)
against the SP8 MX kernel (variant 0): bit-equality on the bias / residual / alpha / RoPE / split-K
forms under the same split (the default split models of the two schedules differ: the w4 one is refit,
plan_split), then interleaved timing on the config-5 forward shapes.  Run on the GPU box: python tools/w4mx_check.py"""
import os as _os
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import json
import sys

import torch

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

dev = "cuda"


def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device=dev) * 2 - 1) * scale).bfloat16()


def run(v, fn):
    call("ospo_set_gemm_variant", v)
    out = fn()
    torch.cuda.synchronize()
    call("ospo_set_gemm_variant", 0)
    return out


def check(name, fn):
    o0 = run(0, fn)   # SP8 MX (the default)
    o1 = run(52, fn)  # w4 MX
    ok = bool(torch.equal(o0, o1))
    print(json.dumps({"case": name, "bit_equal": ok, "max_abs_diff": float((o0.float() - o1.float()).abs().max()),
                      "finite": bool(torch.isfinite(o1.float()).all())}), flush=True)
    return ok


def correctness():
    ok = True
    torch.manual_seed(1)
    for (M, N, K, K2) in [(1000, 512, 512, 64), (4800, 4096, 4096, 64), (777, 768, 1024, 128), (300, 256, 1024, 0),
                          (4800, 12288, 4096, 128), (4800, 4096, 11008, 64), (4608, 4096, 2048, 0)]:
        a, b = rnd(M, K), rnd(N, K, scale=0.05)
        qa, qb = ops.MX8.of(a), ops.MX8.of(b)
        a2 = rnd(M, K2) if K2 else None
        b2 = rnd(N, K2, scale=0.05) if K2 else None
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        bias, res = rnd(N, scale=0.5), rnd(M, N, scale=0.5)

        def f(out=out, qa=qa, qb=qb, a2=a2, b2=b2):
            out.fill_(7)
            ops.gemm_nt_mx8(qa, qb, out, a2=a2, b2=b2, split=1)  # (the two schedules' split models differ)
            return out.clone()
        ok &= check(f"plain M{M} N{N} K{K} K2{K2}", f)

        def g(out=out, qa=qa, qb=qb, a2=a2, b2=b2, bias=bias, res=res):
            out.fill_(7)
            ops.gemm_nt_mx8(qa, qb, out, a2=a2, b2=b2, alpha=0.75, bias=bias, residual=res, split=1)
            return out.clone()
        ok &= check(f"bias+res M{M} N{N} K{K} K2{K2}", g)
        for sp in (2, 4):
            def h(out=out, qa=qa, qb=qb, a2=a2, b2=b2, sp=sp):
                out.fill_(7)
                ops.gemm_nt_mx8(qa, qb, out, a2=a2, b2=b2, split=sp)
                return out.clone()
            ok &= check(f"split{sp} M{M} N{N} K{K} K2{K2}", h)
    M, N, K = 1200, 12288, 4096
    a, b, a2, b2 = rnd(M, K), rnd(N, K, scale=0.05), rnd(M, 64), rnd(N, 64, scale=0.05)
    qa, qb = ops.MX8.of(a), ops.MX8.of(b)
    cos, sin = ops.rope_tables(600, 128, 1e4, dev)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

    def r():
        out.fill_(7)
        ops.gemm_nt_mx8(qa, qb, out, a2=a2, b2=b2, rope=(cos, sin, 600, 8192))
        return out.clone()
    ok &= check("rope qkv M1200", r)
    print(json.dumps({"all_bit_equal": bool(ok)}), flush=True)
    return ok


def timing():
    M = 4800
    shapes = [("qkv_fwd", M, 12288, 4096, 128), ("o_fwd", M, 4096, 4096, 64), ("gu_fwd", M, 22016, 4096, 64),
              ("down_fwd", M, 4096, 11008, 64), ("sq4096", 4096, 4096, 4096, 0)]
    for name, m, n, k, k2 in shapes:
        qa, qb = ops.MX8.of(rnd(m, k)), ops.MX8.of(rnd(n, k, scale=0.05))
        a2 = rnd(m, k2) if k2 else None
        b2 = rnd(n, k2, scale=0.05) if k2 else None
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        res = {0: [], 52: []}
        for _ in range(5):
            for v in (0, 52):
                call("ospo_set_gemm_variant", v)
                ops.gemm_nt_mx8(qa, qb, out, a2=a2, b2=b2)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    ops.gemm_nt_mx8(qa, qb, out, a2=a2, b2=b2)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / 10)
            call("ospo_set_gemm_variant", 0)
        fl = 2.0 * m * n * k
        line = {"shape": name}
        for v, ts in res.items():
            t = sorted(ts)[2]
            line["sp8" if v == 0 else "w4mx"] = {"us": round(t * 1e3, 1), "tflops": round(fl / t / 1e9, 1)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    ok = correctness()
    if ok and "--no-time" not in sys.argv:
        timing()
    sys.exit(0 if ok else 1)
