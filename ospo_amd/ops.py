"""Torch-tensor front end of the HIP kernels (device memory + stream plumbing only).

Every function enqueues on ``torch.cuda.current_stream()`` and calls the C ABI
in ``_lib``; there is no eager-PyTorch fallback on this path.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib
from ._lib import OspoError, call, query

BF16 = torch.bfloat16

# Optional live kernel timer (bench.py): HIP events around each gemm_nt launch on
# the launching stream, aggregated per tile configuration.
_TIMER = None


class KernelTimer:
    def __init__(self):
        self.recs = []  # (tag, algorithmic flops, algorithmic bytes, start event, end event)

    def start(self, stream):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def add(self, tag, flops, e0, stream, nbytes=0.0):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(stream)
        self.recs.append((tag, flops, nbytes, e0, e1))

    def summary(self):
        """{tag: {count, flops, bytes, ms}} (call after synchronize)."""
        out = {}
        for tag, fl, nb, e0, e1 in self.recs:
            d = out.setdefault(tag, {"count": 0, "flops": 0.0, "bytes": 0.0, "ms": 0.0})
            d["count"] += 1
            d["flops"] += fl
            d["bytes"] += nb
            d["ms"] += e0.elapsed_time(e1)
        return out


# workspace counter heads (include/ospo_hip.h ospo_ws_kind): queried from the library, so a resize of a C-side
# head cannot leave Python zeroing the wrong range
WS_GEMM_TAIL, WS_SKINNY, WS_LORA_GDB, WS_DECODE_LINEAR = 0, 1, 2, 3


def ws_counter_bytes(kind: int) -> int:
    n = int(query("ospo_ws_counter_bytes", kind))
    if n <= 0 or n % 4:
        raise OspoError(f"ospo_ws_counter_bytes({kind}) = {n}")
    return n


def zero_ws_counters(ws: torch.Tensor, kind: int) -> None:
    """Zero the counter head at the start of a caller-owned workspace (any dtype)."""
    n = ws_counter_bytes(kind)
    ws.view(torch.uint8)[:n].zero_()


def set_kernel_timer(t: Optional[KernelTimer]):
    global _TIMER
    _TIMER = t


def gemm_nt_tile(M: int, N: int) -> int:
    return query("ospo_gemm_nt_tile", M, N)


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


def _chk(t: torch.Tensor, dtype, name: str):
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor")


def _ld(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a row-major 2-D view")
    return t.stride(0)


# ------------------------------------------------------------------ GEMM
_GEMM_WS = {}


def gemm_ws_bytes(M: int, N: int, K: int, K2: int = 0, mx: bool = False, split: int = 0) -> int:
    """Split-K workspace bytes a 256x256 GEMM of this shape uses (ospo_gemm_nt_ws_bytes; 0: no split)."""
    return int(query("ospo_gemm_nt_ws_bytes", M, N, K, K2, int(mx), int(split)))


def gemm_workspace(device=None, stream=None) -> torch.Tensor:
    """The split-K workspace the GEMM wrappers pass when the caller gives none: one per (device,
    stream), so GEMMs that share it are stream-ordered.  The library splits at most one round of
    tail pieces (tail x split <= 25/32 CUs in the bf16 kernel), so CUs x 256 KiB covers every shape
    plus 4 KiB of zeroed arrival counters that only the ablation library's in-launch tail combine reads
    (OSPO_GEMM_INL=1, measured and rejected: DESIGN.md section 11b).  Allocated once, on the stream that uses it (the caching
    allocator reuses freed memory stream-ordered)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    st = torch.cuda.current_stream(dev) if stream is None else stream
    key = (dev.index, st.cuda_stream)
    ws = _GEMM_WS.get(key)
    if ws is None:
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        with torch.cuda.stream(st):
            ws = _GEMM_WS[key] = torch.zeros(cus * 65536 + ws_counter_bytes(WS_GEMM_TAIL) // 4,
                                              dtype=torch.float32, device=dev)
    return ws


def _ws_args(ws: Optional[torch.Tensor], device, stream):
    if ws is None:
        ws = gemm_workspace(device, stream)
    _chk(ws, torch.float32, "ws")
    return ws.data_ptr(), ws.numel() * 4


def gemm_clock_probe(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, stamps: torch.Tensor) -> None:
    """out = a . b^T through the product's bf16 K loop, unsplit, with per-workgroup s_memtime / s_memrealtime
    stamps (int64 [tiles, 8]; ospo_gemm_clock_probe_bf16): bench.py's box probe."""
    for t, nme in ((a, "a"), (b, "b"), (out, "out")):
        _chk(t, BF16, nme)
    M, K = a.shape
    N = b.shape[0]
    if b.shape[1] != K or tuple(out.shape) != (M, N) or any(t.stride(0) != t.shape[1] for t in (a, b, out)):
        raise ValueError("gemm_clock_probe: a [M, K], b [N, K], out [M, N], all dense")
    if stamps.dtype != torch.int64 or not stamps.is_contiguous():
        raise ValueError("gemm_clock_probe: stamps must be contiguous int64")
    call("ospo_gemm_clock_probe_bf16", _p(a), _p(b), _p(out), M, N, K, _p(stamps), stamps.numel() * 8, _s())


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, *, a2=None, b2=None, alpha: float = 1.0,
            bias=None, residual=None, rope=None, dropout=None, split: int = 0, ws=None,
            keep_bits=None) -> torch.Tensor:
    """out[M,N] = bf16(alpha*(a.b^T + a2.b2^T) + bias) [+ residual]  (nn.Linear layout b=[N,K]).
    rope=(cos, sin, T, ncols): RoPE forward fused on output columns < ncols (ospo_gemm_nt_rope_bf16).
    dropout=(seed, p): the a2.b2^T term is masked like the adapter input's dropout (ospo_gemm_nt_dropout_bf16);
    keep_bits: that mask as the forward's lora_skinny keep-bit output (uint8 [M * N / 8]) instead of re-hashed.
    split: the tail round's split-K (0 = the library's cost model, 1 = none, 2..8 pinned); ws: the fp32
    split-K workspace (default: gemm_workspace of the current stream)."""
    for t, n in ((a, "a"), (b, "b"), (out, "out")):
        _chk(t, BF16, n)
    M, K = a.shape
    N = b.shape[0]
    if b.shape[1] != K or out.shape[0] != M or out.shape[1] != N:
        raise ValueError(f"gemm_nt shape mismatch a{tuple(a.shape)} b{tuple(b.shape)} out{tuple(out.shape)}")
    K2 = 0
    if a2 is not None:
        K2 = a2.shape[1]
        if a2.shape[0] != M or b2.shape != (N, K2):
            raise ValueError("gemm_nt K-extension shape mismatch")
    st = torch.cuda.current_stream()
    wsp, wsb = _ws_args(ws, a.device, st)
    e0 = _TIMER.start(st) if _TIMER is not None else None
    if dropout is not None and dropout[1] > 0:
        if bias is not None or residual is not None or alpha != 1.0 or rope is not None or a2 is None:
            raise ValueError("gemm_nt: dropout needs a2/b2 and excludes bias / residual / alpha / rope")
        if keep_bits is not None and (keep_bits.dtype != torch.uint8 or keep_bits.numel() * 8 < M * N):
            raise ValueError("gemm_nt: keep_bits must be uint8 with >= M*N/8 elements")
        call("ospo_gemm_nt_dropout_bf16", _p(a), _ld(a), _p(b), _ld(b), M, N, K, _p(a2), _ld(a2), _p(b2), _ld(b2),
             K2, _p(out), _ld(out), int(dropout[0]) & 0xFFFFFFFF, float(dropout[1]), _p(keep_bits), int(split), wsp,
             wsb, st.cuda_stream)
    elif rope is not None:
        if bias is not None or residual is not None or alpha != 1.0:
            raise ValueError("gemm_nt: rope excludes bias / residual / alpha")
        cos, sin, T, ncols = rope
        call("ospo_gemm_nt_rope_bf16", _p(a), _ld(a), _p(b), _ld(b), M, N, K,
             _p(a2), _ld(a2) if a2 is not None else 0, _p(b2), _ld(b2) if b2 is not None else 0, K2,
             _p(out), _ld(out), _p(cos), _p(sin), int(T), int(ncols), int(split), wsp, wsb, st.cuda_stream)
    else:
        call("ospo_gemm_nt_bf16", _p(a), _ld(a), _p(b), _ld(b), M, N, K,
             _p(a2), _ld(a2) if a2 is not None else 0, _p(b2), _ld(b2) if b2 is not None else 0, K2, float(alpha),
             _p(bias), _p(residual), _ld(residual) if residual is not None else 0, _p(out), _ld(out), int(split),
             wsp, wsb, st.cuda_stream)
    if e0 is not None:
        # algorithmic flops: the frozen product only (the LoRA K-extension is not counted)
        # algorithmic bytes: A, B, C once each (+ the bf16 residual read)
        nbytes = 2.0 * (M * K + N * K + M * N + (M * N if residual is not None else 0))
        _TIMER.add(f"gemm_nt_{gemm_nt_tile(M, N)}x{N if N < 256 else 256}", 2.0 * M * N * K, e0, st, nbytes)
    return out


def gemm_nt_swiglu_bwd(a: torch.Tensor, b: torch.Tensor, gu: torch.Tensor, dgu: torch.Tensor, *, a2=None, b2=None,
                       dropout=None, split: int = 0, ws=None) -> torch.Tensor:
    """dgu[M, 2F] = SwiGLU backward of dh = bf16(a.b^T + a2.b2^T) (b = down_proj's W^T, [F, K]) at gu [M, 2F],
    without storing dh (ospo_gemm_nt_swiglu_bwd_bf16; bit-identical to gemm_nt(..., dropout) + swiglu_bwd).
    dropout=(seed, p): the a2.b2^T term is masked as in gemm_nt."""
    for t, n in ((a, "a"), (b, "b"), (gu, "gu"), (dgu, "dgu")):
        _chk(t, BF16, n)
    M, K = a.shape
    F = b.shape[0]
    if b.shape[1] != K or gu.shape != (M, 2 * F) or dgu.shape != (M, 2 * F):
        raise ValueError(f"gemm_nt_swiglu_bwd shape mismatch a{tuple(a.shape)} b{tuple(b.shape)} "
                         f"gu{tuple(gu.shape)} dgu{tuple(dgu.shape)}")
    K2 = 0
    if a2 is not None:
        K2 = a2.shape[1]
        if a2.shape[0] != M or b2.shape != (F, K2):
            raise ValueError("gemm_nt_swiglu_bwd K-extension shape mismatch")
    seed, p = (0, 0.0) if dropout is None else (int(dropout[0]) & 0xFFFFFFFF, float(dropout[1]))
    if p > 0 and a2 is None:
        raise ValueError("gemm_nt_swiglu_bwd: dropout needs a2/b2")
    st = torch.cuda.current_stream()
    wsp, wsb = _ws_args(ws, a.device, st)
    e0 = _TIMER.start(st) if _TIMER is not None else None
    call("ospo_gemm_nt_swiglu_bwd_bf16", _p(a), _ld(a), _p(b), _ld(b), M, F, K,
         _p(a2), _ld(a2) if a2 is not None else 0, _p(b2), _ld(b2) if b2 is not None else 0, K2,
         _p(gu), _ld(gu), _p(dgu), _ld(dgu), seed, p, int(split), wsp, wsb, st.cuda_stream)
    if e0 is not None:
        # algorithmic: the frozen product's flops; bytes A, B once, gu read and dgu written (2F columns each)
        nbytes = 2.0 * (M * K + F * K + 4 * M * F)
        _TIMER.add(f"gemm_nt_{gemm_nt_tile(M, F)}x{F if F < 256 else 256}", 2.0 * M * F * K, e0, st, nbytes)
    return dgu


# ------------------------------------------------------------ MXFP8 (config 5)
class MX8:
    """An MXFP8 operand on the device: e4m3 bytes q [rows, K] + E8M0 scales in the GEMM's tile
    layout (include/ospo_hip.h ospo_quant_mx8).  Preallocate once and refill with quant_mx8."""

    def __init__(self, rows: int, K: int, device):
        if K % 128:
            raise ValueError("MX8: K must be a multiple of 128")
        self.rows, self.K = rows, K
        self.q = torch.empty(rows, K, dtype=torch.uint8, device=device)
        nbytes = query("ospo_mx8_scale_bytes", rows, K)
        self.s = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        self.m = 0  # rows filled by the last quant_mx8

    @classmethod
    def of(cls, x: torch.Tensor) -> "MX8":
        t = cls(x.shape[0], x.shape[1], x.device)
        return quant_mx8(x, t)


def quant_mx8(x: torch.Tensor, out: MX8) -> MX8:
    """out <- MXFP8(x), x bf16 [M, K] (M <= out.rows)."""
    _chk(x, BF16, "x")
    M, K = x.shape
    if K != out.K or M > out.rows:
        raise ValueError(f"quant_mx8: x{tuple(x.shape)} does not fit MX8[{out.rows}, {out.K}]")
    call("ospo_quant_mx8", _p(x), _ld(x), M, K, _p(out.q), out.q.stride(0), _p(out.s), _s())
    out.m = M
    return out


def gemm_nt_mx8(a: MX8, b: MX8, out: torch.Tensor, *, a2=None, b2=None, alpha: float = 1.0, bias=None,
                residual=None, rope=None, dropout=None, split: int = 0, ws=None) -> torch.Tensor:
    """out[M, N] = bf16(alpha*(deq(a).deq(b)^T + a2.b2^T) + bias) [+ residual] on block-scaled fp8 MFMA;
    M = a.m rows (the last quant_mx8), b = the weight [N, K].  rope / dropout as gemm_nt."""
    _chk(out, BF16, "out")
    M, N, K = a.m, b.m, a.K
    if b.K != K or out.shape[0] != M or out.shape[1] != N:
        raise ValueError(f"gemm_nt_mx8 shape mismatch a[{M},{K}] b[{N},{b.K}] out{tuple(out.shape)}")
    K2 = 0
    if a2 is not None:
        K2 = a2.shape[1]
        if a2.shape[0] != M or b2.shape != (N, K2):
            raise ValueError("gemm_nt_mx8 K-extension shape mismatch")
    cos = sin = None
    T = ncols = 0
    if rope is not None:
        cos, sin, T, ncols = rope
    seed, p = (0, 0.0) if dropout is None else (int(dropout[0]) & 0xFFFFFFFF, float(dropout[1]))
    st = torch.cuda.current_stream()
    wsp, wsb = _ws_args(ws, out.device, st)
    e0 = _TIMER.start(st) if _TIMER is not None else None
    call("ospo_gemm_nt_mx8", _p(a.q), a.q.stride(0), _p(a.s), _p(b.q), b.q.stride(0), _p(b.s), M, N, K,
         _p(a2), _ld(a2) if a2 is not None else 0, _p(b2), _ld(b2) if b2 is not None else 0, K2, float(alpha),
         _p(bias), _p(residual), _ld(residual) if residual is not None else 0, _p(out), _ld(out),
         _p(cos), _p(sin), int(T), int(ncols), seed, p, int(split), wsp, wsb, st.cuda_stream)
    if e0 is not None:
        nbytes = 1.0 * (M * K + N * K) + 2.0 * (M * N + (M * N if residual is not None else 0))
        _TIMER.add("gemm_nt_mx8_256x256", 2.0 * M * N * K, e0, st, nbytes)
    return out


def gemm_f32acc(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, *, a_kmajor: bool, b_kmajor: bool,
                k_splits: int = 1, alpha: float = 1.0, diag: Optional[tuple] = None,
                b_dropout: Optional[tuple] = None, keep_bits: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[M,N] (fp32) += alpha * op(a) . op(b)^T.
    a_kmajor: a is [K, M] else [M, K];  b_kmajor: b is [K, N] else [N, K].
    diag=(nblk, r): block-diagonal scatter (see include/ospo_hip.h).
    b_dropout=(seed, p): LoRA dropout recomputed on the K-major b (lora_skinny's mask and scaling), or read from
    keep_bits (lora_skinny's keep-bit output of b, uint8 [K * N / 8]) when given."""
    _chk(a, BF16, "a")
    _chk(b, BF16, "b")
    _chk(out, torch.float32, "out")
    K, M = a.shape if a_kmajor else a.shape[::-1]
    Kb, N = b.shape if b_kmajor else b.shape[::-1]
    if K != Kb:
        raise ValueError(f"gemm_f32acc K mismatch {K} vs {Kb}")
    nblk, r = diag if diag else (0, 0)
    ldc = _ld(out) if not diag else 0
    if b_dropout is not None:
        seed, p = b_dropout
        if keep_bits is not None and (keep_bits.dtype != torch.uint8 or keep_bits.numel() * 8 < K * N):
            raise ValueError("gemm_f32acc: keep_bits must be uint8 with >= K*N/8 elements")
        call("ospo_gemm_f32acc_bdrop", _p(a), _ld(a), int(a_kmajor), _p(b), _ld(b), int(b_kmajor), M, N, K,
             int(k_splits), float(alpha), _p(out), ldc, nblk, r, int(seed) & 0xFFFFFFFF, float(p), _p(keep_bits), _s())
        return out
    call("ospo_gemm_f32acc", _p(a), _ld(a), int(a_kmajor), _p(b), _ld(b), int(b_kmajor), M, N, K, int(k_splits),
         float(alpha), _p(out), ldc, nblk, r, _s())
    return out


def lora_wgrad(x: torch.Tensor, s: torch.Tensor, out: torch.Tensor, *, mode: int, s_cols: int, splits: int,
               nmod: int = 0, r: int = 0, dropout: Optional[tuple] = None) -> torch.Tensor:
    """LoRA weight gradients streamed over the big operand x [Mk, N] (ospo_lora_wgrad), fp32 atomics into out:
    mode 0 (dA): out[j, n] += sum_m s[m, j] x[m, n], j < s_cols (s [Mk, Rp], Rp = 64 or 128);
    mode 1 (dB): out[n, jr] += sum_m x[m, n] s[m, (n // nmod) * r + jr]  (block diagonal, out [N, r]).
    dropout=(seed, p) (mode 0): x is masked with the adapter input's forward mask as it is read."""
    _chk(x, BF16, "x")
    _chk(s, BF16, "s")
    _chk(out, torch.float32, "out")
    K, N = x.shape
    if s.shape[0] != K:
        raise ValueError(f"lora_wgrad: {s.shape[0]} rows of s, {K} of x")
    seed, p = dropout if dropout is not None else (0, 0.0)
    ldc = _ld(out) if mode == 0 else 0
    call("ospo_lora_wgrad", _p(x), _ld(x), N, _p(s), _ld(s), int(s_cols), K, int(mode), int(nmod), int(r), _p(out),
         ldc, int(splits), int(seed) & 0xFFFFFFFF, float(p), _s())
    return out


def lora_da(x: torch.Tensor, s: torch.Tensor, out: torch.Tensor, *, s_cols: int, splits: int = 0,
            dropout: Optional[tuple] = None, keep_bits: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dA of one adapter group as one stream over x [K, N] (ospo_lora_da): out[j, n] += sum_m s[m, j]
    dropout(x)[m, n] for j < s_cols, fp32 atomics into out [s_cols, >= N] (s [K, Rp], Rp = 64 or 128,
    K % 64 == 0, N % 128 == 0).  dropout=(seed, p): x is masked with the adapter input's forward mask as it
    is read -- from keep_bits (lora_skinny's keep-bit output of this x) when given, else re-hashed.
    splits: K-tile ranges per 128-column stripe (0: ~2 workgroups per CU)."""
    if keep_bits is not None and (keep_bits.dtype != torch.uint8 or keep_bits.numel() * 8 < x.shape[0] * x.shape[1]):
        raise ValueError("lora_da: keep_bits must be uint8 with >= K*N/8 elements")
    _chk(x, BF16, "x")
    _chk(s, BF16, "s")
    _chk(out, torch.float32, "out")
    K, N = x.shape
    if s.shape[0] != K:
        raise ValueError(f"lora_da: {s.shape[0]} rows of s, {K} of x")
    if splits <= 0:
        splits = lora_da_splits(K, N, x.device)
    seed, p = dropout if dropout is not None else (0, 0.0)
    call("ospo_lora_da", _p(x), _ld(x), N, _p(s), _ld(s), int(s_cols), K, _p(out), _ld(out), int(splits),
         int(seed) & 0xFFFFFFFF, float(p), _p(keep_bits) if p > 0 else None, _s())
    return out


def lora_da_splits(K: int, N: int, device=None) -> int:
    """K-tile ranges per 128-column stripe of lora_da: ~2 workgroups per CU, >= 4 K-tiles each.  (Round 6, on
    the side stream in the step: 1, 2 or 4 workgroups per CU within 0.1 % of each other over 4 alternating rounds,
    profiles/r06/da_wgs_per_cu_ab.txt.)"""
    cus = torch.cuda.get_device_properties(device).multi_processor_count if torch.cuda.is_available() else 256
    stripes = max(1, N // 128)
    return int(max(1, min(K // 64 // 4, round(2 * cus / stripes))))


def f32_to_bf16(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    _chk(src, torch.float32, "src")
    _chk(dst, BF16, "dst")
    if src.numel() != dst.numel() or not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("f32_to_bf16: size/contiguity mismatch")
    call("ospo_f32_to_bf16", _p(src), _p(dst), src.numel(), float(scale), _s())
    return dst


# ---------------------------------------------------------------- RMSNorm
def _mx_target(mx, M: int, K: int, who: str):
    if K != mx.K or M > mx.rows:
        raise ValueError(f"{who}: output [{M}, {K}] does not fit MX8[{mx.rows}, {mx.K}]")


def rmsnorm_fwd(x, w, y, rstd, eps: float, mx: "MX8 | None" = None):
    """y = rmsnorm(x) * w; with mx, also mx <- MXFP8(y) in the same pass (== quant_mx8(y, mx))."""
    M, D = x.shape
    if mx is None:
        call("ospo_rmsnorm_fwd", _p(x), _p(w), _p(y), _p(rstd), M, D, float(eps), _s())
        return y
    _mx_target(mx, M, D, "rmsnorm_fwd")
    call("ospo_rmsnorm_fwd_mx8", _p(x), _p(w), _p(y), _p(rstd), M, D, float(eps), _p(mx.q), mx.q.stride(0),
         _p(mx.s), _s())
    mx.m = M
    return y


def rmsnorm_bwd(dy, x, w, rstd, dx, dres=None, mx: "MX8 | None" = None):
    """dx = rmsnorm_bwd(dy) [+ dres]; with mx, also mx <- MXFP8(dx) in the same pass."""
    M, D = x.shape
    if mx is None:
        call("ospo_rmsnorm_bwd", _p(dy), _p(x), _p(w), _p(rstd), _p(dres), _p(dx), M, D, _s())
        return dx
    _mx_target(mx, M, D, "rmsnorm_bwd")
    call("ospo_rmsnorm_bwd_mx8", _p(dy), _p(x), _p(w), _p(rstd), _p(dres), _p(dx), M, D, _p(mx.q),
         mx.q.stride(0), _p(mx.s), _s())
    mx.m = M
    return dx


# ------------------------------------------------------------------- RoPE
def rope(qkv, q_col, k_col, S, T, n_heads, head_dim, cos_tab, sin_tab, backward=False):
    call("ospo_rope_bwd" if backward else "ospo_rope_fwd", _p(qkv), _ld(qkv), q_col, k_col, S, T, n_heads,
         head_dim, _p(cos_tab), _p(sin_tab), _s())
    return qkv


def rope_tables(T: int, head_dim: int, theta: float, device) -> tuple:
    """HF LlamaRotaryEmbedding: fp32 inv_freq/outer product, cos/sin cast to bf16; first half only."""
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    freqs = torch.outer(torch.arange(T, dtype=torch.float32), inv_freq)
    return (freqs.cos().to(BF16).contiguous().to(device), freqs.sin().to(BF16).contiguous().to(device))


# ----------------------------------------------------------------- SwiGLU
def swiglu_fwd(gu, h, mx: "MX8 | None" = None):
    """h = silu(g) * u; with mx, also mx <- MXFP8(h) in the same pass."""
    M, F2 = gu.shape
    if mx is None:
        call("ospo_swiglu_fwd", _p(gu), _ld(gu), _p(h), _ld(h), M, F2 // 2, _s())
        return h
    _mx_target(mx, M, F2 // 2, "swiglu_fwd")
    call("ospo_swiglu_fwd_mx8", _p(gu), _ld(gu), _p(h), _ld(h), M, F2 // 2, _p(mx.q), mx.q.stride(0), _p(mx.s),
         _s())
    mx.m = M
    return h


def swiglu_bwd(dh, gu, dgu, mx: "MX8 | None" = None):
    """dgu = d(g|u); with mx, also mx <- MXFP8(dgu) (K = 2F) in the same pass."""
    M, F2 = gu.shape
    if mx is None:
        call("ospo_swiglu_bwd", _p(dh), _ld(dh), _p(gu), _ld(gu), _p(dgu), _ld(dgu), M, F2 // 2, _s())
        return dgu
    _mx_target(mx, M, F2, "swiglu_bwd")
    call("ospo_swiglu_bwd_mx8", _p(dh), _ld(dh), _p(gu), _ld(gu), _p(dgu), _ld(dgu), M, F2 // 2, _p(mx.q),
         mx.q.stride(0), _p(mx.s), _s())
    mx.m = M
    return dgu


# -------------------------------------------------------------- attention
def flash_attn_fwd(qkv, q_col, k_col, v_col, o, lse, S, T, n_heads, head_dim, scale, mx: "MX8 | None" = None):
    """Causal flash attention; with mx, also mx <- MXFP8(o) from the output stores (== quant_mx8(o, mx))."""
    if mx is None:
        call("ospo_flash_attn_fwd", _p(qkv), _ld(qkv), q_col, k_col, v_col, _p(o), _ld(o), _p(lse), S, T, n_heads,
             head_dim, float(scale), _s())
        return o, lse
    _mx_target(mx, S * T, n_heads * head_dim, "flash_attn_fwd")
    call("ospo_flash_attn_fwd_mx8", _p(qkv), _ld(qkv), q_col, k_col, v_col, _p(o), _ld(o), _p(lse), S, T, n_heads,
         head_dim, float(scale), _p(mx.q), mx.q.stride(0), _p(mx.s), mx.K, _s())
    mx.m = S * T
    return o, lse


def flash_attn_bwd_ws_bytes(S: int, T: int, n_heads: int) -> int:
    return int(query("ospo_flash_attn_bwd_ws_bytes", S, T, n_heads))


def flash_attn_bwd_ws(S: int, T: int, n_heads: int, device) -> torch.Tensor:
    """The bf16 dS^T workspace of the 5-product backward (zeroed once; see ospo_flash_attn_bwd)."""
    return torch.zeros(flash_attn_bwd_ws_bytes(S, T, n_heads) // 2, dtype=BF16, device=device)


def flash_attn_bwd(qkv, q_col, k_col, v_col, o, dout, lse, delta_ws, ds_ws, dqkv, S, T, n_heads, head_dim, scale,
                   rope_cos=None, rope_sin=None, mx: "MX8 | None" = None):
    """Attention backward; with rope_cos/rope_sin the RoPE backward is fused into the dq/dk stores.
    ds_ws (flash_attn_bwd_ws): dK/dV store dS^T and dQ = dS.K reads it (5 MFMA products); None: the
    dQ kernel recomputes S and dP (7 products).  With mx (needs ds_ws), also mx <- MXFP8 of the dqkv
    matrix's first mx.K columns from the dq / dk / dv stores (== quant_mx8(dqkv, mx))."""
    if ds_ws is not None and ds_ws.numel() * 2 < flash_attn_bwd_ws_bytes(S, T, n_heads):
        raise ValueError("flash_attn_bwd: dS workspace too small")
    if mx is None:
        call("ospo_flash_attn_bwd", _p(qkv), _ld(qkv), q_col, k_col, v_col, _p(o), _ld(o), _p(dout), _ld(dout),
             _p(lse), _p(delta_ws), _p(ds_ws), _p(dqkv), _ld(dqkv), S, T, n_heads, head_dim, float(scale),
             _p(rope_cos), _p(rope_sin), _s())
        return dqkv
    _mx_target(mx, S * T, dqkv.shape[1], "flash_attn_bwd")
    call("ospo_flash_attn_bwd_mx8", _p(qkv), _ld(qkv), q_col, k_col, v_col, _p(o), _ld(o), _p(dout), _ld(dout),
         _p(lse), _p(delta_ws), _p(ds_ws), _p(dqkv), _ld(dqkv), S, T, n_heads, head_dim, float(scale),
         _p(rope_cos), _p(rope_sin), _p(mx.q), mx.q.stride(0), _p(mx.s), mx.K, _s())
    mx.m = S * T
    return dqkv


# -------------------------------------------------------- embed / gather
def assemble_inputs(text_ids, B, Lt, table, img_emb, N, D, x0):
    call("ospo_assemble_inputs", _p(text_ids), B, Lt, _p(table), table.shape[0], _p(img_emb), N, D, _p(x0), _s())
    return x0


def gen_aligner_in(ids, gen_embed, w1, b1, out):
    R = ids.numel()
    V, E = gen_embed.shape
    D = w1.shape[0]
    call("ospo_gen_aligner_in", _p(ids), R, _p(gen_embed), V, E, _p(w1), _p(b1), D, _p(out), _s())
    return out


def gather_rows(src, S, T, t0, N, dst):
    call("ospo_gather_rows", _p(src), _ld(src), S, T, t0, N, src.shape[1], _p(dst), _s())
    return dst


def scatter_rows(src, S, T, t0, N, dst):
    call("ospo_scatter_rows", _p(src), S, T, t0, N, src.shape[1], _p(dst), _ld(dst), dst.shape[0], _s())
    return dst


def row_dot_sum(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, rows_per_group: int, *, add=None,
                add_scale: float = 1.0, accumulate: bool = False) -> torch.Tensor:
    """out[g] (fp32) (+)= sum over rows_per_group rows of x (bf16 [G * rows_per_group, D]) of row . w (fp32 [D])
    [+ add_scale * add[0]] -- ospo_row_dot_sum (deterministic fp32 reduction)."""
    _chk(x, BF16, "x")
    _chk(w, torch.float32, "w")
    _chk(out, torch.float32, "out")
    R, D = x.shape
    if R % rows_per_group or out.numel() < R // rows_per_group or w.numel() != D:
        raise ValueError(f"row_dot_sum: x{tuple(x.shape)} w{tuple(w.shape)} out{tuple(out.shape)} rows {rows_per_group}")
    G = R // rows_per_group
    nb = int(query("ospo_row_dot_sum_ws_bytes", G, rows_per_group, D))
    ws = torch.empty((nb + 15) // 16 * 4, dtype=torch.float32, device=x.device)
    call("ospo_row_dot_sum", _p(x), _ld(x), G, rows_per_group, D, _p(w), _p(add), float(add_scale), int(accumulate),
         _p(out), _p(ws), ws.numel() * 4, _s())
    return out


def gelu_fwd(x, y):
    call("ospo_gelu_fwd", _p(x), _p(y), x.numel(), _s())
    return y


def gelu_bwd(dy, x_pre, dx):
    call("ospo_gelu_bwd", _p(dy), _p(x_pre), _p(dx), dy.numel(), _s())
    return dx


# ---------------------------------------------------------------- logprob
def logprob_fwd(logits, labels, N, lse, tok, seq):
    R, V = logits.shape
    call("ospo_logprob_fwd", _p(logits), V, _p(labels), R, N, _p(lse), _p(tok), _p(seq), _s())
    return seq


def logprob_bwd(logits, labels, lse, N, g_seq, dlogits):
    R, V = logits.shape
    call("ospo_logprob_bwd", _p(logits), V, _p(labels), _p(lse), R, N, _p(g_seq), _p(dlogits), _s())
    return dlogits


# ------------------------------------------------------------------ SimPO
LOSS_TYPES = {"sigmoid": 0, "hinge": 1}


def loss_type_id(loss_type: str) -> int:
    if loss_type not in LOSS_TYPES:
        raise ValueError(f"Unknown loss type: {loss_type}. Should be one of ['sigmoid', 'hinge']")
    return LOSS_TYPES[loss_type]


def simpo_fwd(logps, B, beta, gbr, ls, loss_type, losses, mean, rewards):
    call("ospo_simpo_fwd", _p(logps), B, float(beta), float(gbr), float(ls), loss_type_id(loss_type), _p(losses),
         _p(mean), _p(rewards), _s())


def simpo_bwd(logps, B, beta, gbr, ls, loss_type, g_loss, glogps):
    call("ospo_simpo_bwd", _p(logps), B, float(beta), float(gbr), float(ls), loss_type_id(loss_type), _p(g_loss),
         _p(glogps), _s())


# ------------------------------------------------------------- LoRA pack
def lora_pack(A_flat, B_flat, nmods, r, Kin, Nmod, Rp, Acat, AcatT, Bcat, BT=None, n_layers=1, layer_stride=0):
    call("ospo_lora_pack", _p(A_flat), _p(B_flat), nmods, r, Kin, Nmod, Rp, _p(Acat), _p(AcatT), _p(Bcat), _p(BT),
         n_layers, layer_stride, _s())


def lora_skinny_ws_bytes(M_out, K, n_tiles) -> int:
    return int(query("ospo_lora_skinny_ws_bytes", M_out, K, n_tiles))


def lora_skinny_ws(M_out, K, n_tiles=4, device="cuda") -> torch.Tensor:
    """Workspace for ospo_lora_skinny's split-K partials."""
    n = lora_skinny_ws_bytes(M_out, K, n_tiles)
    return torch.zeros((n + 15) // 16 * 4, dtype=torch.float32, device=device)


def lora_skinny(a, bt, out, M, M_out, K, n_tiles, a_koff=0, scale=1.0, b_rows=None, ws=None, module_tiles=1,
                dropout=None, xd=None, keep_bits=None):
    """out[:M_out, :] (bf16) = scale * a . bt^T per 16-column n-tile (see ospo_lora_skinny).
    dropout=(seed, p): LoRA dropout on a (dense mode); the masked a is written to xd if given, the keep
    decisions as bits (uint8 [>= M * K / 8], row-major) to keep_bits if given."""
    if ws is None:
        ws = lora_skinny_ws(M_out, K, n_tiles, a.device)
    seed, p = dropout if dropout is not None else (0, 0.0)
    if keep_bits is not None and (keep_bits.dtype != torch.uint8 or keep_bits.numel() * 8 < M * K):
        raise ValueError("lora_skinny: keep_bits must be uint8 with >= M*K/8 elements")
    call("ospo_lora_skinny", _p(a), _ld(a), _p(bt), _ld(bt), bt.shape[0] if b_rows is None else b_rows, M, M_out,
         K, n_tiles, a_koff, module_tiles, float(scale), _p(out), _ld(out), out.shape[1], _p(ws),
         ws.numel() * ws.element_size(), int(seed) & 0xFFFFFFFF, float(p), _p(xd), _ld(xd) if xd is not None else 0,
         _p(keep_bits), _s())


def swiglu_fwd_lora_down(gu, h, bt, out, M, M_out, F, n_tiles, scale=1.0, b_rows=None, ws=None, dropout=None,
                         keep_bits=None):
    """h[:M] = SwiGLU(gu) (as swiglu_fwd) and out[:M_out] = scale * dropout(h) . bt^T (as lora_skinny on h) in
    one stream over gu (ospo_swiglu_fwd_lora_down); keep_bits as lora_skinny's."""
    _chk(gu, BF16, "gu")
    _chk(h, BF16, "h")
    if ws is None:
        ws = lora_skinny_ws(M_out, F, n_tiles, gu.device)
    seed, p = dropout if dropout is not None else (0, 0.0)
    if keep_bits is not None and (keep_bits.dtype != torch.uint8 or keep_bits.numel() * 8 < M * F):
        raise ValueError("swiglu_fwd_lora_down: keep_bits must be uint8 with >= M*F/8 elements")
    call("ospo_swiglu_fwd_lora_down", _p(gu), _ld(gu), _p(h), _ld(h), M, M_out, F, _p(bt), _ld(bt),
         bt.shape[0] if b_rows is None else b_rows, n_tiles, float(scale), _p(out), _ld(out), out.shape[1], _p(ws),
         ws.numel() * ws.element_size(), int(seed) & 0xFFFFFFFF, float(p), _p(keep_bits), _s())


def query_gdb_ws(M, nmods, Nmod, r=16) -> int:
    """Bytes of ospo_lora_gdb_r's workspace (a module's r columns are r / 16 halves of 16)."""
    return int(query("ospo_lora_gdb_ws_bytes", M, nmods * (r // 16), Nmod))


def lora_gdb_ws(M, nmods, Nmod, device="cuda", r=16) -> torch.Tensor:
    """Workspace for ospo_lora_gdb_r: its row-block counters (zero at allocation, left zero) and the fp32 partials
    of g."""
    n = query_gdb_ws(M, nmods, Nmod, r)
    return torch.zeros((n + 15) // 16 * 4, dtype=torch.float32, device=device)


def lora_gdb(dy, bt, u, out, dB, M, M_out, nmods, Nmod, scale, ws=None, r=16):
    """One stream over dy (LoRA r = 16 or 32): out[:M_out] (bf16) = scale * dy . B (block diagonal, as
    lora_skinny's g; rows M.. and columns r*nmods.. zero) and dB [nmods*Nmod, r] (fp32) += dy^T . u."""
    _chk(dB, torch.float32, "dB")
    if ws is None:
        ws = lora_gdb_ws(M, nmods, Nmod, dy.device, r)
    call("ospo_lora_gdb_r", _p(dy), _ld(dy), _p(bt), _ld(bt), _p(u), _ld(u), M, M_out, nmods, Nmod, int(r),
         float(scale), _p(out), _ld(out), out.shape[1], _p(dB), _p(ws), ws.numel() * ws.element_size(), _s())


def swiglu_lora_gdb(dh, gu, dgu, bt, u, out, dB, M, M_out, scale, ws=None, r=16):
    """dgu[:M] = swiglu_bwd(dh, gu) and lora_gdb(dgu, nmods=2, Nmod=F, r) in one stream over (dh, gu)
    (ospo_swiglu_lora_gdb_r; same bits as swiglu_bwd + lora_gdb)."""
    _chk(dB, torch.float32, "dB")
    F = dh.shape[1]
    if gu.shape[1] < 2 * F or dgu.shape[1] < 2 * F:
        raise ValueError(f"swiglu_lora_gdb: gu/dgu need 2F = {2 * F} columns")
    if ws is None:
        ws = lora_gdb_ws(M, 2, F, dh.device, r)
    call("ospo_swiglu_lora_gdb_r", _p(dh), _ld(dh), _p(gu), _ld(gu), _p(dgu), _ld(dgu), _p(bt), _ld(bt), _p(u),
         _ld(u), M, M_out, F, int(r), float(scale), _p(out), _ld(out), out.shape[1], _p(dB), _p(ws),
         ws.numel() * ws.element_size(), _s())


# -------------------------------------------------------------- optimizer
def sumsq(g, out, ws=None):
    """out[0] += sum(g^2) in a fixed order (ws: 2048-float scratch, allocated here when None)."""
    if ws is None:
        ws = torch.empty(2048, dtype=torch.float32, device=g.device)
    call("ospo_sumsq", _p(g), g.numel(), _p(out), _p(ws), _s())


def adamw_clip(p, g, m, v, lr, beta1, beta2, eps, wd, step, sumsq_buf, max_norm):
    call("ospo_adamw_clip", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1), float(beta2),
         float(eps), float(wd), int(step), _p(sumsq_buf), float(max_norm), _s())


# ------------------------------------------------------ step-3 T2I decode (config 4)
def decode_gemv_ws(R: int, N: int, K: int, device) -> torch.Tensor:
    nbytes = query("ospo_decode_gemv_ws_bytes", R, N, K)
    return torch.zeros(max(nbytes // 4, 4), dtype=torch.float32, device=device)


def tile_decode_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] nn.Linear weight -> the MFMA-tiled decode layout [N/16, K/32, 512] (include/ospo_hip.h,
    ospo_decode_gemv with ldw = 0): tile (nb, ks) holds rows 16 nb.., k 32 ks.. lane-ordered, element
    8 (16 g + l16) + e = w[16 nb + l16, 32 ks + 8 g + e].  A one-time layout copy of a frozen weight."""
    if w.dtype != BF16 or w.dim() != 2:
        raise ValueError(f"tile_decode_weight: expected a 2-D bf16 weight, got {w.dtype} {tuple(w.shape)}")
    N, K = w.shape
    if N % 16 or K % 32:
        raise ValueError(f"tile_decode_weight: [{N}, {K}] needs N % 16 == 0 and K % 32 == 0")
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().view(N // 16, K // 32, 512)


def _decode_w(w: torch.Tensor):
    """(N, K, ldw) of a decode weight: row-major [N, K] or tiled [N/16, K/32, 512] (ldw = 0)."""
    if w.dim() == 3:
        if w.shape[2] != 512 or not w.is_contiguous():
            raise ValueError(f"tiled decode weight must be a contiguous [N/16, K/32, 512] tensor, got {tuple(w.shape)}")
        return w.shape[0] * 16, w.shape[1] * 32, 0
    return w.shape[0], w.shape[1], _ld(w)


def decode_gemv(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, *, bias=None, gelu: bool = False, residual=None,
                ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[R, N] = act(x . w^T + bias) (+ residual), R <= 64 (weight-streaming decode GEMV); w row-major
    [N, K] or tiled by ``tile_decode_weight``."""
    for t, n in ((x, "x"), (w, "w"), (out, "out")):
        _chk(t, BF16, n)
    R, K = x.shape
    N, Kw, ldw = _decode_w(w)
    if Kw != K or out.shape != (R, N):
        raise ValueError(f"decode_gemv shape mismatch x{tuple(x.shape)} w{tuple(w.shape)} out{tuple(out.shape)}")
    call("ospo_decode_gemv", _p(w), ldw, _p(x), _ld(x), R, N, K, _p(bias), int(gelu), _p(residual),
         _ld(residual) if residual is not None else 0, _p(out), _ld(out), _p(ws), 0 if ws is None else ws.numel() * 4,
         _s())
    return out


DL_EPI = {"plain": 0, "kv": 1, "swiglu": 2}


def decode_linear_ws(R: int, N: int, K: int, device) -> torch.Tensor:
    """Workspace of ospo_decode_linear: zeroed (its 4 KiB counter head must start at zero; every call
    leaves it zero)."""
    nbytes = int(query("ospo_decode_linear_ws_bytes", R, N, K))
    if nbytes == 0:
        raise ValueError(f"decode_linear: unsupported shape R={R} N={N} K={K}")
    return torch.zeros((nbytes + 15) // 16 * 4, dtype=torch.float32, device=device)


def head_major_qkv(w: torch.Tensor, n_heads: int) -> torch.Tensor:
    """[3D, K] q|k|v weight (nn.Linear rows q, k, v) -> rows in head-major 128-row groups q_h, k_h, v_h
    (ospo_decode_qkv_heads' W_hm before tile_decode_weight)."""
    N, K = w.shape
    if N != 3 * n_heads * 128:
        raise ValueError(f"head_major_qkv: {N} rows is not 3 x {n_heads} heads x 128")
    return w.view(3, n_heads, 128, K).permute(1, 0, 2, 3).reshape(N, K).contiguous()


def decode_qkv_heads(x: torch.Tensor, w_hm: torch.Tensor, q_out: torch.Tensor, ws: torch.Tensor, *, norm, kv,
                     h0: int, nh: int) -> torch.Tensor:
    """decode_linear(x, w, q_out, ws, epi="kv", norm=norm, kv=kv) for heads h0 .. h0 + nh - 1 only
    (ospo_decode_qkv_heads): w_hm = tile_decode_weight(head_major_qkv(w))."""
    _chk(x, BF16, "x")
    _chk(q_out, BF16, "q_out")
    R, D = x.shape
    ss_in, ln_w, eps = norm
    pos, (cs, sn), kc, vc, H, Tmax = kv
    call("ospo_decode_qkv_heads", _p(w_hm), _p(x), _ld(x), R, D, _p(ss_in), ss_in.numel() // 32, _p(ln_w), float(eps),
         _p(q_out), _ld(q_out), _p(pos), _p(cs), _p(sn), _p(kc), _p(vc), H, int(h0), int(nh), Tmax, _p(ws),
         ws.numel() * 4, _s())
    return q_out


def attn_cache_heads(q, k_cache, v_cache, R, nq, n_heads, Tmax, start, pos, scale, out, h0: int, nh: int):
    """attn_cache for heads h0 .. h0 + nh - 1 (ospo_attn_cache_heads)."""
    call("ospo_attn_cache_heads", _p(q), _ld(q), _p(k_cache), _p(v_cache), int(R), int(nq), int(n_heads), int(h0),
         int(nh), int(Tmax), _p(start), _p(pos), float(scale), _p(out), _ld(out), _s())
    return out


def decode_mlp(xmid: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor, h: torch.Tensor, out: torch.Tensor,
               ws: torch.Tensor, *, norm, ss_out, step, layer: int, flags: torch.Tensor, tmo: torch.Tensor) -> bool:
    """The decode MLP in one launch (ospo_decode_mlp, round 5): decode_linear(xmid, w_gu, h, epi="swiglu",
    norm=norm) then decode_linear(h, w_down, out, residual=xmid, ss_out=ss_out), bit for bit.  w_gu from
    interleave_gate_up + tile_decode_weight, w_down tiled; step: the device decode-step counter (int32 [1]);
    flags: int32 [>= 2F / 128], zero before the first use of each (step, layer); tmo: int32 [1] (nonzero after a
    wait that gave up).  Returns False (nothing launched) when the shapes do not map onto the one-launch form."""
    for t, nme in ((xmid, "xmid"), (h, "h"), (out, "out")):
        _chk(t, BF16, nme)
    R, D = xmid.shape
    F = h.shape[1]
    ss_in, ln_w, eps = norm
    for t, nme in ((flags, "flags"), (tmo, "tmo"), (step, "step")):
        if t.dtype != torch.int32 or not t.is_contiguous():
            raise ValueError(f"decode_mlp: {nme} must be contiguous int32")
    if flags.numel() < 2 * F // 128:
        raise ValueError("decode_mlp: flags needs 2F / 128 words")
    rc = getattr(_lib.lib(), "ospo_decode_mlp")(
        _p(w_gu), _p(w_down), _p(xmid), _ld(xmid), R, D, F, _p(ss_in), ss_in.numel() // 32, _p(ln_w), float(eps),
        _p(h), _ld(h), _p(out), _ld(out), _p(ss_out), _p(step), int(layer), _p(flags), _p(tmo), _p(ws),
        ws.numel() * 4, _s())
    if rc == 4:  # OSPO_ERR_UNSUPPORTED: the caller runs the two launches
        return False
    if rc != 0:
        raise ValueError(f"ospo_decode_mlp: {_lib.lib().ospo_strerror(rc).decode()} (status {rc})")
    return True


def decode_attn_o(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, R: int, n_heads: int, Tmax: int,
                  start: torch.Tensor, pos: torch.Tensor, scale: float, attn_out: torch.Tensor, w_o: torch.Tensor,
                  residual: torch.Tensor, out: torch.Tensor, ss_out: torch.Tensor, ws: torch.Tensor, *, step,
                  layer: int, flags: torch.Tensor, tmo: torch.Tensor) -> bool:
    """The cached attention and the o projection in one launch (ospo_decode_attn_o, round 5): attn_cache(q, ...,
    attn_out) then decode_linear(attn_out, w_o, out, residual=residual, ss_out=ss_out), bit for bit.  flags: int32
    [>= 2 * n_heads] (per-head flags, then tickets), zero before the first call; tmo: int32 [1].  Returns False (nothing
    launched) when the o split plan does not map onto the one-launch form."""
    for t, nme in ((q, "q"), (attn_out, "attn_out"), (residual, "residual"), (out, "out")):
        _chk(t, BF16, nme)
    for t, nme in ((flags, "flags"), (tmo, "tmo"), (step, "step"), (start, "start"), (pos, "pos")):
        if t.dtype != torch.int32 or not t.is_contiguous():
            raise ValueError(f"decode_attn_o: {nme} must be contiguous int32")
    if flags.numel() < 2 * n_heads:
        raise ValueError("decode_attn_o: flags needs 2 * n_heads words")
    rc = getattr(_lib.lib(), "ospo_decode_attn_o")(
        _p(q), _ld(q), _p(k_cache), _p(v_cache), int(R), int(n_heads), int(Tmax), _p(start), _p(pos), float(scale),
        _p(attn_out), _ld(attn_out), _p(w_o), _p(residual), _ld(residual), _p(out), _ld(out), _p(ss_out), _p(step),
        int(layer), _p(flags), _p(tmo), _p(ws), ws.numel() * 4, _s())
    if rc == 4:  # OSPO_ERR_UNSUPPORTED: the caller runs the two launches
        return False
    if rc != 0:
        raise ValueError(f"ospo_decode_attn_o: {_lib.lib().ospo_strerror(rc).decode()} (status {rc})")
    return True


def interleave_gate_up(gu: torch.Tensor) -> torch.Tensor:
    """[gate; up] rows [2F, K] -> the order ospo_decode_linear's swiglu epilogue reads: 128-row group g =
    gate rows 64g .. 64g+63, then up rows F + 64g .. (F % 64 == 0)."""
    N, K = gu.shape
    F = N // 2
    if N % 128:
        raise ValueError(f"interleave_gate_up: 2F = {N} must be a multiple of 128")
    return gu.view(2, F // 64, 64, K).permute(1, 0, 2, 3).reshape(N, K).contiguous()


def decode_linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, ws: torch.Tensor, *, epi: str = "plain",
                  norm=None, bias=None, gelu: bool = False, residual=None, ss_out=None, kv=None) -> torch.Tensor:
    """One decode-step Linear in one launch (ospo_decode_linear): w tiled (tile_decode_weight);
    norm = (ss_in [G, 32] fp32, ln_w, eps) folds the RMSNorm of x into the staging; epi "plain" (bias,
    gelu, residual, ss_out [N/128, 32]), "kv" (kv = (pos_dev, (cos, sin), k_cache, v_cache, n_heads,
    Tmax); out = q) or "swiglu" (w from interleave_gate_up; out = h [R, N/2])."""
    for t, nme in ((x, "x"), (w, "w"), (out, "out")):
        _chk(t, BF16, nme)
    R, K = x.shape
    N, Kw, ldw = _decode_w(w)
    if ldw != 0 or Kw != K:
        raise ValueError(f"decode_linear needs a tiled weight with K = {K}, got {tuple(w.shape)}")
    ss_in, ln_w, eps = norm if norm is not None else (None, None, 0.0)
    if ss_in is not None and (ss_in.dtype != torch.float32 or not ss_in.is_contiguous()):
        raise ValueError("decode_linear: ss_in must be contiguous fp32 [groups, 32]")
    if ss_out is not None and (ss_out.dtype != torch.float32 or ss_out.numel() < N // 128 * 32):
        raise ValueError("decode_linear: ss_out must be fp32 with N/128 x 32 entries")
    pos = cs = sn = kc = vc = None
    H = Tmax = 0
    if kv is not None:
        pos, (cs, sn), kc, vc, H, Tmax = kv
    call("ospo_decode_linear", _p(w), _p(x), _ld(x), R, N, K, _p(ss_in), 0 if ss_in is None else ss_in.numel() // 32,
         _p(ln_w), float(eps), DL_EPI[epi], _p(bias), int(gelu), _p(residual),
         _ld(residual) if residual is not None else 0, _p(out), _ld(out), _p(ss_out), _p(pos), _p(cs), _p(sn), _p(kc),
         _p(vc), H, Tmax, _p(ws), ws.numel() * 4, _s())
    return out


def decode_gemv_fusable(R: int, N: int, K: int) -> bool:
    return bool(query("ospo_decode_gemv_fusable", R, N, K))


def decode_gemv_kv(x, w, ws, pos_dev, rope, k_cache, v_cache, n_heads, Tmax, q_out):
    """q|k|v = x . w^T then RoPE + KV store (ospo_decode_gemv_kv; == decode_gemv + kv_store)."""
    _chk(x, BF16, "x")
    _chk(w, BF16, "w")
    R, K = x.shape
    N, Kw, ldw = _decode_w(w)
    if Kw != K or N != 3 * n_heads * 128:
        raise ValueError(f"decode_gemv_kv shape mismatch x{tuple(x.shape)} w{tuple(w.shape)}")
    cos, sin = rope
    call("ospo_decode_gemv_kv", _p(w), ldw, _p(x), _ld(x), R, n_heads, 128, K, _p(ws), ws.numel() * 4,
         _p(pos_dev), _p(cos), _p(sin), _p(k_cache), _p(v_cache), Tmax, _p(q_out), _ld(q_out), _s())


def decode_gemv_swiglu(x, w, ws, h):
    """h = swiglu(x . w^T), w = [gate; up] (ospo_decode_gemv_swiglu; == decode_gemv + swiglu_fwd)."""
    _chk(x, BF16, "x")
    _chk(w, BF16, "w")
    _chk(h, BF16, "h")
    R, K = x.shape
    N, Kw, ldw = _decode_w(w)
    F = N // 2
    if Kw != K or h.shape[0] < R or h.shape[1] != F:
        raise ValueError(f"decode_gemv_swiglu: h{tuple(h.shape)} w{tuple(w.shape)} for R={R}, F={F}")
    call("ospo_decode_gemv_swiglu", _p(w), ldw, _p(x), _ld(x), R, F, K, _p(ws), ws.numel() * 4, _p(h), _ld(h),
         _s())
    return h


def kv_store(qkv, R, nq, pos_dev, k_cache, v_cache, n_heads, Tmax, *, rope=None, q_out=None):
    cos, sin = rope if rope is not None else (None, None)
    call("ospo_kv_store", _p(qkv), _ld(qkv), R, nq, _p(pos_dev), int(rope is not None), _p(cos), _p(sin), _p(k_cache),
         _p(v_cache), n_heads, 128, Tmax, _p(q_out), _ld(q_out) if q_out is not None else 0, _s())


def attn_cache(q, k_cache, v_cache, R, nq, n_heads, Tmax, start, pos_dev, scale, out):
    call("ospo_attn_cache", _p(q), _ld(q), _p(k_cache), _p(v_cache), R, nq, n_heads, 128, Tmax, _p(start),
         _p(pos_dev), float(scale), _p(out), _ld(out), _s())
    return out


def cfg_sample(logits, B, cfg_weight, temperature, u, step_dev, n_steps, tokens, next_ids, probs_out=None):
    V = logits.shape[1]
    call("ospo_cfg_sample", _p(logits), _ld(logits), V, B, float(cfg_weight), float(temperature), _p(u), _p(step_dev),
         n_steps, _p(tokens), _p(next_ids), _p(probs_out), _s())


def embed_rows(ids, table, out):
    call("ospo_embed_rows", _p(ids), ids.numel(), _p(table), table.shape[0], table.shape[1], _p(out), _s())
    return out


def decode_advance(pos_dev, step_dev):
    call("ospo_decode_advance", _p(pos_dev), _p(step_dev), _s())
