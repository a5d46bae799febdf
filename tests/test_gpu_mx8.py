"""MXFP8 variant (BASELINE config 5) on the MI355X, through the C ABI: the quantizer is
bit-exact against oracle/mx8_ref.py (elements AND the scale bytes in the tile layout), and the
block-scaled MFMA GEMM equals the fp32 product of the dequantized operands (exactly on
integer-valued data, to bf16 rounding otherwise), with every epilogue the bf16 GEMM has."""
import pytest
import torch

from oracle import mx8_ref as MX

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from ospo_amd import _lib
    _lib.lib()
    torch.manual_seed(0)


def ops():
    from ospo_amd import ops as _ops
    return _ops


def rnd(*shape, s=1.0):
    return (torch.randn(*shape, device=DEV) * s).to(torch.bfloat16)


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def wild(M, K):
    """bf16 data over many binades, with all-zero, tiny (subnormal-scale) and huge blocks."""
    x = torch.randn(M, K, device=DEV) * torch.exp2(torch.randint(-20, 12, (M, 1), device=DEV).float())
    x[0, :32] = 0.0
    if M > 1:
        x[1, 32:64] = 1e-38
        x[1, 64:96] = 3e38
    if M > 2:
        x[2, :] = torch.tensor(448.0 * 1.0625)  # mantissa above 1.75: the round-up scale
    return x.to(torch.bfloat16)


def spread(M, K):
    """finite bf16 data over many binades (rows scaled 2^-20..2^6), one all-zero block."""
    x = torch.randn(M, K, device=DEV) * torch.exp2(torch.randint(-20, 7, (M, 1), device=DEV).float())
    x[0, :32] = 0.0
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,K", [(1, 128), (300, 512), (4800, 4096), (257, 11008)])
def test_quant_mx8_bit_exact(M, K):
    x = wild(M, K)
    t = ops().MX8(M, K, DEV)
    t.s.fill_(0xAB)  # the padding rows must come back as 0
    ops().quant_mx8(x, t)
    q_ref, s_ref = MX.quantize_mx8(x.cpu())
    assert torch.equal(t.q.cpu(), q_ref)
    assert torch.equal(t.s.cpu(), MX.scale_tile_layout(s_ref))


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 512, 512), (4800, 4096, 4096), (100, 768, 11008)])
def test_gemm_mx8_exact_integers(M, N, K):
    """Small integers quantize exactly (|x| <= 3 -> 384, 256, 128 x 2^-7) and the sums are exact."""
    a = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
    b = torch.randint(-3, 4, (N, K), device=DEV).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt_mx8(ops().MX8.of(a), ops().MX8.of(b), out)
    ref = (a.float() @ b.float().T).to(torch.bfloat16)
    assert torch.equal(out, ref), (out.float() - ref.float()).abs().max()


def test_gemm_mx8_asymmetric_identity():
    M = N = K = 256
    a = torch.eye(M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.arange(N * K, device=DEV).reshape(N, K).remainder(17).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt_mx8(ops().MX8.of(a), ops().MX8.of(b), out)
    assert torch.equal(out, b.T.contiguous())


@pytest.mark.parametrize("M,N,K,K2", [(600, 512, 256, 64), (4800, 4096, 4096, 64), (777, 256, 1024, 128),
                                      (4800, 12288, 4096, 64)])
def test_gemm_mx8_vs_dequantized(M, N, K, K2):
    """Random data: equals bf16(alpha*(deq(a).deq(b)^T + a2.b2^T) + bias) + residual to bf16 rounding."""
    a, b = rnd(M, K), rnd(N, K, s=0.05)
    a2, b2 = rnd(M, K2), rnd(N, K2, s=0.05)
    bias, res = rnd(N), rnd(M, N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt_mx8(ops().MX8.of(a), ops().MX8.of(b), out, a2=a2, b2=b2, alpha=0.5, bias=bias, residual=res)
    fa = MX.fake_quant(a.cpu()).to(DEV)
    fb = MX.fake_quant(b.cpu()).to(DEV)
    acc = 0.5 * (fa @ fb.T + a2.float() @ b2.float().T) + bias.float()
    ref = (acc.to(torch.bfloat16).float() + res.float()).to(torch.bfloat16)
    d = (out.float() - ref.float()).abs()
    # one bf16 rounding of each of the two sums (the residual add can cancel), plus the block-scaled
    # MFMA's inner product, which is not exact fp32: up to 2^-12 of sum|a_k b_k| per instruction on
    # random e4m3 codes (tools/mx8_probe.hip), ~6e-6 on Gaussian data (tools/mx8_diag.py)
    absum = 0.5 * (fa.abs() @ fb.abs().T + a2.float().abs() @ b2.float().abs().T)
    tol = (acc.abs() + res.float().abs() + ref.float().abs()) * 2.0 ** -8 + absum * 2.0 ** -10
    assert bool((d <= tol).all()), float((d / tol).max())
    assert relerr(out.float(), ref.float()) < 2e-3  # ~ the bf16 output rounding alone
    # and the fp8 product is a ~1e-2-accurate approximation of the bf16 one (sanity on the scales)
    exact = 0.5 * (a.float() @ b.float().T + a2.float() @ b2.float().T) + bias.float() + res.float()
    assert relerr(out.float(), exact) < 6e-2


@pytest.mark.parametrize("M,H,T", [(600, 4, 600), (1200, 2, 600)])
def test_gemm_mx8_rope_fused_equals_unfused(M, H, T):
    D = H * 128
    x, w = rnd(M, 512), rnd(3 * D, 512, s=0.05)
    a2, b2 = rnd(M, 64), rnd(3 * D, 64, s=0.05)
    cos, sin = ops().rope_tables(T, 128, 10000.0, DEV)
    xa, wb = ops().MX8.of(x), ops().MX8.of(w)
    fused = torch.empty(M, 3 * D, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt_mx8(xa, wb, fused, a2=a2, b2=b2, rope=(cos, sin, T, 2 * D))
    sep = torch.empty_like(fused)
    ops().gemm_nt_mx8(xa, wb, sep, a2=a2, b2=b2)
    ops().rope(sep, 0, D, M // T, T, H, 128, cos, sin)
    assert torch.equal(fused, sep)


@pytest.mark.parametrize("M,N,K,K2", [(300, 512, 256, 64), (4800, 4096, 4096, 64), (600, 1024, 512, 128)])
def test_gemm_mx8_dropout_backward(M, N, K, K2):
    from ospo_amd import dropout as Dm
    p, seed = 0.05, 998877
    a, b = rnd(M, K), rnd(N, K, s=0.05)
    a2, b2 = rnd(M, K2), rnd(N, K2, s=0.05)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt_mx8(ops().MX8.of(a), ops().MX8.of(b), out, a2=a2, b2=b2, dropout=(seed, p))
    keep = torch.from_numpy(Dm.keep_mask(M, N, seed, p)).to(DEV)
    fa = MX.fake_quant(a.cpu()).to(DEV)
    fb = MX.fake_quant(b.cpu()).to(DEV)
    ref = fa @ fb.T + keep.float() / (1 - p) * (a2.float() @ b2.float().T)
    assert relerr(out.float(), ref) < 4e-3


def test_gemm_mx8_rejects_bad_shapes():
    from ospo_amd._lib import call
    a = ops().MX8.of(rnd(64, 256))
    b = ops().MX8.of(rnd(256, 256))
    out = torch.empty(64, 256, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(ValueError):  # K % 128
        call("ospo_gemm_nt_mx8", a.q.data_ptr(), 256, a.s.data_ptr(), b.q.data_ptr(), 256, b.s.data_ptr(), 64, 256,
             200, None, 0, None, 0, 0, 1.0, None, None, 0, out.data_ptr(), 256, None, None, 0, 0, 0, 0.0, 0, None, 0,
             None)
    with pytest.raises(ValueError):  # MX8 operand K mismatch
        ops().gemm_nt_mx8(a, ops().MX8.of(rnd(256, 384)), out)


def test_gemm_mx8_split_tail_rope_equals_unsplit():
    """MX8 rope GEMM with a forced split-K tail (RoPE applied in the fixup) == the unsplit kernel, on
    codes whose products are exact (power-of-two scales, small integers)."""
    M, H, T, K = 4800, 10, 600, 2048  # 19 x 15 = 285 tiles: 29 in the tail round, 17 K-tiles
    D = H * 128
    x = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
    w = torch.randint(-1, 2, (3 * D, K), device=DEV).to(torch.bfloat16)
    a2 = torch.randint(-3, 4, (M, 64), device=DEV).to(torch.bfloat16)
    b2 = torch.randint(-1, 2, (3 * D, 64), device=DEV).to(torch.bfloat16)
    cos, sin = ops().rope_tables(T, 128, 10000.0, DEV)
    xa, wb = ops().MX8.of(x), ops().MX8.of(w)
    outs = []
    for s in (1, 3):  # 1: no split
        o = torch.empty(M, 3 * D, device=DEV, dtype=torch.bfloat16)
        ops().gemm_nt_mx8(xa, wb, o, a2=a2, b2=b2, rope=(cos, sin, T, 2 * D), split=s)
        outs.append(o)
    assert ops().gemm_ws_bytes(M, 3 * D, K, 64, mx=True, split=3) == 29 * 3 * 65536 * 4  # the split really ran
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,D", [(1, 128), (300, 512), (4800, 4096)])
@pytest.mark.parametrize("bwd", [False, True])
def test_rmsnorm_mx8_output_equals_quantized_output(M, D, bwd):
    """The fp8 step's fused producers: rmsnorm fwd/bwd with an MXFP8 copy of their bf16 output ==
    the plain kernel's output, and the copy == quant_mx8 of it, byte for byte (elements + scales)."""
    x, w = spread(M, D), rnd(D)
    rstd = torch.empty(M, device=DEV)
    y = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    ops().rmsnorm_fwd(x, w, y, rstd, 1e-6)
    if bwd:
        dy, dres = rnd(M, D), rnd(M, D, s=0.5)
        ref = torch.empty_like(y)
        ops().rmsnorm_bwd(dy, x, w, rstd, ref, dres=dres)
        fused, mx = torch.empty_like(y), ops().MX8(M, D, DEV)
        ops().rmsnorm_bwd(dy, x, w, rstd, fused, dres=dres, mx=mx)
    else:
        ref = y
        fused, mx = torch.empty_like(y), ops().MX8(M, D, DEV)
        ops().rmsnorm_fwd(x, w, fused, torch.empty_like(rstd), 1e-6, mx=mx)
    assert torch.equal(fused, ref)
    q = ops().quant_mx8(ref, ops().MX8(M, D, DEV))
    assert mx.m == M
    assert torch.equal(mx.q[:M], q.q[:M])
    assert torch.equal(mx.s, q.s)


@pytest.mark.parametrize("M,F", [(1, 128), (257, 11008), (4800, 1024)])
@pytest.mark.parametrize("bwd", [False, True])
def test_swiglu_mx8_output_equals_quantized_output(M, F, bwd):
    gu = spread(M, 2 * F)
    if bwd:
        dh = rnd(M, F)
        ref = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
        ops().swiglu_bwd(dh, gu, ref)
        fused, mx = torch.empty_like(ref), ops().MX8(M, 2 * F, DEV)
        ops().swiglu_bwd(dh, gu, fused, mx=mx)
    else:
        ref = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
        ops().swiglu_fwd(gu, ref)
        fused, mx = torch.empty_like(ref), ops().MX8(M, F, DEV)
        ops().swiglu_fwd(gu, fused, mx=mx)
    assert torch.equal(fused, ref)
    q = ops().quant_mx8(ref, ops().MX8(M, ref.shape[1], DEV))
    assert torch.equal(mx.q[:M], q.q[:M])
    assert torch.equal(mx.s, q.s)


def test_mx8_producers_reject_bad_targets():
    x, w = rnd(64, 256), rnd(256)
    rstd = torch.empty(64, device=DEV)
    y = torch.empty_like(x)
    with pytest.raises(ValueError):  # K mismatch
        ops().rmsnorm_fwd(x, w, y, rstd, 1e-6, mx=ops().MX8(64, 384, DEV))
    with pytest.raises(ValueError):  # too few rows
        ops().rmsnorm_fwd(x, w, y, rstd, 1e-6, mx=ops().MX8(32, 256, DEV))


@pytest.mark.parametrize("S,T,H", [(2, 200, 4), (8, 600, 2)])
def test_flash_attention_mx8_outputs_equal_quantized_outputs(S, T, H):
    """Config 5: attention forward / backward with an MXFP8 copy of their stores (the o_proj and the q|k|v
    dX GEMM operands) write the plain kernels' bf16 outputs, and the copies == quant_mx8 of them, byte for
    byte (elements + scales); the backward with the fused RoPE as in the step."""
    import math
    hd = 128
    D = H * hd
    M = S * T
    qkv = rnd(M, 3 * D)
    cos, sin = ops().rope_tables(T, hd, 1e4, DEV)
    scale = 1 / math.sqrt(hd)
    o_ref, o = (torch.zeros(M, D, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    lse = torch.empty(S * H * T, device=DEV)
    ops().flash_attn_fwd(qkv, 0, D, 2 * D, o_ref, lse, S, T, H, hd, scale)
    mx = ops().MX8(M, D, DEV)
    ops().flash_attn_fwd(qkv, 0, D, 2 * D, o, torch.empty_like(lse), S, T, H, hd, scale, mx=mx)
    assert torch.equal(o, o_ref)
    q = ops().quant_mx8(o_ref, ops().MX8(M, D, DEV))
    assert mx.m == M and torch.equal(mx.q[:M], q.q[:M]) and torch.equal(mx.s, q.s)
    do = rnd(M, D)
    delta = torch.empty(S * H * T, device=DEV)
    dsw = ops().flash_attn_bwd_ws(S, T, H, DEV)
    g_ref, g = (torch.zeros(M, 3 * D, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    ops().flash_attn_bwd(qkv, 0, D, 2 * D, o_ref, do, lse, delta, dsw, g_ref, S, T, H, hd, scale,
                         rope_cos=cos, rope_sin=sin)
    mx3 = ops().MX8(M, 3 * D, DEV)
    ops().flash_attn_bwd(qkv, 0, D, 2 * D, o_ref, do, lse, delta, dsw, g, S, T, H, hd, scale,
                         rope_cos=cos, rope_sin=sin, mx=mx3)
    assert torch.equal(g, g_ref)
    q3 = ops().quant_mx8(g_ref, ops().MX8(M, 3 * D, DEV))
    assert torch.equal(mx3.q[:M], q3.q[:M]) and torch.equal(mx3.s, q3.s)
    with pytest.raises(RuntimeError):  # the MXFP8 copy needs the 5-product (dS workspace) kernels
        ops().flash_attn_bwd(qkv, 0, D, 2 * D, o_ref, do, lse, delta, None, g, S, T, H, hd, scale, mx=mx3)
