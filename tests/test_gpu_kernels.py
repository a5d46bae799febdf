"""Per-kernel numerics on the MI355X: each HIP kernel (through the C ABI) against
a plain PyTorch fp32 reference of the same op (or the oracle where it defines
the op).  Integer-valued operands are used where the result must be exact."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import simpo_ref as O

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


def bf(x):
    return x.to(torch.bfloat16)


def rnd(*shape, s=1.0):
    return (torch.randn(*shape, device=DEV) * s).to(torch.bfloat16)


def ints(*shape, lo=-3, hi=4):
    return torch.randint(lo, hi, shape, device=DEV).to(torch.bfloat16)


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


# ------------------------------------------------------------------ GEMM NT
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 256, 128), (4800, 512, 256), (160, 1024, 192),
                                   (64, 64, 64), (100, 192, 128)])
def test_gemm_nt_exact_integers(M, N, K):
    a, b = ints(M, K), ints(N, K)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, out)
    ref = a.float() @ b.float().T  # |ref| <= 9*K*... small ints, exactly representable
    ref_bf = bf(ref).float()
    assert torch.equal(out.float(), ref_bf), (out.float() - ref_bf).abs().max()


@pytest.mark.parametrize("M,N,K,K2,split", [(4800, 4096, 4096, 64, 0), (4800, 4096, 4096, 64, 3),
                                            (1000, 2048, 1024, 128, 2), (777, 1280, 320, 64, 0),
                                            (4608, 4096, 2048, 0, 4)])
def test_gemm_nt_schedule_exact_integers_long_k(M, N, K, K2, split):
    """The default 256x256 schedule over many K-tiles (steady loop), the LoRA extension tiles after the main
    ones, ragged M and split-K tails (workgroups whose K-range starts mid-way): exact on small integers."""
    a, b = ints(M, K, lo=-2, hi=3), ints(N, K, lo=-2, hi=3)
    a2 = ints(M, K2) if K2 else None
    b2 = ints(N, K2) if K2 else None
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, out, a2=a2, b2=b2, split=split)
    # the pinned splits really ran: tail tiles (tiles - 256) x split partial tiles
    tail = {(4800, 3): 48, (4608, 4): 32}.get((M, split), 0)
    assert ops().gemm_ws_bytes(M, N, K, K2, split=split) == tail * split * 65536 * 4 or split in (0, 1)
    ref = a.double() @ b.double().T + (a2.double() @ b2.double().T if K2 else 0)
    assert torch.equal(out.float(), bf(ref.float()).float()), (out.float() - ref.float()).abs().max()


def test_gemm_nt_asymmetric_identity():
    """A = I-like selector with an asymmetric B catches a transposed C write."""
    M = N = K = 256
    a = torch.eye(M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.arange(N * K, device=DEV).reshape(N, K).remainder(251).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, out)
    assert torch.equal(out, b.T.contiguous())


@pytest.mark.parametrize("M,N,K,K2", [(600, 512, 256, 64), (4800, 1024, 512, 64), (777, 256, 128, 128)])
def test_gemm_nt_lora_bias_residual(M, N, K, K2):
    a, b = rnd(M, K), rnd(N, K, s=0.05)
    a2, b2 = rnd(M, K2), rnd(N, K2, s=0.05)
    bias, res = rnd(N), rnd(M, N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, out, a2=a2, b2=b2, alpha=0.5, bias=bias, residual=res)
    acc = 0.5 * (a.float() @ b.float().T + a2.float() @ b2.float().T) + bias.float()
    ref = bf(bf(acc).float() + res.float()).float()
    assert relerr(out.float(), ref) < 4e-3


def test_gemm_nt_rejects_bad_shapes():
    a, b = rnd(64, 96), rnd(64, 96)
    out = torch.empty(64, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        ops().gemm_nt(a, b, out)  # K % 64 != 0


# --------------------------------------------------------------- GEMM f32acc
@pytest.mark.parametrize("a_k,b_k,M,N,K,splits", [
    (False, False, 4800, 64, 256, 4),    # u = x . A^T
    (False, True, 600, 64, 512, 3),      # g = dy . B
    (True, True, 64, 512, 640, 5),       # dA = g^T x
    (True, True, 1024, 64, 640, 4),      # dB = dy^T u
    (True, True, 128, 128, 256, 1),
    (True, True, 128, 4096, 1280, 12),  # 64 x 256 tiles (grid >= 384)
    (True, True, 4096, 64, 640, 8),     # 256 x 64 tiles
    (True, True, 256, 1024, 640, 8),    # 64 x 64 fallback
])
def test_gemm_f32acc_layouts(a_k, b_k, M, N, K, splits):
    A = ints(K, M) if a_k else ints(M, K)
    B = ints(K, N) if b_k else ints(N, K)
    Aop = A.float().T if a_k else A.float()
    Bop = B.float().T if b_k else B.float()
    out = torch.full((M, N), 0.5, device=DEV, dtype=torch.float32)
    ops().gemm_f32acc(A, B, out, a_kmajor=a_k, b_kmajor=b_k, k_splits=splits, alpha=2.0)
    ref = 0.5 + 2.0 * (Aop @ Bop.T)
    assert torch.equal(out, ref), (out - ref).abs().max()


def test_gemm_f32acc_dA_used_rows_of_padded_g():
    """dA = g[:, :used]^T x with g padded to Rp = 64 columns: only the used rows are written."""
    K, Rp, used, N = 4800, 64, 48, 4096
    g = ints(K, Rp)
    x = ints(K, N)
    out = torch.full((used + 1, N), 7.0, device=DEV, dtype=torch.float32)
    ops().gemm_f32acc(g[:, :used], x, out[:used], a_kmajor=True, b_kmajor=True, k_splits=8)
    ref = 7.0 + g[:, :used].float().T @ x.float()
    assert torch.equal(out[:used], ref)
    assert torch.all(out[used] == 7.0)


@pytest.mark.parametrize("K,N,used,splits", [(4800, 4096, 48, 1), (4800, 4096, 48, 8), (4800, 11008, 16, 4),
                                              (640, 256, 32, 1)])
def test_gemm_f32acc_dropout_recompute_equals_stored_mask(K, N, used, splits):
    """dA with the LoRA dropout mask recomputed on the staged activations == dA on the masked copy
    the forward's skinny product writes (the same bf16 values, the same accumulation): bit-exact."""
    p, seed = 0.05, 987654
    x = rnd(K, N)
    g = rnd(K, 64)
    xd = torch.empty_like(x)
    u = torch.empty(K, 64, device=DEV, dtype=torch.bfloat16)
    A = torch.zeros(64, N, device=DEV, dtype=torch.bfloat16)
    ops().lora_skinny(x, A, u, K, K, N, 1, 0, 1.0, b_rows=16, dropout=(seed, p), xd=xd)
    ref = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().gemm_f32acc(g[:, :used], xd, ref, a_kmajor=True, b_kmajor=True, k_splits=splits)
    out = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().gemm_f32acc(g[:, :used], x, out, a_kmajor=True, b_kmajor=True, k_splits=splits, b_dropout=(seed, p))
    if splits == 1:
        assert torch.equal(out, ref)
    else:  # the K-split partials meet in fp32 atomics, in no fixed order
        assert relerr(out, ref) < 1e-6


@pytest.mark.parametrize("K,N,used,splits,M", [(4800, 4096, 48, 8, 4800), (4800, 11008, 16, 4, 4744),
                                                (640, 256, 32, 1, 600)])
def test_gemm_f32acc_dropout_keep_bits_equal_rehash(K, N, used, splits, M):
    """dA's tile product with the mask read from the forward's keep bits == re-hashed: bit-exact with one
    split, reassociation-close with atomics; rows >= M (zero g) contribute nothing whatever their bits."""
    p, seed = 0.05, 24680
    x = rnd(K, N)
    g = rnd(K, 64)
    g[M:] = 0
    bits = torch.full((K * N // 8,), 0xFF, device=DEV, dtype=torch.uint8)
    ops().lora_skinny(x, torch.zeros(64, N, device=DEV, dtype=torch.bfloat16),
                      torch.empty(K, 64, device=DEV, dtype=torch.bfloat16), M, K, N, 1, 0, 1.0, b_rows=16,
                      dropout=(seed, p), keep_bits=bits)
    for sp in (1, splits):
        ref = torch.zeros(used, N, device=DEV, dtype=torch.float32)
        ops().gemm_f32acc(g[:, :used], x, ref, a_kmajor=True, b_kmajor=True, k_splits=sp, b_dropout=(seed, p))
        out = torch.zeros(used, N, device=DEV, dtype=torch.float32)
        ops().gemm_f32acc(g[:, :used], x, out, a_kmajor=True, b_kmajor=True, k_splits=sp, b_dropout=(seed, p),
                          keep_bits=bits)
        if sp == 1:
            assert torch.equal(out, ref)
        else:
            assert relerr(out, ref) < 1e-6


def test_gemm_f32acc_blockdiag_scatter():
    """dB of a packed q|k|v LoRA: keep only the diagonal blocks, peft layout."""
    r, nblk, nm = 16, 256, 3
    M = 320
    dy = ints(M, nm * nblk)
    u = ints(M, 64)
    out = torch.zeros(nm * nblk * r, device=DEV, dtype=torch.float32)
    ops().gemm_f32acc(dy, u, out.view(nm * nblk, r), a_kmajor=True, b_kmajor=True, k_splits=2, diag=(nblk, r))
    full = dy.float().T @ u.float()  # [nm*nblk, 64]
    ref = torch.cat([full[i * nblk:(i + 1) * nblk, i * r:(i + 1) * r] for i in range(nm)], 0).reshape(-1)
    assert torch.equal(out, ref)


# ------------------------------------------------------------------ RMSNorm
@pytest.mark.parametrize("M,D", [(37, 256), (600, 4096), (5, 2048)])
def test_rmsnorm(M, D):
    x, w = rnd(M, D), bf(1 + 0.1 * torch.randn(D, device=DEV))
    y = torch.empty_like(x)
    rstd = torch.empty(M, device=DEV)
    ops().rmsnorm_fwd(x, w, y, rstd, 1e-6)
    ref = O.rmsnorm(x, w, 1e-6)
    assert relerr(y.float(), ref.float()) < 4e-3
    # backward vs fp32 autograd
    dy, dres = rnd(M, D), rnd(M, D)
    xf = x.float().requires_grad_(True)
    yf = w.float() * (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6))
    yf.backward(dy.float())
    dx = torch.empty_like(x)
    ops().rmsnorm_bwd(dy, x, w, rstd, dx, dres=dres)
    assert relerr(dx.float(), xf.grad + dres.float()) < 4e-3


# --------------------------------------------------------------------- RoPE
@pytest.mark.parametrize("M,H,T", [(2 * 72, 2, 72), (300, 4, 150), (4800, 8, 600)])
def test_gemm_rope_fused_equals_unfused(M, H, T):
    """ospo_gemm_nt_rope_bf16 == gemm_nt then ospo_rope_fwd, bit for bit (same rounding points)."""
    hd, K = 128, 512
    D = H * hd
    N = 3 * D if (3 * D) % 256 == 0 else 4 * D
    a, b = rnd(M, K), rnd(N, K, s=0.05)
    a2, b2 = rnd(M, 64), rnd(N, 64, s=0.05)
    cos, sin = ops().rope_tables(T, hd, 1e4, DEV)
    ref = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, ref, a2=a2, b2=b2)
    ops().rope(ref, 0, D, M // T, T, H, hd, cos, sin)
    out = torch.empty_like(ref)
    ops().gemm_nt(a, b, out, a2=a2, b2=b2, rope=(cos, sin, T, 2 * D))
    assert torch.equal(out, ref)


def test_gemm_rope_half_tile():
    """rope_cols = 128 mod 256 (H = 3, q heads only): the last RoPE tile rotates one head and copies
    the other; checked against a torch statement of HF's rounding points."""
    M, H, T, hd, K = 300, 3, 150, 128, 256
    D = H * hd
    N = 4 * D
    a, b = rnd(M, K), rnd(N, K, s=0.05)
    cos, sin = ops().rope_tables(T, hd, 1e4, DEV)
    plain = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, plain)
    out = torch.empty_like(plain)
    ops().gemm_nt(a, b, out, rope=(cos, sin, T, D))
    assert torch.equal(out[:, D:], plain[:, D:])
    t = torch.arange(M, device=DEV) % T
    c, s_ = cos[t].float()[:, None, :], sin[t].float()[:, None, :]  # [M, 1, 64]
    x = plain[:, :D].float().view(M, H, hd)
    x1, x2 = x[..., :64], x[..., 64:]
    bf = lambda z: z.bfloat16().float()
    lo = (bf(x1 * c) + bf(-x2 * s_)).bfloat16()
    hi = (bf(x2 * c) + bf(x1 * s_)).bfloat16()
    assert torch.equal(out[:, :D].view(M, H, hd), torch.cat([lo, hi], -1))


def test_rope_fwd_bwd():
    S, T, H, hd = 2, 72, 3, 128
    D = H * hd
    qkv = rnd(S * T + 5, 3 * D)
    cos, sin = ops().rope_tables(T, hd, 1e4, DEV)
    x = qkv.clone()
    ops().rope(x, 0, D, S, T, H, hd, cos, sin)
    c, s = O.rope_cos_sin(T, hd, 1e4, torch.bfloat16)
    c, s = c.to(DEV), s.to(DEV)
    for col in (0, D):
        src = qkv[: S * T, col:col + D].view(S, T, H, hd).transpose(1, 2)
        ref = O.apply_rope(src, c, s).transpose(1, 2).reshape(S * T, D)
        assert torch.equal(x[: S * T, col:col + D], ref)
    assert torch.equal(x[:, 2 * D:], qkv[:, 2 * D:])  # v untouched
    assert torch.equal(x[S * T:], qkv[S * T:])        # pad rows untouched
    # bwd: transpose rotation (fp32 autograd reference)
    g = rnd(S * T, 3 * D)
    src = qkv[: S * T, :D].float().view(S, T, H, hd).transpose(1, 2).requires_grad_(True)
    out = O.apply_rope(src, c.float(), s.float())
    out.backward(g[:, :D].float().view(S, T, H, hd).transpose(1, 2))
    gx = g.clone()
    ops().rope(gx, 0, D, S, T, H, hd, cos, sin, backward=True)
    ref = src.grad.transpose(1, 2).reshape(S * T, D)
    assert relerr(gx[:, :D].float(), ref) < 4e-3


# ------------------------------------------------------------------- SwiGLU
def test_swiglu():
    M, Fd = 333, 512
    gu = rnd(M, 2 * Fd)
    h = torch.empty(M, Fd, device=DEV, dtype=torch.bfloat16)
    ops().swiglu_fwd(gu, h)
    ref = F.silu(gu[:, :Fd]) * gu[:, Fd:]
    assert relerr(h.float(), ref.float()) < 2e-3
    assert (h != ref).float().mean().item() < 0.01
    dh = rnd(M, Fd)
    g = gu.float().requires_grad_(True)
    (F.silu(g[:, :Fd]) * g[:, Fd:]).backward(dh.float())
    dgu = torch.empty_like(gu)
    ops().swiglu_bwd(dh, gu, dgu)
    assert relerr(dgu.float(), g.grad) < 5e-3


# ---------------------------------------------------------------- attention
def bf16_scores(q, k, scale):
    """The kernels' attention scores: (q.k^T) * scale in fp32.  Until round 5 they restated HF eager bf16,
    bf16(bf16(q.k^T) * scale); round 6 keeps the scores fp32, so the fp32 product is the
    reference here (the oracle's bf16 path keeps HF's roundings; the step tests bound the difference)."""
    return (q @ k.transpose(-1, -2)) * scale


def attn_ref(q, k, v, scale):
    T = q.shape[-2]
    s = bf16_scores(q, k, scale)
    s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.softmax(s, -1) @ v


@pytest.mark.parametrize("ws", [True, False], ids=["ds5", "recompute7"])
@pytest.mark.parametrize("S,T,H", [(2, 72, 2), (1, 64, 1), (2, 600, 2), (1, 130, 3), (1, 520, 2)])
def test_flash_attention(S, T, H, ws):
    hd = 128
    D = H * hd
    rows = S * T + 7
    qkv = rnd(rows, 3 * D)
    o = torch.zeros(rows, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(S * H * T, device=DEV)
    scale = 1 / math.sqrt(hd)
    ops().flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, scale)
    qf = qkv[: S * T].float().view(S, T, 3, H, hd).permute(2, 0, 3, 1, 4).requires_grad_(True)
    ref = attn_ref(qf[0], qf[1], qf[2], scale)
    ref_rows = ref.transpose(1, 2).reshape(S * T, D)
    assert relerr(o[: S * T].float(), ref_rows) < 8e-3
    s_ = bf16_scores(qf[0], qf[1], scale)
    s_ = s_.masked_fill(torch.ones(T, T, dtype=torch.bool, device=DEV).triu(1), float("-inf"))
    assert relerr(lse.view(S, H, T), torch.logsumexp(s_, -1)) < 1e-4
    # backward
    do = rnd(rows, D)
    ref.backward(do[: S * T].float().view(S, T, H, hd).transpose(1, 2))
    dqkv = torch.zeros(rows, 3 * D, device=DEV, dtype=torch.bfloat16)
    delta = torch.empty(S * H * T, device=DEV)
    dsw = ops().flash_attn_bwd_ws(S, T, H, DEV) if ws else None
    if dsw is not None:
        dsw.fill_(float("nan"))  # dQ must not read any dS^T entry the dK/dV kernel did not write
    ops().flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, dsw, dqkv, S, T, H, hd, scale)
    g = qf.grad.permute(1, 3, 0, 2, 4).reshape(S * T, 3 * D)
    for i, nm in enumerate("qkv"):
        e = relerr(dqkv[: S * T, i * D:(i + 1) * D].float(), g[:, i * D:(i + 1) * D])
        assert e < 2e-2, (nm, e)


@pytest.mark.parametrize("ws", [True, False], ids=["ds5", "recompute7"])
@pytest.mark.parametrize("S,T,H", [(2, 130, 2), (1, 600, 1)])
def test_flash_attention_bwd_fused_rope(S, T, H, ws):
    """dq/dk with the RoPE backward fused into the stores == the unfused chain
    (attention bwd, then ospo_rope_bwd), and both track fp32 autograd through
    rope -> attention w.r.t. the PRE-RoPE q, k."""
    hd = 128
    D = H * hd
    rows = S * T + 3
    pre = rnd(rows, 3 * D)
    cos, sin = ops().rope_tables(T, hd, 1e4, DEV)
    qkv = pre.clone()
    ops().rope(qkv, 0, D, S, T, H, hd, cos, sin)
    o = torch.zeros(rows, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(S * H * T, device=DEV)
    scale = 1 / math.sqrt(hd)
    ops().flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, scale)
    do = rnd(rows, D)
    delta = torch.empty(S * H * T, device=DEV)
    fused = torch.zeros(rows, 3 * D, device=DEV, dtype=torch.bfloat16)
    dsw = ops().flash_attn_bwd_ws(S, T, H, DEV) if ws else None
    ops().flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, dsw, fused, S, T, H, hd, scale,
                         rope_cos=cos, rope_sin=sin)
    plain = torch.zeros(rows, 3 * D, device=DEV, dtype=torch.bfloat16)
    ops().flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, dsw, plain, S, T, H, hd, scale)
    ops().rope(plain, 0, D, S, T, H, hd, cos, sin, backward=True)
    assert relerr(fused[: S * T].float(), plain[: S * T].float()) < 8e-3
    assert torch.equal(fused[: S * T, 2 * D:], plain[: S * T, 2 * D:])  # dv untouched by RoPE
    # fp32 autograd through rope -> attention (scores rounded like the kernel)
    c, s_ = O.rope_cos_sin(T, hd, 1e4, torch.bfloat16)
    c, s_ = c.to(DEV).float(), s_.to(DEV).float()
    src = pre[: S * T].float().view(S, T, 3, H, hd).permute(2, 0, 3, 1, 4).requires_grad_(True)
    q = O.apply_rope(src[0], c, s_)
    k = O.apply_rope(src[1], c, s_)
    ref = attn_ref(q, k, src[2], scale)
    ref.backward(do[: S * T].float().view(S, T, H, hd).transpose(1, 2))
    g = src.grad.permute(1, 3, 0, 2, 4).reshape(S * T, 3 * D)
    for i, nm in enumerate("qkv"):
        e = relerr(fused[: S * T, i * D:(i + 1) * D].float(), g[:, i * D:(i + 1) * D])
        assert e < 2e-2, (nm, e)


# ------------------------------------------------------- embed / gather / gelu
def test_assemble_and_aligner():
    B, Lt, N, D, V = 2, 5, 8, 256, 50
    ids = torch.tensor([[3, 4, 5, -1, -1], [7, 8, 9, 10, 11]], device=DEV, dtype=torch.int32)
    table = rnd(V, D)
    img = rnd(2 * B * N, D)
    x0 = torch.empty(2 * B * (Lt + N), D, device=DEV, dtype=torch.bfloat16)
    ops().assemble_inputs(ids, B, Lt, table, img, N, D, x0)
    T = Lt + N
    for s in range(2 * B):
        for t in range(T):
            row = x0[s * T + t]
            if t < Lt:
                i = int(ids[s % B, t])
                exp = table[i] if i >= 0 else torch.zeros_like(row)
            else:
                exp = img[s * N + t - Lt]
            assert torch.equal(row, exp)
    E = 8
    gid = torch.randint(0, 100, (37,), device=DEV, dtype=torch.int32)
    emb, w1, b1 = rnd(100, E), rnd(D, E, s=0.3), rnd(D, s=0.1)
    out = torch.empty(37, D, device=DEV, dtype=torch.bfloat16)
    ops().gen_aligner_in(gid, emb, w1, b1, out)
    ref = F.gelu(F.linear(emb[gid.long()].float(), w1.float(), b1.float()))
    assert relerr(out.float(), ref) < 4e-3
    # the vectorised E = 8 kernel against the scalar one (reached through an unaligned output view):
    # same per-output arithmetic, so bit-identical
    big = torch.empty(37 * D + 1, device=DEV, dtype=torch.bfloat16)
    out_s = big[1:].view(37, D)
    ops().gen_aligner_in(gid, emb, w1, b1, out_s)
    assert torch.equal(out, out_s)


def test_gather_scatter_gelu():
    S, T, t0, N, D = 3, 20, 4, 15, 64
    src = rnd(S * T + 3, D)
    dst = torch.empty(S * N, D, device=DEV, dtype=torch.bfloat16)
    ops().gather_rows(src, S, T, t0, N, dst)
    ref = src[: S * T].view(S, T, D)[:, t0:t0 + N].reshape(S * N, D)
    assert torch.equal(dst, ref)
    back = torch.full((S * T + 3, D), 7.0, device=DEV, dtype=torch.bfloat16)
    ops().scatter_rows(dst, S, T, t0, N, back)
    exp = torch.zeros_like(back)
    exp[: S * T].view(S, T, D)[:, t0:t0 + N] = dst.view(S, N, D)
    assert torch.equal(back, exp)
    x = rnd(1000 * 8)
    y = torch.empty_like(x)
    ops().gelu_fwd(x, y)
    assert relerr(y.float(), F.gelu(x.float())) < 4e-3
    dy = rnd(1000 * 8)
    dx = torch.empty_like(x)
    ops().gelu_bwd(dy, x, dx)
    xf = x.float().requires_grad_(True)
    F.gelu(xf).backward(dy.float())
    assert relerr(dx.float(), xf.grad) < 4e-3


# ------------------------------------------------------------ logprob / SimPO
def test_logprob_fwd_bwd():
    S, N, V = 4, 24, 16384
    logits = rnd(S * N, V, s=2.0)
    labels = torch.randint(0, V, (S * N,), device=DEV, dtype=torch.int32)
    lse = torch.empty(S * N, device=DEV)
    tok = torch.empty(S * N, device=DEV)
    seq = torch.empty(S, device=DEV)
    ops().logprob_fwd(logits, labels, N, lse, tok, seq)
    lf = logits.float().requires_grad_(True)
    lp = torch.gather(lf.log_softmax(-1), 1, labels.long()[:, None])[:, 0]
    ref_seq = lp.view(S, N).mean(-1)
    assert relerr(seq, ref_seq) < 1e-5
    g = torch.randn(S, device=DEV)
    ref_seq.backward(g)
    dl = torch.empty_like(logits)
    ops().logprob_bwd(logits, labels, lse, N, g, dl)
    assert relerr(dl.float(), lf.grad) < 4e-3


@pytest.mark.parametrize("beta,gbr,ls,lt", [(10.0, 0.5, 0.0, "sigmoid"), (2.0, 0.0, 0.1, "sigmoid"),
                                            (10.0, 0.5, 0.0, "hinge")])
def test_simpo(beta, gbr, ls, lt):
    B = 5
    lp = (torch.randn(2 * B, device=DEV) * 0.3 - 9.7).requires_grad_(True)
    losses, cr, rr = O.simpo_loss(lp[:B], lp[B:], beta, gbr, ls, lt)
    losses.mean().backward()
    lo, mean, rew, glp = (torch.empty(B, device=DEV), torch.empty(1, device=DEV), torch.empty(2 * B, device=DEV),
                          torch.empty(2 * B, device=DEV))
    ops().simpo_fwd(lp.detach(), B, beta, gbr, ls, lt, lo, mean, rew)
    ops().simpo_bwd(lp.detach(), B, beta, gbr, ls, lt, torch.ones(1, device=DEV), glp)
    torch.testing.assert_close(lo, losses.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(mean[0], losses.mean().detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rew, torch.cat([cr, rr]), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(glp, lp.grad, rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        ops().simpo_fwd(lp.detach(), B, beta, gbr, ls, "ipo", lo, mean, rew)


# ---------------------------------------------------------------- LoRA pack
def test_lora_pack():
    nm, r, Kin, Nmod, Rp = 3, 16, 256, 128, 64
    A = rnd(nm * r, Kin)
    Bf = rnd(nm, Nmod, r)
    Acat = torch.empty(Rp, Kin, device=DEV, dtype=torch.bfloat16)
    AcatT = torch.empty(Kin, Rp, device=DEV, dtype=torch.bfloat16)
    Bcat = torch.empty(nm * Nmod, Rp, device=DEV, dtype=torch.bfloat16)
    BT = torch.empty(nm * r, Nmod, device=DEV, dtype=torch.bfloat16)
    ops().lora_pack(A, Bf, nm, r, Kin, Nmod, Rp, Acat, AcatT, Bcat, BT)
    expA = torch.zeros(Rp, Kin, device=DEV, dtype=torch.bfloat16)
    expA[: nm * r] = A
    assert torch.equal(Acat, expA) and torch.equal(AcatT, expA.T)
    expB = torch.zeros(nm * Nmod, Rp, device=DEV, dtype=torch.bfloat16)
    for i in range(nm):
        expB[i * Nmod:(i + 1) * Nmod, i * r:(i + 1) * r] = Bf[i]
    assert torch.equal(Bcat, expB)
    assert torch.equal(BT, torch.cat([Bf[i].T for i in range(nm)], 0))
    # two layers in one launch: sources at a layer stride in a flat buffer, outputs [L][...]
    na, nb = nm * r * Kin, nm * Nmod * r
    stride = na + nb + 40
    flat = torch.zeros(2 * stride, device=DEV, dtype=torch.bfloat16)
    A2, B2 = rnd(nm * r, Kin), rnd(nm, Nmod, r)
    for l, (a_, b_) in enumerate(((A, Bf), (A2, B2))):
        flat[l * stride: l * stride + na] = a_.reshape(-1)
        flat[l * stride + na: l * stride + na + nb] = b_.reshape(-1)
    Ac2 = torch.empty(2, Rp, Kin, device=DEV, dtype=torch.bfloat16)
    AT2 = torch.empty(2, Kin, Rp, device=DEV, dtype=torch.bfloat16)
    Bc2 = torch.empty(2, nm * Nmod, Rp, device=DEV, dtype=torch.bfloat16)
    BT2 = torch.empty(2, nm * r, Nmod, device=DEV, dtype=torch.bfloat16)
    ops().lora_pack(flat, flat[na:], nm, r, Kin, Nmod, Rp, Ac2, AT2, Bc2, BT2, n_layers=2, layer_stride=stride)
    assert torch.equal(Ac2[0], Acat) and torch.equal(AT2[0], AcatT) and torch.equal(Bc2[0], Bcat)
    assert torch.equal(BT2[0], BT)
    assert torch.equal(Ac2[1, : nm * r], A2) and torch.equal(BT2[1], torch.cat([B2[i].T for i in range(nm)], 0))


@pytest.mark.parametrize("pad", [40, 41], ids=["vector8", "scalar"])
def test_lora_pack_r8_paths(pad):
    """r = 8 over 4 modules, 3 layers: the 16-B kernel (layer stride a multiple of 8 elements) and the
    element-wise fallback (odd stride) give the same exact copies."""
    nm, r, Kin, Nmod, Rp, L = 4, 8, 128, 64, 32, 3
    na, nb = nm * r * Kin, nm * Nmod * r
    stride = na + nb + pad
    flat = torch.zeros(L * stride + 8, device=DEV, dtype=torch.bfloat16)
    As, Bs = [rnd(nm * r, Kin) for _ in range(L)], [rnd(nm, Nmod, r) for _ in range(L)]
    for l in range(L):
        flat[l * stride: l * stride + na] = As[l].reshape(-1)
        flat[l * stride + na: l * stride + na + nb] = Bs[l].reshape(-1)
    Ac = torch.empty(L, Rp, Kin, device=DEV, dtype=torch.bfloat16)
    AT = torch.empty(L, Kin, Rp, device=DEV, dtype=torch.bfloat16)
    Bc = torch.empty(L, nm * Nmod, Rp, device=DEV, dtype=torch.bfloat16)
    BT = torch.empty(L, nm * r, Nmod, device=DEV, dtype=torch.bfloat16)
    ops().lora_pack(flat, flat[na:], nm, r, Kin, Nmod, Rp, Ac, AT, Bc, BT, n_layers=L, layer_stride=stride)
    for l in range(L):
        assert torch.equal(Ac[l], As[l]) and torch.equal(AT[l], As[l].T)
        expB = torch.zeros(nm * Nmod, Rp, device=DEV, dtype=torch.bfloat16)
        for i in range(nm):
            expB[i * Nmod:(i + 1) * Nmod, i * r:(i + 1) * r] = Bs[l][i]
        assert torch.equal(Bc[l], expB)
        assert torch.equal(BT[l], torch.cat([Bs[l][i].T for i in range(nm)], 0))


@pytest.mark.parametrize("M,K,used", [(4800, 4096, 48), (300, 11008, 16), (77, 512, 32), (1, 256, 64),
                                      (600, 4096, 96)])
def test_lora_skinny_down(M, K, used):
    """u = s x A_cat^T: dense mode, partial n-tiles, rows M..M_out-1 and pad columns zeroed
    (96 used of Rp = 128: LoRA r = 32 on q|k|v, 6 n-tiles in two chunks)."""
    Rp = 64 if used <= 64 else 128
    x = rnd(M + 5, K)
    Acat = torch.zeros(Rp, K, device=DEV, dtype=torch.bfloat16)
    Acat[:used] = rnd(used, K)
    M_out = (M + 63) // 64 * 64
    out = torch.full((M_out + 3, Rp), 7.0, device=DEV, dtype=torch.bfloat16)
    nt = (used + 15) // 16
    ws = ops().lora_skinny_ws(M_out, K, nt)
    ref = 2.0 * (x[:M].float() @ Acat.float().T)
    for rep in range(2):  # second call reuses the workspace
        ops().lora_skinny(x, Acat, out, M, M_out, K, nt, 0, 2.0, b_rows=used, ws=ws)
        assert relerr(out[:M].float(), ref) < 8e-3
        assert torch.all(out[M:M_out] == 0) and torch.all(out[:M, 16 * nt:] == 0)
        assert torch.all(out[M_out:] == 7.0)


@pytest.mark.parametrize("M,K,used", [(600, 4096, 48), (77, 11008, 16)])
def test_lora_skinny_dropout(M, K, used):
    """u = s dropout(x) A^T with the counter-based mask; xd = dropout(x) stored for the backward."""
    import numpy as np
    from ospo_amd import dropout as Dm
    p, seed = 0.05, 123457
    Rp = 64
    x = rnd(M, K)
    Acat = torch.zeros(Rp, K, device=DEV, dtype=torch.bfloat16)
    Acat[:used] = rnd(used, K)
    out = torch.empty(M, Rp, device=DEV, dtype=torch.bfloat16)
    xd = torch.full((M, K), 3.0, device=DEV, dtype=torch.bfloat16)
    ops().lora_skinny(x, Acat, out, M, M, K, (used + 15) // 16, 0, 2.0, b_rows=used, dropout=(seed, p), xd=xd)
    keep = torch.from_numpy(Dm.keep_mask(M, K, seed, p)).to(DEV)
    ref_xd = torch.where(keep, (x.float() / (1 - p)).to(torch.bfloat16), torch.zeros((), dtype=torch.bfloat16,
                                                                                           device=DEV))
    assert torch.equal(xd, ref_xd)
    ref = 2.0 * (ref_xd.float() @ Acat.float().T)
    assert relerr(out.float(), ref) < 8e-3


def test_lora_skinny_split_sum_in_launch_leaves_counters_zero():
    """The u product's split sum runs in the launch (last arriver per row block, write-through partials): the
    same ws serves calls of different shapes back to back, results are deterministic, and the row-block
    counters at the ws head are zero after every call (the next call's precondition)."""
    ws = ops().lora_skinny_ws(4864, 11008, 8, DEV)
    outs = []
    for M, K, used in [(4800, 4096, 48), (4800, 11008, 16), (4800, 4096, 48), (600, 4096, 32), (4800, 4096, 48)]:
        torch.manual_seed(K + used)
        x = rnd(M, K)
        A = torch.zeros(64, K, device=DEV, dtype=torch.bfloat16)
        A[:used] = rnd(used, K, s=0.05)
        M_out = (M + 63) // 64 * 64
        out = torch.full((M_out, 64), 7.0, device=DEV, dtype=torch.bfloat16)
        ops().lora_skinny(x, A, out, M, M_out, K, (used + 15) // 16, 0, 2.0, b_rows=used, ws=ws)
        torch.cuda.synchronize()
        assert torch.all(ws[:1024] == 0), "row-block counters not reset"
        ref = 2.0 * (x.float() @ A[:used].float().T)
        assert relerr(out[:M, :used].float(), ref) < 8e-3
        assert torch.all(out[M:] == 0) and torch.all(out[:M, 16 * ((used + 15) // 16):] == 0)
        outs.append(out.clone())
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[0], outs[4])


@pytest.mark.parametrize("M,K,used", [(4800, 4096, 48), (4800, 11008, 16), (130, 4096, 32), (600, 4096, 96)])
def test_lora_skinny_dropout_streamed(M, K, used):
    """The step's form (no masked copy requested): the LDS-line streaming kernel masks x in registers."""
    from ospo_amd import dropout as Dm
    p, seed = 0.05, 424243
    Rp = 64 if used <= 64 else 128
    x = rnd(M, K)
    Acat = torch.zeros(Rp, K, device=DEV, dtype=torch.bfloat16)
    Acat[:used] = rnd(used, K, s=0.05)
    M_out = (M + 63) // 64 * 64
    out = torch.full((M_out, Rp), 7.0, device=DEV, dtype=torch.bfloat16)
    bits = torch.full((M_out * K // 8,), 0x5A, device=DEV, dtype=torch.uint8)
    ops().lora_skinny(x, Acat, out, M, M_out, K, (used + 15) // 16, 0, 2.0, b_rows=used, dropout=(seed, p),
                      keep_bits=bits)
    keep = torch.from_numpy(Dm.keep_mask(M, K, seed, p)).to(DEV)
    xd = torch.where(keep, (x.float() / (1 - p)).to(torch.bfloat16), torch.zeros((), dtype=torch.bfloat16, device=DEV))
    ref = 2.0 * (xd.float() @ Acat.float().T)
    assert relerr(out[:M].float(), ref) < 8e-3
    assert torch.all(out[M:] == 0) and torch.all(out[:M, 16 * ((used + 15) // 16):] == 0)
    # the keep-bit output: bit k % 8 of byte (m K + k) / 8 == the mask, rows >= M untouched
    got = ((bits[: M * K // 8].view(M, K // 8).to(torch.int32).unsqueeze(-1) >> torch.arange(8, device=DEV)) & 1)
    assert torch.equal(got.view(M, K).bool(), keep)
    assert torch.all(bits[M * K // 8:] == 0x5A)


@pytest.mark.parametrize("M,M_out,F,used,drop", [(4800, 4800, 11008, 16, True), (4744, 4800, 11008, 16, True),
                                                   (600, 640, 1024, 32, False), (130, 192, 512, 48, True)])
def test_swiglu_fwd_lora_down_equals_two_launches(M, M_out, F, used, drop):
    """SwiGLU forward fused with the down adapter's u product == swiglu_fwd then lora_skinny on h: h, u and
    the keep bits bit-identical (the same roundings, the same split-K partials and sums)."""
    p, seed = 0.05, 8642
    gu = rnd(M_out, 2 * F)
    A = torch.zeros(64, F, device=DEV, dtype=torch.bfloat16)
    A[:used] = rnd(used, F, s=0.05)
    nt = (used + 15) // 16
    dr = (seed, p) if drop else None
    h_ref = torch.zeros(M_out, F, device=DEV, dtype=torch.bfloat16)
    ops().swiglu_fwd(gu[:M], h_ref[:M])
    u_ref = torch.full((M_out, 64), 7.0, device=DEV, dtype=torch.bfloat16)
    bits_ref = torch.zeros(M_out * F // 8, device=DEV, dtype=torch.uint8)
    ops().lora_skinny(h_ref, A, u_ref, M, M_out, F, nt, 0, 2.0, b_rows=used, dropout=dr,
                      keep_bits=bits_ref if drop else None)
    h = torch.zeros(M_out, F, device=DEV, dtype=torch.bfloat16)
    u = torch.full((M_out, 64), 7.0, device=DEV, dtype=torch.bfloat16)
    bits = torch.zeros_like(bits_ref)
    ops().swiglu_fwd_lora_down(gu, h, A, u, M, M_out, F, nt, 2.0, b_rows=used, dropout=dr,
                               keep_bits=bits if drop else None)
    assert torch.equal(h, h_ref)
    assert torch.equal(u, u_ref)
    assert torch.equal(bits, bits_ref)


@pytest.mark.parametrize("M,N,K,K2", [(300, 512, 256, 64), (4800, 4096, 4096, 64), (600, 1024, 512, 128)])
def test_gemm_dropout_backward(M, N, K, K2):
    """dX = dy.W + mask (.) (g.A) / (1-p): the K-extension is masked like the adapter input."""
    from ospo_amd import dropout as Dm
    p, seed = 0.05, 998877
    a, b = rnd(M, K), rnd(N, K, s=0.05)
    a2, b2 = rnd(M, K2), rnd(N, K2, s=0.05)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, out, a2=a2, b2=b2, dropout=(seed, p))
    keep = torch.from_numpy(Dm.keep_mask(M, N, seed, p)).to(DEV)
    ref = a.float() @ b.float().T + keep.float() / (1 - p) * (a2.float() @ b2.float().T)
    assert relerr(out.float(), ref) < 4e-3


@pytest.mark.parametrize("M,N,K,K2,split", [(4800, 4096, 4096, 64, 0), (4800, 11008, 4096, 64, 0),
                                             (1280, 3840, 4096, 64, 2), (300, 512, 256, 64, 1), (600, 1024, 512, 128, 0)])
def test_gemm_dropout_keep_bits_equal_rehash(M, N, K, K2, split):
    """The dX GEMM's dropout mask from the forward's keep bits (lora_skinny keep_bits, staged with tile 0)
    == the re-hashed mask: bit-identical outputs, split-K tails included (N % 128 == 0 shapes)."""
    p, seed = 0.05, 55221
    a, b = rnd(M, K), rnd(N, K, s=0.05)
    a2, b2 = rnd(M, K2), rnd(N, K2, s=0.05)
    # the keep bits of the [M, N] adapter input, as the forward's u product writes them
    x = rnd(M, N)
    bits = torch.zeros(M * N // 8, device=DEV, dtype=torch.uint8)
    u = torch.empty(M, 64, device=DEV, dtype=torch.bfloat16)
    ops().lora_skinny(x, torch.zeros(64, N, device=DEV, dtype=torch.bfloat16), u, M, M, N, 1, 0, 1.0, b_rows=16,
                      dropout=(seed, p), keep_bits=bits)
    ref = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, ref, a2=a2, b2=b2, dropout=(seed, p), split=split)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(a, b, out, a2=a2, b2=b2, dropout=(seed, p), split=split, keep_bits=bits)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("M,M_out,nm,Nmod", [(4800, 4800, 3, 4096), (4800, 4864, 2, 11008), (777, 832, 1, 4096),
                                            (100, 128, 1, 1024), (1000, 1024, 4, 512)])
def test_lora_gdb_exact_integers(M, M_out, nm, Nmod):
    """The fused g = s dy.B / dB += dy^T u stream: exact on small integers against the two products
    it replaces (block diagonal over the modules; rows >= M of u and dy ignored, g rows M.. zeroed)."""
    _lora_gdb_exact(M, M_out, nm, Nmod, 16)


@pytest.mark.parametrize("M,M_out,nm,Nmod", [(4800, 4864, 3, 4096), (4800, 4864, 1, 4096), (640, 704, 1, 11008),
                                            (1000, 1100, 2, 1024)])
def test_lora_gdb_rank32_exact_integers(M, M_out, nm, Nmod):
    """Round 6, LoRA r = 32 (ospo_lora_gdb_r: a module's 32 columns are two halves of 16 over the same dy
    columns, dB [nmods*Nmod, 32]): exact on small integers as the r = 16 form."""
    _lora_gdb_exact(M, M_out, nm, Nmod, 32)


def _lora_gdb_exact(M, M_out, nm, Nmod, r):
    dy = ints(M_out, nm * Nmod, lo=-2, hi=3)
    BT = ints(nm * r, Nmod, lo=-2, hi=3)
    Rp = 64 if nm * r <= 64 else 128
    u = ints(M_out, Rp, lo=-2, hi=3)
    u[M:] = 99.0  # rows past M must not contribute
    out = torch.full((M_out, Rp), 7.0, device=DEV, dtype=torch.bfloat16)
    dB = torch.ones(nm * Nmod, r, device=DEV, dtype=torch.float32)  # accumulates onto what is there
    ops().lora_gdb(dy, BT, u, out, dB, M, M_out, nm, Nmod, 1.0, r=r)
    dyd, Bd, ud = dy[:M].double(), BT.double(), u[:M].double()
    g_ref = torch.cat([dyd[:, j * Nmod:(j + 1) * Nmod] @ Bd[j * r:(j + 1) * r].T for j in range(nm)], 1)
    assert torch.equal(out[:M, : nm * r].float(), bf(g_ref.float()).float())
    assert torch.all(out[M:] == 0) and torch.all(out[:, nm * r:] == 0)
    dB_ref = torch.cat([dyd[:, j * Nmod:(j + 1) * Nmod].T @ ud[:, j * r:(j + 1) * r] for j in range(nm)], 0) + 1.0
    assert torch.equal(dB.double(), dB_ref)


@pytest.mark.parametrize("M,M_out,nm,Nmod", [(4800, 4864, 1, 4096), (4800, 4800, 3, 4096), (1000, 1100, 1, 1024),
                                            (130, 130, 2, 512)])
def test_lora_gdb_in_launch_sum(M, M_out, nm, Nmod):
    """Round 5 (the workspace's counter head; with OSPO_HIP_LIB = the ablation library and OSPO_GDB_INL=1 the
    in-launch partial sum): g exact on small integers (rows M .. M_out -- also past the last row block -- and pad
    columns zero), the same bits over repeated calls on one workspace, whose counter head is zero after every
    call (no wait gave up)."""
    r = 16
    dy = ints(M_out, nm * Nmod, lo=-2, hi=3)
    BT = ints(nm * r, Nmod, lo=-2, hi=3)
    Rp = 64 if nm * r <= 64 else 128
    u = ints(M_out, Rp, lo=-2, hi=3)
    ws = ops().lora_gdb_ws(M, nm, Nmod, DEV)
    dyd, Bd = dy[:M].double(), BT.double()
    g_ref = torch.cat([dyd[:, j * Nmod:(j + 1) * Nmod] @ Bd[j * r:(j + 1) * r].T for j in range(nm)], 1)
    first = None
    for it in range(3):
        out = torch.full((M_out, Rp), 7.0, device=DEV, dtype=torch.bfloat16)
        dB = torch.zeros(nm * Nmod, r, device=DEV, dtype=torch.float32)
        ops().lora_gdb(dy, BT, u, out, dB, M, M_out, nm, Nmod, 0.5, ws=ws)
        torch.cuda.synchronize()
        assert torch.all(ws[:2052] == 0), it  # the counters (and the give-up word) left zero
        assert torch.equal(out[:M, : nm * r].float(), bf(0.5 * g_ref.float()).float())
        assert torch.all(out[M:] == 0) and torch.all(out[:, nm * r:] == 0)
        first = out.clone() if first is None else first
        assert torch.equal(out, first)


@pytest.mark.parametrize("M,M_out,F", [(4800, 4800, 11008), (4800, 4864, 11008), (777, 832, 4096), (100, 128, 1024),
                                       (1000, 1024, 384), (64, 64, 128), (3001, 3008, 2816)])
def test_swiglu_lora_gdb_equals_two_launches(M, M_out, F):
    """ospo_swiglu_lora_gdb == ospo_swiglu_bwd then ospo_lora_gdb (nmods 2, Nmod F): dgu and g bit-equal (rows
    >= M of dgu untouched), dB equal up to the f32 atomics' order and against fp64."""
    _swiglu_lora_gdb_vs_two(M, M_out, F, 16)


@pytest.mark.parametrize("M,M_out,F", [(4800, 4864, 11008), (700, 768, 1024), (100, 128, 512)])
def test_swiglu_lora_gdb_rank32_equals_two_launches(M, M_out, F):
    """Round 6, LoRA r = 32 (ospo_swiglu_lora_gdb_r, 256-row workgroups with four halves' images): as the
    r = 16 form against ospo_swiglu_bwd + ospo_lora_gdb_r."""
    _swiglu_lora_gdb_vs_two(M, M_out, F, 32)


def _swiglu_lora_gdb_vs_two(M, M_out, F, r):
    dh, gu = rnd(M_out, F), rnd(M_out, 2 * F, s=3.0)
    BT, u = rnd(2 * r, F), rnd(M_out, 64)
    dgu_ref = torch.full((M_out, 2 * F), 5.0, device=DEV, dtype=torch.bfloat16)
    out_ref = torch.full((M_out, 64), 7.0, device=DEV, dtype=torch.bfloat16)
    dB_ref = torch.zeros(2 * F, r, device=DEV)
    ops().swiglu_bwd(dh[:M], gu[:M], dgu_ref[:M])
    ops().lora_gdb(dgu_ref, BT, u, out_ref, dB_ref, M, M_out, 2, F, 0.75, r=r)
    dgu = torch.full((M_out, 2 * F), 5.0, device=DEV, dtype=torch.bfloat16)
    out = torch.full((M_out, 64), 7.0, device=DEV, dtype=torch.bfloat16)
    dB = torch.zeros(2 * F, r, device=DEV)
    ops().swiglu_lora_gdb(dh, gu, dgu, BT, u, out, dB, M, M_out, 0.75, r=r)
    assert torch.equal(dgu, dgu_ref)
    assert torch.equal(out, out_ref)
    assert relerr(dB, dB_ref) < 1e-6
    # dB against fp64 dgu^T u over the kernel's own dgu (silu keeps dgu off the integers)
    u_i = ints(M_out, 64, lo=-2, hi=3)
    dB2 = torch.zeros(2 * F, r, device=DEV)
    ops().swiglu_lora_gdb(dh, gu, dgu, BT, u_i, out, dB2, M, M_out, 1.0, r=r)
    ref2 = torch.cat([dgu[:M, j * F:(j + 1) * F].double().T @ u_i[:M, j * r:(j + 1) * r].double() for j in range(2)])
    assert relerr(dB2.double(), ref2) < 1e-6


@pytest.mark.parametrize("M,nm,Nmod,r", [(4800, 3, 4096, 16), (640, 2, 11008, 16), (100, 1, 4096, 16),
                                         (300, 3, 1024, 32), (200, 2, 2048, 32)])
def test_lora_skinny_up_blockdiag(M, nm, Nmod, r):
    """g = s dy B over the block-diagonal B_cat, via per-module B^T (r / 16 n-tiles per module)."""
    Rp = (nm * r + 63) // 64 * 64
    dy = rnd(M, nm * Nmod)
    Bf = rnd(nm, Nmod, r)
    BT = torch.cat([Bf[i].T for i in range(nm)], 0).contiguous()
    out = torch.empty(M, Rp, device=DEV, dtype=torch.bfloat16)
    nt = nm * r // 16
    ops().lora_skinny(dy, BT, out, M, M, Nmod, nt, Nmod if nm > 1 else 0, 2.0, module_tiles=r // 16)
    ref = torch.cat([dy[:, i * Nmod:(i + 1) * Nmod].float() @ Bf[i].float() for i in range(nm)], 1) * 2.0
    assert relerr(out[:, : nm * r].float(), ref) < 8e-3
    assert torch.all(out[:, nm * r:] == 0)


# -------------------------------------------------------------- optimizer
def test_clip_adamw_matches_torch():
    n = 10000
    p0 = rnd(n, s=0.02)
    g = torch.randn(n, device=DEV) * 0.05
    ps = {"w": p0.cpu().clone()}
    state = {}
    O.clip_and_adamw(ps, {"w": g.cpu()}, state, lr=4e-5, betas=(0.9, 0.95), eps=1e-8, max_norm=1.0)
    O.clip_and_adamw(ps, {"w": (g * 0.5).cpu()}, state, lr=4e-5, betas=(0.9, 0.95), eps=1e-8, max_norm=1.0)
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    for step, gg in ((1, g), (2, g * 0.5)):
        ss = torch.zeros(1, device=DEV)
        ops().sumsq(gg, ss)
        assert abs(ss.item() - float((gg.double() ** 2).sum())) / float((gg.double() ** 2).sum()) < 1e-5
        ops().adamw_clip(p, gg, m, v, 4e-5, 0.9, 0.95, 1e-8, 0.0, step, ss, 1.0)
    ref = ps["w"].to(DEV)
    # within one bf16 ulp, or one AdamW step (the clip coefficient is computed from
    # fp32 grads here and from bf16 grads in torch, which can flip a rounding)
    tol = torch.maximum(ref.float().abs() * 2 ** -7 * 1.01, torch.full_like(ref.float(), 1.5 * 4e-5 * 2))
    assert bool(((p.float() - ref.float()).abs() <= tol).all())
    assert (p != ref).float().mean().item() < 0.02


def test_sumsq_deterministic():
    """The grad-norm sum is summed in a fixed order: repeated calls give the same bits (DP ranks holding the
    same all-reduced grads must clip by the same coefficient), within 1e-5 of the fp64 sum."""
    g = torch.randn(4_700_001, device=DEV) * 0.05
    outs = []
    for _ in range(4):
        ss = torch.zeros(1, device=DEV)
        ops().sumsq(g, ss)
        outs.append(ss.item())
    assert len(set(outs)) == 1, outs
    ref = float((g.double() ** 2).sum())
    assert abs(outs[0] - ref) / ref < 1e-5


@pytest.mark.parametrize("split", [2, 3, 4])
def test_gemm_split_tail_equals_unsplit(split):
    """Split-K tail tiles (partials + fixup, RoPE and residual epilogues applied in the fixup) give the
    same bf16 output as the unsplit kernel: exact integers so the fp32 partial order cannot matter."""
    M, H, T, K = 4800, 10, 600, 1024
    D = H * 128
    N = 3 * D                                     # 19 x 15 = 285 tiles: a tail round of 29 tiles
    a, b = ints(M, K), ints(N, K, lo=-1, hi=2)
    a2, b2 = ints(M, 64), ints(N, 64, lo=-1, hi=2)
    cos, sin = ops().rope_tables(T, 128, 1e4, DEV)
    res = ints(M, N)
    outs = {}
    for s in (1, split):  # 1: no split
        o1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops().gemm_nt(a, b, o1, a2=a2, b2=b2, rope=(cos, sin, T, 2 * D), split=s)
        o2 = torch.empty_like(o1)
        ops().gemm_nt(a, b, o2, a2=a2, b2=b2, residual=res, split=s)
        outs[s] = (o1, o2)
    assert ops().gemm_ws_bytes(M, N, K, 64, split=split) == 29 * split * 65536 * 4  # the split really ran
    ref = torch.empty_like(outs[1][1])
    ops().gemm_nt(a, b, ref, a2=a2, b2=b2)
    ops().rope(ref, 0, D, M // T, T, H, 128, cos, sin)
    assert torch.equal(outs[split][0], ref)
    assert torch.equal(outs[split][0], outs[1][0])
    assert torch.equal(outs[split][1], outs[1][1])


@pytest.mark.parametrize("M,F,K,K2,p,split", [(4800, 11008, 4096, 64, 0.05, 0), (600, 1024, 512, 64, 0.05, 2),
                                              (300, 512, 256, 0, 0.0, 0), (1000, 2048, 512, 128, 0.05, 3),
                                              (1000, 2048, 512, 64, 0.0, 2)])
def test_gemm_swiglu_bwd_fused_equals_two_launches(M, F, K, K2, p, split):
    """down_proj dX GEMM with the SwiGLU backward in its epilogue (dh never stored) is bit-identical to
    the dh GEMM (+ masked LoRA extension) followed by swiglu_bwd, on the same split-K decisions."""
    seed = 4242
    dy, w = rnd(M, K), rnd(F, K, s=0.05)
    a2 = rnd(M, K2) if K2 else None
    b2 = rnd(F, K2, s=0.05) if K2 else None
    gu = rnd(M, 2 * F, s=2.0)
    dr = (seed, p) if p > 0 else None
    dh = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt(dy, w, dh, a2=a2, b2=b2, dropout=dr, split=split)
    ref = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    ops().swiglu_bwd(dh, gu, ref)
    out = torch.full((M, 2 * F), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops().gemm_nt_swiglu_bwd(dy, w, gu, out, a2=a2, b2=b2, dropout=dr, split=split)
    assert torch.equal(out, ref)
    # and against an fp32 statement of the op (HF LlamaMLP: h = bf16(silu(g)) * u)
    g, u, d = gu[:, :F].float(), gu[:, F:].float(), dh.float()
    sg = torch.sigmoid(g)
    ref32 = torch.cat([bf(d * u).float() * sg * (1 + g * (1 - sg)), d * bf(g * sg).float()], 1)
    assert relerr(out.float(), ref32) < 1e-2


@pytest.mark.parametrize("S,T,H", [(2, 600, 4), (1, 200, 2)])
def test_flash_attention_bwd_5_product_form_equals_7(S, T, H):
    """The 5-product backward (dK/dV store dS^T, dQ = dS.K) against the 7-product one (dQ recomputes S
    and dP): all three outputs agree to fp32 summation order; dV is bit-identical while both forms run
    the same 16x16x32 dK / dV kernel (the default; the 32x32x16 attn_bwd_dkdv5_kernel, an ablation
    build option since round 6, agrees to 1.2e-4)."""
    hd = 128
    D = H * hd
    rows = S * T
    qkv = rnd(rows, 3 * D)
    o = torch.zeros(rows, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(S * H * T, device=DEV)
    scale = 1 / math.sqrt(hd)
    ops().flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, scale)
    do = rnd(rows, D)
    delta = torch.empty(S * H * T, device=DEV)
    a = torch.zeros(rows, 3 * D, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros_like(a)
    ops().flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, ops().flash_attn_bwd_ws(S, T, H, DEV), a, S, T, H, hd,
                         scale)
    ops().flash_attn_bwd(qkv, 0, D, 2 * D, o, do, lse, delta, None, b, S, T, H, hd, scale)
    for i in range(3):
        assert relerr(a[:, i * D:(i + 1) * D].float(), b[:, i * D:(i + 1) * D].float()) < 4e-3
    assert torch.equal(a[:, 2 * D:], b[:, 2 * D:])


@pytest.mark.parametrize("K,N,used,Rp,splits", [(4800, 4096, 48, 64, 8), (320, 11008, 16, 64, 2),
                                                (640, 4096, 96, 128, 3), (192, 256, 32, 64, 1)])
def test_lora_wgrad_da_exact_integers(K, N, used, Rp, splits):
    """dA = g^T x streamed over x (ospo_lora_wgrad mode 0): exact on integer operands (every product and
    partial sum is an integer below 2^24), all used rank rows, any split."""
    x = ints(K, N)
    g = ints(K, Rp)
    out = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().lora_wgrad(x, g, out, mode=0, s_cols=used, splits=splits)
    ref = g[:, :used].float().T @ x.float()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("nm,nmod,r,Rp,splits", [(3, 4096, 16, 64, 3), (2, 11008, 16, 64, 2), (1, 4096, 32, 64, 4),
                                                 (3, 256, 32, 128, 1)])
def test_lora_wgrad_db_blockdiag_exact_integers(nm, nmod, r, Rp, splits):
    """dB = dy^T u (mode 1): each module's dy columns against its own r columns of u, peft layout [N, r]."""
    K = 448
    dy = ints(K, nm * nmod)
    u = ints(K, Rp)
    out = torch.zeros(nm * nmod, r, device=DEV, dtype=torch.float32)
    ops().lora_wgrad(dy, u, out, mode=1, s_cols=nm * r, splits=splits, nmod=nmod, r=r)
    full = dy.float().T @ u.float()
    ref = torch.cat([full[i * nmod:(i + 1) * nmod, i * r:(i + 1) * r] for i in range(nm)], 0)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("K,N,used,Rp,splits", [(4800, 4096, 48, 64, 8), (4800, 11008, 16, 64, 4),
                                                (4800, 4096, 32, 64, 0), (640, 4096, 64, 128, 3),
                                                (192, 256, 33, 64, 1), (64, 128, 1, 64, 1)])
def test_lora_da_exact_integers(K, N, used, Rp, splits):
    """dA = g^T x as one stream over x (ospo_lora_da): exact on integer operands (every product and partial
    sum an integer below 2^24), all used rank rows and only those, any split, the step's group shapes."""
    x = ints(K, N)
    g = ints(K, Rp)
    out = torch.full((used + 1, N), 7.0, device=DEV, dtype=torch.float32)
    ops().lora_da(x, g, out, s_cols=used, splits=splits)
    ref = 7.0 + g[:, :used].float().T @ x.float()
    assert torch.equal(out[:used], ref)
    assert torch.all(out[used] == 7.0)


@pytest.mark.parametrize("K,N,used", [(640, 4096, 48), (4800, 11008, 16), (4800, 4096, 32)])
def test_lora_da_dropout_recompute_equals_stored_mask(K, N, used):
    """ospo_lora_da with dropout (x masked in registers by the forward's hash, one hash per pair of
    columns shared across partner lanes by DPP) == dA on the masked copy the forward skinny product writes:
    bit-exact with one split, fp32-reassociation close with atomics over several."""
    p, seed = 0.05, 4242
    x = rnd(K, N)
    g = rnd(K, 64)
    xd = torch.empty_like(x)
    u = torch.empty(K, 64, device=DEV, dtype=torch.bfloat16)
    A = torch.zeros(64, N, device=DEV, dtype=torch.bfloat16)
    ops().lora_skinny(x, A, u, K, K, N, 1, 0, 1.0, b_rows=16, dropout=(seed, p), xd=xd)
    ref = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().lora_da(xd, g, ref, s_cols=used, splits=1)
    out = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().lora_da(x, g, out, s_cols=used, splits=1, dropout=(seed, p))
    assert torch.equal(out, ref)
    out2 = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().lora_da(x, g, out2, s_cols=used, dropout=(seed, p))
    assert relerr(out2, ref) < 1e-6
    assert relerr(out, (g[:, :used].float().T @ xd.float())) < 1e-5


@pytest.mark.parametrize("K,N,used,M", [(4800, 4096, 48, 4800), (4800, 11008, 16, 4744), (640, 4096, 32, 600)])
def test_lora_da_keep_bits_equal_rehash(K, N, used, M):
    """dA masked by the forward's keep bits == dA re-hashing the mask: bit-exact with one split; rows >= M
    (no bits written, zero g) contribute nothing whatever their bits hold."""
    p, seed = 0.05, 777
    x = rnd(K, N)
    g = rnd(K, 64)
    g[M:] = 0
    A = torch.zeros(64, N, device=DEV, dtype=torch.bfloat16)
    u = torch.empty(K, 64, device=DEV, dtype=torch.bfloat16)
    bits = torch.full((K * N // 8,), 0xFF, device=DEV, dtype=torch.uint8)
    ops().lora_skinny(x, A, u, M, K, N, 1, 0, 1.0, b_rows=16, dropout=(seed, p), keep_bits=bits)
    ref = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().lora_da(x, g, ref, s_cols=used, splits=1, dropout=(seed, p))
    out = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().lora_da(x, g, out, s_cols=used, splits=1, dropout=(seed, p), keep_bits=bits)
    assert torch.equal(out, ref)
    out2 = torch.zeros(used, N, device=DEV, dtype=torch.float32)
    ops().lora_da(x, g, out2, s_cols=used, dropout=(seed, p), keep_bits=bits)
    assert relerr(out2, ref) < 1e-6


def test_lora_da_rejects_bad_shapes():
    from ospo_amd._lib import call
    x = torch.zeros(64, 256, device=DEV, dtype=torch.bfloat16)
    g = torch.zeros(64, 64, device=DEV, dtype=torch.bfloat16)
    out = torch.zeros(16, 256, device=DEV, dtype=torch.float32)
    P = lambda t: t.data_ptr()  # noqa: E731
    for args in [(256, 200, 64, 16, 64, 1),   # N % 128
                 (256, 256, 64, 16, 96, 1),   # K % 64
                 (256, 256, 48, 16, 64, 1),   # lds not 64 / 128
                 (256, 256, 64, 65, 64, 1),   # s_cols > 64
                 (256, 256, 64, 16, 64, 2)]:  # splits > K / 64
        ldx, N, lds, s_cols, K, splits = args
        with pytest.raises(ValueError):
            call("ospo_lora_da", P(x), ldx, N, P(g), lds, s_cols, K, P(out), 256, splits, 0, 0.0, None, None)
    with pytest.raises(ValueError):  # keep bits without dropout
        call("ospo_lora_da", P(x), 256, 256, P(g), 64, 16, 64, P(out), 256, 1, 0, 0.0, P(x), None)


def test_lora_wgrad_dropout_recompute_equals_stored_mask():
    """mode 0 with dropout: x masked in registers with the forward skinny product's hash and bf16 rounding
    == dA on the masked copy that product writes."""
    p, seed, K, N = 0.05, 4242, 640, 4096
    x = rnd(K, N)
    g = rnd(K, 64)
    xd = torch.empty_like(x)
    u = torch.empty(K, 64, device=DEV, dtype=torch.bfloat16)
    A = torch.zeros(64, N, device=DEV, dtype=torch.bfloat16)
    ops().lora_skinny(x, A, u, K, K, N, 1, 0, 1.0, b_rows=16, dropout=(seed, p), xd=xd)
    ref = torch.zeros(48, N, device=DEV, dtype=torch.float32)
    ops().lora_wgrad(xd, g, ref, mode=0, s_cols=48, splits=1)
    out = torch.zeros(48, N, device=DEV, dtype=torch.float32)
    ops().lora_wgrad(x, g, out, mode=0, s_cols=48, splits=1, dropout=(seed, p))
    assert torch.equal(out, ref)
    assert relerr(out, (g[:, :48].float().T @ xd.float())) < 1e-5



def test_gemm_clock_probe_product_and_stamps():
    """ospo_gemm_clock_probe_bf16 (bench.py's box probe): the w4 product unsplit, bit-exact on integer operands
    (every partial sum an integer below 2^24, one bf16 rounding as torch's fp32 product rounded), and its
    per-workgroup stamps ordered with an in-kernel clock in a plausible range (s_memtime ticks over
    s_memrealtime's 100 MHz)."""
    M = N = K = 512
    g = torch.Generator(device=DEV).manual_seed(5)
    a = torch.randint(-4, 5, (M, K), device=DEV, generator=g).bfloat16()
    b = torch.randint(-4, 5, (N, K), device=DEV, generator=g).bfloat16()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    stamps = torch.zeros((M // 256) * (N // 256), 8, dtype=torch.int64, device=DEV)
    ops().gemm_clock_probe(a, b, out, stamps)
    torch.cuda.synchronize()
    assert torch.equal(out, (a.float() @ b.float().T).bfloat16())
    st = stamps.cpu()
    assert bool((st[:, 4] >= st[:, 2]).all()) and bool((st[:, 3] > st[:, 0]).all())
    ghz = (st[:, 3] - st[:, 0]).double() / (st[:, 4] - st[:, 2]).clamp_min(1).double() * 0.1
    assert bool(((ghz > 0.3) & (ghz < 3.5)).all()), ghz.tolist()
