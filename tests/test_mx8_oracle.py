"""CPU checks of the MXFP8 oracle (oracle/mx8_ref.py) -- pins it against an independent
pure-Python statement of OCP e4m3 round-to-nearest-even and of the MX block rule."""
import math
import random

import pytest
import torch

from oracle import mx8_ref as MX


def e4m3_decode(b):
    s, e, m = b >> 7, (b >> 3) & 15, b & 7
    if e == 15 and m == 7:
        return math.nan
    v = (1 + m / 8) * 2.0 ** (e - 7) if e else (m / 8) * 2.0 ** -6
    return -v if s else v


_FINITE = [(b, e4m3_decode(b)) for b in range(256) if not math.isnan(e4m3_decode(b))]


def e4m3_rne(x):
    """Nearest finite e4m3fn of the same sign, ties to even mantissa (x already clamped to +-448)."""
    neg = math.copysign(1.0, x) < 0
    best, bd = None, math.inf
    for b, v in _FINITE:
        if (b >> 7) != int(neg):
            continue
        d = abs(v - x)
        if d < bd or (d == bd and b % 2 == 0):
            best, bd = b, d
    return best


def test_torch_e4m3_cast_is_rne():
    rng = random.Random(0)
    xs = [rng.uniform(-1, 1) * 2.0 ** rng.randint(-12, 8) for _ in range(3000)]
    for b, v in _FINITE:  # exact codes and midpoints (ties)
        xs.append(v)
        nxt = e4m3_decode(b + 1) if b + 1 < 256 else math.nan
        if not math.isnan(nxt) and (b & 0x7F) != 0x7E:
            xs.append((v + nxt) / 2)
    t = torch.tensor(xs, dtype=torch.float32)
    got = t.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8).tolist()
    want = [e4m3_rne(max(-448.0, min(448.0, float(x)))) for x in t.tolist()]
    assert got == want


def test_quantize_block_rule():
    torch.manual_seed(0)
    x = (torch.randn(8, 256) * torch.exp2(torch.randint(-30, 30, (8, 1)).float())).to(torch.bfloat16)
    x[0, :32] = 0
    q, s = MX.quantize_mx8(x)
    xf = x.float()
    for r in range(8):
        for blk in range(8):
            v = xf[r, 32 * blk: 32 * blk + 32]
            amax = float(v.abs().max())
            # smallest power of two X with amax / X <= 448
            want = 0 if amax == 0 else min(max(math.ceil(math.log2(amax / 448.0)) + 127, 0), 254)
            assert amax <= 448.0 * 2.0 ** (want - 127)
            assert int(s[r, blk]) == want
            X = 2.0 ** (want - 127)
            for k in range(0, 32, 7):
                xv = float(v[k]) / X
                assert int(q[r, 32 * blk + k]) == e4m3_rne(max(-448.0, min(448.0, xv)))


def test_dequantize_error_bound():
    torch.manual_seed(1)
    x = torch.randn(64, 512).to(torch.bfloat16)
    d = MX.fake_quant(x)
    _, s = MX.quantize_mx8(x)
    X = torch.pow(2.0, s.float() - 127).repeat_interleave(32, dim=1)
    # no clipping (amax / X <= 448); e4m3: 3 mantissa bits -> half-ulp <= 2^-4 relative on normals,
    # subnormal step 2^-9 * X
    bound = torch.maximum(x.float().abs() * 2.0 ** -4, X * 2.0 ** -10)
    assert bool(((d - x.float()).abs() <= bound + 1e-30).all())


def test_scale_tile_layout_matches_formula():
    torch.manual_seed(2)
    M, K = 300, 384
    s = torch.randint(0, 255, (M, K // 32), dtype=torch.uint8)
    flat = MX.scale_tile_layout(s)
    Mp = 512
    assert flat.numel() == Mp * (K // 32)
    KT = K // 128
    for row in list(range(0, M, 37)) + [M - 1]:
        for b in range(K // 32):
            idx = (((row // 64) * KT + b // 4) * 64 + (b % 4) * 16 + row % 16) * 4 + (row % 64) // 16
            assert int(flat[idx]) == int(s[row, b])
    # padding rows are zero
    pad = torch.zeros(Mp, K // 32, dtype=torch.uint8)
    pad[:M] = 1
    assert int(MX.scale_tile_layout(pad).sum()) == M * (K // 32)


def test_mx8_linear_backward_is_quantized_ste():
    torch.manual_seed(3)
    x = torch.randn(5, 64, 256).to(torch.bfloat16).requires_grad_(True)
    W = (torch.randn(384, 256) * 0.05).to(torch.bfloat16)
    y = MX.mx8_linear(x, W)
    assert y.shape == (5, 64, 384) and y.dtype == torch.bfloat16
    ref = (MX.fake_quant(x.detach().reshape(-1, 256)) @ MX.fake_quant(W).T).to(torch.bfloat16)
    assert torch.equal(y.detach().reshape(-1, 384), ref)
    dy = torch.randn_like(y)
    y.backward(dy)
    dref = (MX.fake_quant(dy.reshape(-1, 384)) @ MX.fake_quant(W.T.contiguous()).T).to(torch.bfloat16)
    assert torch.equal(x.grad.reshape(-1, 256), dref)


@pytest.mark.parametrize("K", [100, 96])
def test_quantize_rejects_bad_k(K):
    with pytest.raises(ValueError):
        MX.scale_tile_layout(torch.zeros(4, K // 32, dtype=torch.uint8)) if K % 32 == 0 else MX.quantize_mx8(
            torch.zeros(4, K))
