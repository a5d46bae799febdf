"""CPU oracle for the MXFP8 variant of the SimPO step (BASELINE config 5).

TEST INFRASTRUCTURE ONLY (the checker, never the product; see oracle/simpo_ref.py).

The reference has no fp8 path: config 5 asks for the same SimPO step with the frozen
decoder Linears (``q/k/v/o/gate/up/down_proj``, peft's base layer inside ``lora.Linear``,
``ospo/utils/model.py:50-60``, called from ``ospo/wrapper/train.py:352``) run on CDNA4 fp8
MFMA.  This module defines that arithmetic so the HIP path can be checked against it:

* OCP Microscaling (MX v1.0) MXFP8-E4M3 along the contraction dim: blocks of 32 values share an
  E8M0 scale X and elements are ``e4m3fn(clamp(x / X, -448, 448))`` with round-to-nearest-even
  (torch's float8_e4m3fn cast).  X is the smallest power of two with max|x| / X <= 448 (the
  round-up / "RCEIL" scale rule of MXFP8 training recipes): the spec's floor rule
  X = 2^(floor(log2 amax) - 8) puts amax / X in [256, 512) and clips block maxima above 448 by up
  to 12.5 %.  With amax = m * 2^E (1 <= m < 2): X = 2^(E - 8) if m <= 1.75 else 2^(E - 7), read
  off the f32 bits exactly.  amax = 0 gives the smallest scale byte (0).
* forward  y  = bf16( deq(q(x)) . deq(q(W))^T ), fp32 accumulation;
* backward dx = bf16( deq(q(dy)) . deq(q(W^T))^T ) -- W^T quantized along the OUT dim, the
  contraction of the backward product; the straight-through estimator (quantisation is not
  differentiated).  The LoRA adapters (A, B, their grads) stay bf16, as on the HIP path.

``scale_tile_layout`` restates the byte layout ``ospo_quant_mx8`` writes (ospo_amd/csrc/mx8.hip)
so the tests can compare the device's scale bytes exactly.
"""
from __future__ import annotations

import torch

E4M3_MAX = 448.0
BLOCK = 32


def quantize_mx8(x: torch.Tensor):
    """x [M, K] (K % 32 == 0) -> (q uint8 [M, K] e4m3fn bytes, sbytes uint8 [M, K/32] E8M0)."""
    M, K = x.shape
    if K % BLOCK:
        raise ValueError("K must be a multiple of 32")
    xf = x.detach().float().reshape(M, K // BLOCK, BLOCK)
    amax = xf.abs().amax(-1)
    bits = amax.view(torch.int32)
    ebits = (bits >> 23) & 0xFF
    up = ((bits & 0x7FFFFF) > 0x600000).to(torch.int32)  # mantissa above 1.75
    sbyte = (ebits - 8 + up).clamp(0, 254)
    inv = ((254 - sbyte).to(torch.int32) << 23).view(torch.float32)  # 2^(127 - sbyte) = 1 / X
    y = (xf * inv.unsqueeze(-1)).clamp(-E4M3_MAX, E4M3_MAX)
    q = y.to(torch.float8_e4m3fn).view(torch.uint8).reshape(M, K)
    return q, sbyte.to(torch.uint8)


def dequantize_mx8(q: torch.Tensor, sbyte: torch.Tensor) -> torch.Tensor:
    """(uint8 e4m3fn [M, K], uint8 [M, K/32]) -> fp32 [M, K] (exact)."""
    M, K = q.shape
    v = q.view(torch.float8_e4m3fn).float().reshape(M, K // BLOCK, BLOCK)
    scale = torch.pow(2.0, sbyte.float() - 127.0)
    return (v * scale.unsqueeze(-1)).reshape(M, K)


def fake_quant(x: torch.Tensor) -> torch.Tensor:
    """deq(q(x)) in fp32."""
    return dequantize_mx8(*quantize_mx8(x))


def scale_tile_layout(sbyte: torch.Tensor) -> torch.Tensor:
    """[M, K/32] scale bytes -> the flat byte image of ospo_quant_mx8 (rows padded to 256, padding 0):
    u32 ((row/64)*(K/128) + k/128)*64 + ((k%128)/32)*16 + row%16, byte (row%64)/16."""
    M, nb = sbyte.shape
    K = nb * BLOCK
    if K % 128:
        raise ValueError("K must be a multiple of 128")
    Mp = (M + 255) // 256 * 256
    s = torch.zeros(Mp, nb, dtype=torch.uint8)
    s[:M] = sbyte
    # row = 64*rb + 16*byte + r16 ; block = 4*kt + q
    s = s.reshape(Mp // 64, 4, 16, K // 128, 4)          # [rb, byte, r16, kt, q]
    s = s.permute(0, 3, 4, 2, 1).contiguous()              # [rb, kt, q, r16, byte]
    return s.reshape(-1)


class _MX8Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(W)
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        y = fake_quant(x2) @ fake_quant(W).T
        return y.to(x.dtype).reshape(*shp[:-1], W.shape[0])

    @staticmethod
    def backward(ctx, dy):
        (W,) = ctx.saved_tensors
        shp = dy.shape
        d2 = dy.reshape(-1, shp[-1]).to(W.dtype)
        dx = fake_quant(d2) @ fake_quant(W.T.contiguous()).T
        return dx.to(dy.dtype).reshape(*shp[:-1], W.shape[1]), None


def mx8_linear(x: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """The frozen base Linear of the fp8 variant (no bias on the decoder Linears)."""
    return _MX8Linear.apply(x, W)
