"""CPU oracle for the VQ image tokenizer.

TEST INFRASTRUCTURE ONLY (the checker, never the product; see oracle/simpo_ref.py).

Functional fp32 restatement of Janus-Pro's ``gen_vision_model.encode`` (``janus/models/vq_model.py``):
``Encoder.forward`` (:105-124: conv_in, 5 levels of 2 ``ResnetBlock`` (:296-343) with ``AttnBlock``
(:346-383) at the last level, ``Downsample`` (:430-447, pad (0,1,0,1) then a stride-2 3x3 conv), the
mid block, GroupNorm(32, eps 1e-6) + swish, conv_out), ``quant_conv`` (1x1) and
``VectorQuantizer.forward`` (:236-282: l2-normalise z and the codebook, d = |z|^2 + |e|^2 - 2 z.e,
``argmin``).  VQ-16 = ``ModelArgs`` defaults: ch 128, ch_mult (1, 1, 2, 2, 4), 2 res blocks,
z_channels 256, codebook 16384 x 8.

``decode_code_ref`` restates the pixel decoder the step-3 sampler calls
(``image_generation.py:174``: ``VQModel.decode_code`` :505-508 = ``VectorQuantizer.get_codebook_entry``
:284-298 (l2-normalised codebook rows), ``post_quant_conv`` (1x1, 8 -> 256), ``Decoder.forward``
:191-214: conv_in, mid (res, attn, res), 5 levels of 3 ``ResnetBlock`` with ``AttnBlock`` at the
first (lowest-resolution) level and ``Upsample`` (:411-427: nearest x2, then a 3x3 conv) after every
level but the last, GroupNorm + swish, conv_out (-> 3 channels)) and the uint8 conversion of
``image_generation.py:175-181`` (clip((dec + 1) / 2 * 255, 0, 255), truncated).

``init_vq_weights`` / ``init_vq_decoder_weights`` draw seeded weights under the reference's
``state_dict`` names, so ``tests/golden/make_golden_vq.py`` can load them into the reference's own
``VQModel`` and pin this restatement to it.  There is no Janus-Pro checkpoint offline.
"""
from __future__ import annotations

import math
from typing import Dict, Sequence, Tuple

import torch
import torch.nn.functional as F

VQ16 = dict(ch=128, ch_mult=(1, 1, 2, 2, 4), num_res_blocks=2, z_channels=256, n_codes=16384, e_dim=8,
            in_channels=3)


def encoder_plan(cfg=VQ16):
    """The module tree of Encoder.__init__ (:48-103) as (kind, prefix, cin, cout) in forward order."""
    ch, mult, nrb = cfg["ch"], cfg["ch_mult"], cfg["num_res_blocks"]
    plan = [("conv", "encoder.conv_in", cfg["in_channels"], ch, 3)]
    in_mult = (1,) + tuple(mult)
    block_in = ch
    for i, m in enumerate(mult):
        block_in = ch * in_mult[i]
        block_out = ch * m
        for j in range(nrb):
            plan.append(("res", f"encoder.conv_blocks.{i}.res.{j}", block_in, block_out, 3))
            block_in = block_out
            if i == len(mult) - 1:
                plan.append(("attn", f"encoder.conv_blocks.{i}.attn.{j}", block_in, block_in, 1))
        if i != len(mult) - 1:
            plan.append(("down", f"encoder.conv_blocks.{i}.downsample.conv", block_in, block_in, 3))
    plan += [("res", "encoder.mid.0", block_in, block_in, 3), ("attn", "encoder.mid.1", block_in, block_in, 1),
             ("res", "encoder.mid.2", block_in, block_in, 3), ("norm_out", "encoder.norm_out", block_in, block_in, 0),
             ("conv", "encoder.conv_out", block_in, cfg["z_channels"], 3),
             ("conv", "quant_conv", cfg["z_channels"], cfg["e_dim"], 1)]
    return plan


def init_vq_weights(seed: int = 0, cfg=VQ16) -> Dict[str, torch.Tensor]:
    """Seeded fp32 weights under the reference's state_dict names: convs N(0, 1/fan_in), biases
    N(0, 0.02), GroupNorm affine 1 + N(0, 0.05) / N(0, 0.05), codebook U(-1/n, 1/n) (as
    VectorQuantizer.__init__, :228) l2-normalised (:229-232)."""
    g = torch.Generator().manual_seed(int(seed))
    w: Dict[str, torch.Tensor] = {}

    def conv(name, cin, cout, k):
        w[name + ".weight"] = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)
        w[name + ".bias"] = torch.randn(cout, generator=g) * 0.02

    def norm(name, c):
        w[name + ".weight"] = 1.0 + torch.randn(c, generator=g) * 0.05
        w[name + ".bias"] = torch.randn(c, generator=g) * 0.05

    for kind, p, cin, cout, k in encoder_plan(cfg):
        if kind in ("conv", "down"):
            conv(p, cin, cout, k)
        elif kind == "res":
            norm(p + ".norm1", cin)
            conv(p + ".conv1", cin, cout, 3)
            norm(p + ".norm2", cout)
            conv(p + ".conv2", cout, cout, 3)
            if cin != cout:
                conv(p + ".nin_shortcut", cin, cout, 1)
        elif kind == "attn":
            norm(p + ".norm", cin)
            for n in ("q", "k", "v", "proj_out"):
                conv(p + "." + n, cin, cin, 1)
        elif kind == "norm_out":
            norm(p, cin)
    n, e = cfg["n_codes"], cfg["e_dim"]
    cb = (torch.rand(n, e, generator=g) * 2 - 1) / n
    w["quantize.embedding.weight"] = F.normalize(cb, p=2, dim=-1)
    return w


def decoder_plan(cfg=VQ16):
    """The module tree of Decoder.__init__ (:128-181) as (kind, prefix, cin, cout, k) in forward order
    (post_quant_conv first)."""
    ch, mult, nrb = cfg["ch"], cfg["ch_mult"], cfg["num_res_blocks"]
    nl = len(mult)
    block_in = ch * mult[nl - 1]
    plan = [("conv", "post_quant_conv", cfg["e_dim"], cfg["z_channels"], 1),
            ("conv", "decoder.conv_in", cfg["z_channels"], block_in, 3),
            ("res", "decoder.mid.0", block_in, block_in, 3), ("attn", "decoder.mid.1", block_in, block_in, 1),
            ("res", "decoder.mid.2", block_in, block_in, 3)]
    for li, i_level in enumerate(reversed(range(nl))):
        block_out = ch * mult[i_level]
        for j in range(nrb + 1):
            plan.append(("res", f"decoder.conv_blocks.{li}.res.{j}", block_in, block_out, 3))
            block_in = block_out
            if i_level == nl - 1:
                plan.append(("attn", f"decoder.conv_blocks.{li}.attn.{j}", block_in, block_in, 1))
        if i_level != 0:
            plan.append(("up", f"decoder.conv_blocks.{li}.upsample.conv", block_in, block_in, 3))
    plan += [("norm_out", "decoder.norm_out", block_in, block_in, 0),
             ("conv", "decoder.conv_out", block_in, cfg["in_channels"], 3)]
    return plan


def init_vq_decoder_weights(seed: int = 1, cfg=VQ16) -> Dict[str, torch.Tensor]:
    """Seeded fp32 decoder weights (post_quant_conv + decoder.*), the same distributions as
    init_vq_weights."""
    g = torch.Generator().manual_seed(int(seed))
    w: Dict[str, torch.Tensor] = {}

    def conv(name, cin, cout, k):
        w[name + ".weight"] = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)
        w[name + ".bias"] = torch.randn(cout, generator=g) * 0.02

    def norm(name, c):
        w[name + ".weight"] = 1.0 + torch.randn(c, generator=g) * 0.05
        w[name + ".bias"] = torch.randn(c, generator=g) * 0.05

    for kind, p, cin, cout, k in decoder_plan(cfg):
        if kind in ("conv", "up"):
            conv(p, cin, cout, k)
        elif kind == "res":
            norm(p + ".norm1", cin)
            conv(p + ".conv1", cin, cout, 3)
            norm(p + ".norm2", cout)
            conv(p + ".conv2", cout, cout, 3)
            if cin != cout:
                conv(p + ".nin_shortcut", cin, cout, 1)
        elif kind == "attn":
            norm(p + ".norm", cin)
            for n in ("q", "k", "v", "proj_out"):
                conv(p + "." + n, cin, cin, 1)
        elif kind == "norm_out":
            norm(p, cin)
    return w


def _gn(x, w, p, swish):
    y = F.group_norm(x, 32, w[p + ".weight"], w[p + ".bias"], eps=1e-6)
    return y * torch.sigmoid(y) if swish else y


def _conv(x, w, p, stride=1, padding=1):
    return F.conv2d(x, w[p + ".weight"], w[p + ".bias"], stride=stride, padding=padding)


def _run(x, w, plan):
    for kind, p, cin, cout, k in plan:
        if kind == "conv":
            x = _conv(x, w, p, padding=k // 2)
        elif kind == "down":
            x = _conv(F.pad(x, (0, 1, 0, 1)), w, p, stride=2, padding=0)
        elif kind == "up":
            x = _conv(F.interpolate(x, scale_factor=2.0, mode="nearest"), w, p)
        elif kind == "res":
            h = _conv(_gn(x, w, p + ".norm1", True), w, p + ".conv1")
            h = _conv(_gn(h, w, p + ".norm2", True), w, p + ".conv2")
            if cin != cout:
                x = _conv(x, w, p + ".nin_shortcut", padding=0)
            x = x + h
        elif kind == "attn":
            h = _gn(x, w, p + ".norm", False)
            q, kk, v = (_conv(h, w, p + "." + n, padding=0) for n in ("q", "k", "v"))
            b, c, hh, ww = q.shape
            q = q.reshape(b, c, hh * ww).permute(0, 2, 1)
            kk = kk.reshape(b, c, hh * ww)
            a = torch.bmm(q, kk) * (int(c) ** (-0.5))
            a = F.softmax(a, dim=2)
            v = v.reshape(b, c, hh * ww)
            o = torch.bmm(v, a.permute(0, 2, 1)).reshape(b, c, hh, ww)
            x = x + _conv(o, w, p + ".proj_out", padding=0)
        elif kind == "norm_out":
            x = _gn(x, w, p, True)
    return x


def encode_ref(pixels: torch.Tensor, w: Dict[str, torch.Tensor], cfg=VQ16) -> Tuple[torch.Tensor, torch.Tensor,
                                                                                    torch.Tensor]:
    """pixels fp32 [B, 3, H, W] in [-1, 1] -> (ids int64 [B, h*w], z fp32 [B, e, h, w] (quant_conv out),
    margin fp32 [B, h*w] = second-smallest minus smallest distance)."""
    z = _run(pixels.float(), w, encoder_plan(cfg))
    ids, margin = quantize_ref(z, w["quantize.embedding.weight"])
    return ids, z, margin


def decode_code_ref(ids: torch.Tensor, w: Dict[str, torch.Tensor], h: int = 24, wd: int = 24, cfg=VQ16):
    """ids int [B, h*w] -> decoded fp32 [B, 3, 16h, 16w] (VQModel.decode_code with shape
    [B, e_dim, h, w], channel_first, image_generation.py:174)."""
    emb = F.normalize(w["quantize.embedding.weight"].float(), p=2, dim=-1)
    B = ids.shape[0]
    zq = emb[ids.reshape(-1).long()].reshape(B, h, wd, cfg["e_dim"]).permute(0, 3, 1, 2).contiguous()
    return _run(zq, w, decoder_plan(cfg))


def to_uint8_images(dec: torch.Tensor):
    """image_generation.py:175-181: NHWC, clip((dec + 1) / 2 * 255, 0, 255) in fp32, stored into a
    uint8 array (truncation toward zero)."""
    import numpy as np
    d = dec.float().cpu().numpy().transpose(0, 2, 3, 1)
    d = np.clip((d + 1) / 2 * 255, 0, 255)
    out = np.zeros(d.shape, dtype=np.uint8)
    out[:] = d
    return out


def quantize_ref(z: torch.Tensor, codebook: torch.Tensor):
    """VectorQuantizer.forward (:236-258) with l2_norm: ids = argmin d (first index on ties)."""
    b, e, h, ww = z.shape
    zf = F.normalize(z.permute(0, 2, 3, 1).reshape(-1, e), p=2, dim=-1)
    emb = F.normalize(codebook, p=2, dim=-1)
    d = torch.sum(zf ** 2, dim=1, keepdim=True) + torch.sum(emb ** 2, dim=1) - 2 * torch.einsum(
        "bd,dn->bn", zf, emb.t())
    ids = torch.argmin(d, dim=1)
    top2 = torch.topk(d, 2, dim=1, largest=False).values
    return ids.reshape(b, h * ww), (top2[:, 1] - top2[:, 0]).reshape(b, h * ww)


def load_pixels(path: str, size: int = 384) -> torch.Tensor:
    """PNG -> fp32 [3, size, size] in [-1, 1]: VLMImageProcessor with the Janus-Pro gen processor's
    mean = std = 0.5 (bicubic resize when the image is not already size x size)."""
    import numpy as np
    from PIL import Image
    im = Image.open(path).convert("RGB")
    if im.size != (size, size):
        im = im.resize((size, size), Image.BICUBIC)
    a = torch.from_numpy(np.asarray(im, dtype=np.uint8).copy()).permute(2, 0, 1).float() / 255.0
    return (a - 0.5) / 0.5
