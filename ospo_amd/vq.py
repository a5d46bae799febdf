"""VQ image tokenizer on the MI355X: Janus-Pro's ``gen_vision_model.encode``
and, for step-3 sampling, its pixel decoder ``decode_code`` (``VQDecoder``).  Encode:
(``janus/models/vq_model.py``: Encoder :46-124, quant_conv, VectorQuantizer :236-282) -- pixels to the
VQ ids the SimPO step consumes (``ospo/wrapper/train.py:246-264`` encodes each chosen / rejected
image; here once, into a token cache, see ``build_token_cache``).

fp32 on the HIP kernels of ``csrc/vq.hip`` (f32-MFMA implicit-GEMM convolutions, GroupNorm, the
AttnBlock as two batched products + softmax, the quantizer); activations NHWC.  No fallback: the
library must be present.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Optional, Sequence

import numpy as np
import torch

from ._lib import call, query

F32 = torch.float32
VQ16 = dict(ch=128, ch_mult=(1, 1, 2, 2, 4), num_res_blocks=2, z_channels=256, n_codes=16384, e_dim=8,
            in_channels=3)


def _p(t):
    return None if t is None else t.data_ptr()


def _s():
    return torch.cuda.current_stream().cuda_stream


class VQEncoder:
    """Device-resident VQ-16 encoder.  ``weights``: the reference's state_dict names
    (``encoder.*``, ``quant_conv.*``, ``quantize.embedding.weight``), any float dtype."""

    def __init__(self, weights: Dict[str, torch.Tensor], device="cuda", cfg=VQ16):
        self.cfg, self.device = cfg, torch.device(device)
        self.w = {}
        for k, v in weights.items():
            if not (k.startswith("encoder.") or k.startswith("quant_conv.") or k == "quantize.embedding.weight"):
                continue
            t = v.detach().to(device=self.device, dtype=F32)
            if t.dim() == 4:  # conv [Cout, Cin, KH, KW] -> [Cout, KH, KW, Cin]
                t = t.permute(0, 2, 3, 1)
            self.w[k] = t.contiguous()
        cb = self.w["quantize.embedding.weight"]
        self.codebook = torch.empty_like(cb)
        call("ospo_vq_l2norm_rows", _p(cb), cb.shape[0], cb.shape[1], _p(self.codebook), _s())
        self.gn_ws = torch.empty(query("ospo_vq_groupnorm_ws_bytes", 64, 32) // 4 + 4, dtype=F32, device=self.device)

    # -------------------------------------------------------------- pieces
    def _conv(self, x, name, stride=1, pad=1, Ho=None, Wo=None, residual=None):
        B, H, W, Cin = x.shape
        wt, b = self.w[name + ".weight"], self.w.get(name + ".bias")
        Cout, KH, KW, _ = wt.shape
        Ho = Ho or (H + 2 * pad - KH) // stride + 1
        Wo = Wo or (W + 2 * pad - KW) // stride + 1
        out = torch.empty(B, Ho, Wo, Cout, dtype=F32, device=self.device)
        call("ospo_vq_conv2d", _p(x), B, H, W, Cin, _p(wt), Cout, KH, KW, stride, pad, pad, Ho, Wo, _p(b),
             _p(residual), _p(out), _s())
        return out

    def _gn(self, x, name, swish):
        B, H, W, C = x.shape
        out = torch.empty_like(x)
        if B > 64:
            raise ValueError("at most 64 images per encode call")
        call("ospo_vq_groupnorm", _p(x), B, H * W, C, 32, _p(self.w[name + ".weight"]), _p(self.w[name + ".bias"]),
             1e-6, int(swish), _p(out), _p(self.gn_ws), self.gn_ws.numel() * 4, _s())
        return out

    def _res(self, x, p, cin, cout):
        h = self._conv(self._gn(x, p + ".norm1", True), p + ".conv1")
        h = self._gn(h, p + ".norm2", True)
        sc = self._conv(x, p + ".nin_shortcut", pad=0) if cin != cout else x
        return self._conv(h, p + ".conv2", residual=sc)

    def _attn(self, x, p):
        B, H, W, C = x.shape
        n = H * W
        h = self._gn(x, p + ".norm", False)
        q, k, v = (self._conv(h, p + "." + m, pad=0) for m in ("q", "k", "v"))
        s = torch.empty(B, n, n, dtype=F32, device=self.device)
        call("ospo_vq_bmm_nt", _p(q), _p(k), B, n, n, C, _p(s), _s())
        call("ospo_vq_softmax_rows", _p(s), B * n, n, float(int(C) ** (-0.5)), _s())
        vt = torch.empty(B, C, n, dtype=F32, device=self.device)
        call("ospo_vq_transpose", _p(v), B, n, C, _p(vt), _s())
        o = torch.empty(B, n, C, dtype=F32, device=self.device)
        call("ospo_vq_bmm_nt", _p(s), _p(vt), B, n, C, n, _p(o), _s())
        return self._conv(o.view(B, H, W, C), p + ".proj_out", pad=0, residual=x)

    # -------------------------------------------------------------- encode
    @torch.inference_mode()
    def encode(self, pixels: torch.Tensor, return_z: bool = False):
        """pixels fp32 [B, 3, H, W] in [-1, 1] (H, W multiples of 16) -> ids int32 [B, (H/16)(W/16)]
        (+ z, the quant_conv output NHWC, and each token's minimum distance when return_z)."""
        cfg = self.cfg
        if pixels.dim() != 4 or pixels.shape[1] != cfg["in_channels"]:
            raise ValueError(f"pixels must be [B, {cfg['in_channels']}, H, W], got {tuple(pixels.shape)}")
        B, _, H, W = pixels.shape
        if H % 16 or W % 16:
            raise ValueError("H and W must be multiples of 16 (4 stride-2 downsamples)")
        x = pixels.to(device=self.device, dtype=F32).permute(0, 2, 3, 1).contiguous()
        ch, mult, nrb = cfg["ch"], cfg["ch_mult"], cfg["num_res_blocks"]
        x = self._conv(x, "encoder.conv_in")
        in_mult = (1,) + tuple(mult)
        block_in = ch
        for i, m in enumerate(mult):  # Encoder.forward :107-116
            block_in, block_out = ch * in_mult[i], ch * m
            for j in range(nrb):
                x = self._res(x, f"encoder.conv_blocks.{i}.res.{j}", block_in, block_out)
                block_in = block_out
                if i == len(mult) - 1:
                    x = self._attn(x, f"encoder.conv_blocks.{i}.attn.{j}")
            if i != len(mult) - 1:  # Downsample: pad (0, 1, 0, 1), 3x3 stride 2, no implicit padding
                Hc, Wc = x.shape[1], x.shape[2]
                x = self._conv(x, f"encoder.conv_blocks.{i}.downsample.conv", stride=2, pad=0, Ho=Hc // 2, Wo=Wc // 2)
        x = self._res(x, "encoder.mid.0", block_in, block_in)
        x = self._attn(x, "encoder.mid.1")
        x = self._res(x, "encoder.mid.2", block_in, block_in)
        x = self._gn(x, "encoder.norm_out", True)
        x = self._conv(x, "encoder.conv_out")
        z = self._conv(x, "quant_conv", pad=0)  # [B, h, w, e]
        n = z.shape[0] * z.shape[1] * z.shape[2]
        ids = torch.empty(n, dtype=torch.int32, device=self.device)
        dmin = torch.empty(n, dtype=F32, device=self.device) if return_z else None
        call("ospo_vq_quantize", _p(z), n, cfg["e_dim"], _p(self.codebook), self.codebook.shape[0], _p(ids), _p(dmin),
             _s())
        ids = ids.view(B, -1)
        return (ids, z, dmin.view(B, -1)) if return_z else ids


class VQDecoder:
    """Device-resident VQ-16 pixel decoder: ``gen_vision_model.decode_code`` (vq_model.py:505-508) as the
    step-3 sampler calls it (``image_generation.py:174``) and the uint8 images it saves (:175-181).
    ``weights``: the reference's state_dict names (``post_quant_conv.*``, ``decoder.*``,
    ``quantize.embedding.weight``).  fp32 on the same convolution / GroupNorm / attention kernels as
    the encoder; the Upsample's nearest 2x is read on the fly by the next convolution."""

    def __init__(self, weights: Dict[str, torch.Tensor], device="cuda", cfg=VQ16):
        self.cfg, self.device = cfg, torch.device(device)
        self.w = {}
        for k, v in weights.items():
            if not (k.startswith("decoder.") or k.startswith("post_quant_conv.") or k == "quantize.embedding.weight"):
                continue
            t = v.detach().to(device=self.device, dtype=F32)
            if t.dim() == 4:
                t = t.permute(0, 2, 3, 1)
            self.w[k] = t.contiguous()
        cb = self.w["quantize.embedding.weight"]
        self.codebook = torch.empty_like(cb)
        call("ospo_vq_l2norm_rows", _p(cb), cb.shape[0], cb.shape[1], _p(self.codebook), _s())
        self.gn_ws = torch.empty(query("ospo_vq_groupnorm_ws_bytes", 64, 32) // 4 + 4, dtype=F32, device=self.device)

    _conv = VQEncoder._conv
    _gn = VQEncoder._gn
    _res = VQEncoder._res
    _attn = VQEncoder._attn

    def _upconv(self, x, name):
        B, H, W, Cin = x.shape
        wt, b = self.w[name + ".weight"], self.w.get(name + ".bias")
        Cout = wt.shape[0]
        out = torch.empty(B, 2 * H, 2 * W, Cout, dtype=F32, device=self.device)
        call("ospo_vq_conv2d_up2", _p(x), B, H, W, Cin, _p(wt), Cout, 3, 3, 1, _p(b), None, _p(out), _s())
        return out

    @torch.inference_mode()
    def decode_code(self, ids: torch.Tensor, h: int = 24, w: int = 24) -> torch.Tensor:
        """ids int [B, h*w] (device or host) -> fp32 NHWC [B, 16h, 16w, 3] in the decoder's output range."""
        cfg = self.cfg
        ids = ids.to(device=self.device, dtype=torch.int32).contiguous()
        B = ids.shape[0]
        if ids.shape[1] != h * w:
            raise ValueError(f"{ids.shape[1]} ids per image, expected {h} x {w}")
        if B > 64:
            raise ValueError("at most 64 images per decode call")
        e = cfg["e_dim"]
        z = torch.empty(B, h, w, e, dtype=F32, device=self.device)
        call("ospo_vq_embed_codes", _p(ids), B * h * w, _p(self.codebook), self.codebook.shape[0], e, _p(z), _s())
        x = self._conv(z, "post_quant_conv", pad=0)
        ch, mult, nrb = cfg["ch"], cfg["ch_mult"], cfg["num_res_blocks"]
        nl = len(mult)
        block_in = ch * mult[nl - 1]
        x = self._conv(x, "decoder.conv_in")
        x = self._res(x, "decoder.mid.0", block_in, block_in)
        x = self._attn(x, "decoder.mid.1")
        x = self._res(x, "decoder.mid.2", block_in, block_in)
        for li, i_level in enumerate(reversed(range(nl))):  # Decoder.forward :199-207
            block_out = ch * mult[i_level]
            for j in range(nrb + 1):
                x = self._res(x, f"decoder.conv_blocks.{li}.res.{j}", block_in, block_out)
                block_in = block_out
                if i_level == nl - 1:
                    x = self._attn(x, f"decoder.conv_blocks.{li}.attn.{j}")
            if i_level != 0:
                x = self._upconv(x, f"decoder.conv_blocks.{li}.upsample.conv")
        x = self._gn(x, "decoder.norm_out", True)
        return self._conv(x, "decoder.conv_out")

    @torch.inference_mode()
    def to_images(self, dec: torch.Tensor) -> torch.Tensor:
        """image_generation.py:175-181: uint8 [B, H, W, 3] = clip((dec + 1) / 2 * 255, 0, 255), truncated."""
        out = torch.empty(dec.shape, dtype=torch.uint8, device=self.device)
        call("ospo_vq_to_uint8", _p(dec), dec.numel(), _p(out), _s())
        return out


def synthetic_vq_decoder_weights(seed: int = 1, cfg=VQ16) -> Dict[str, torch.Tensor]:
    """Random VQ-16 decoder weights (post_quant_conv + decoder.*), fan-in scaled convs."""
    g = torch.Generator().manual_seed(int(seed))
    w: Dict[str, torch.Tensor] = {}
    ch, mult, nrb = cfg["ch"], cfg["ch_mult"], cfg["num_res_blocks"]

    def conv(name, cin, cout, k):
        w[name + ".weight"] = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)
        w[name + ".bias"] = torch.randn(cout, generator=g) * 0.02

    def norm(name, c):
        w[name + ".weight"] = 1.0 + torch.randn(c, generator=g) * 0.05
        w[name + ".bias"] = torch.randn(c, generator=g) * 0.05

    def res(p, cin, cout):
        norm(p + ".norm1", cin)
        conv(p + ".conv1", cin, cout, 3)
        norm(p + ".norm2", cout)
        conv(p + ".conv2", cout, cout, 3)
        if cin != cout:
            conv(p + ".nin_shortcut", cin, cout, 1)

    def attn(p, c):
        norm(p + ".norm", c)
        for n in ("q", "k", "v", "proj_out"):
            conv(p + "." + n, c, c, 1)

    nl = len(mult)
    block_in = ch * mult[nl - 1]
    conv("post_quant_conv", cfg["e_dim"], cfg["z_channels"], 1)
    conv("decoder.conv_in", cfg["z_channels"], block_in, 3)
    res("decoder.mid.0", block_in, block_in)
    attn("decoder.mid.1", block_in)
    res("decoder.mid.2", block_in, block_in)
    for li, i_level in enumerate(reversed(range(nl))):
        block_out = ch * mult[i_level]
        for j in range(nrb + 1):
            res(f"decoder.conv_blocks.{li}.res.{j}", block_in, block_out)
            block_in = block_out
            if i_level == nl - 1:
                attn(f"decoder.conv_blocks.{li}.attn.{j}", block_in)
        if i_level != 0:
            conv(f"decoder.conv_blocks.{li}.upsample.conv", block_in, block_in, 3)
    norm("decoder.norm_out", block_in)
    conv("decoder.conv_out", block_in, cfg["in_channels"], 3)
    return w


def build_token_cache(encoder: VQEncoder, items: Iterable, out_path: str, size: int = 384, batch: int = 16):
    """items: (key, image path) pairs -> ``out_path`` .npz of int32 VQ ids per key (the
    ``dataset.train.token_cache`` the SimPO dataloader reads: keys "{item_id}/chosen|rejected").
    Pixels: VLMImageProcessor with the gen processor's mean = std = 0.5 (bicubic resize to size)."""
    from PIL import Image
    keys, pix, out = [], [], {}

    def flush():
        if not keys:
            return
        ids = encoder.encode(torch.stack(pix)).cpu().numpy()
        for k, row in zip(keys, ids):
            out[k] = row.astype(np.int32)
        keys.clear()
        pix.clear()

    for key, path in items:
        im = Image.open(path).convert("RGB")
        if im.size != (size, size):
            im = im.resize((size, size), Image.BICUBIC)
        a = torch.from_numpy(np.asarray(im, dtype=np.uint8).copy()).permute(2, 0, 1).float() / 255.0
        keys.append(key)
        pix.append((a - 0.5) / 0.5)
        if len(keys) == batch:
            flush()
    flush()
    np.savez_compressed(out_path, **out)
    return out


def load_vq_weights(path: Optional[str], seed: int = 0) -> Dict[str, torch.Tensor]:
    """VQ-16 weights from a safetensors file (``gen_vision_model.*`` keys of a Janus-Pro checkpoint, or
    bare ``encoder.* / quant_conv.* / quantize.*``), else seeded synthetic ones (no checkpoint offline)."""
    if path:
        from safetensors.torch import load_file
        sd = load_file(path)
        out = {}
        for k, v in sd.items():
            k2 = k[len("gen_vision_model."):] if k.startswith("gen_vision_model.") else k
            if k2.startswith(("encoder.", "quant_conv.", "quantize.embedding")):
                out[k2] = v
        if "quantize.embedding.weight" not in out:
            raise ValueError(f"{path}: no VQ weights (gen_vision_model.* / encoder.*) found")
        return out
    print(f"[ospo_amd.vq] no VQ weights given: seeded synthetic VQ-16 weights (seed {seed})")
    return synthetic_vq_weights(seed)


def synthetic_vq_weights(seed: int = 0, cfg=VQ16) -> Dict[str, torch.Tensor]:
    """Random VQ-16 weights under the reference's state_dict names (fan-in scaled convs, unit-norm codebook)."""
    g = torch.Generator().manual_seed(int(seed))
    w: Dict[str, torch.Tensor] = {}
    ch, mult = cfg["ch"], cfg["ch_mult"]

    def conv(name, cin, cout, k):
        w[name + ".weight"] = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)
        w[name + ".bias"] = torch.randn(cout, generator=g) * 0.02

    def norm(name, c):
        w[name + ".weight"] = 1.0 + torch.randn(c, generator=g) * 0.05
        w[name + ".bias"] = torch.randn(c, generator=g) * 0.05

    def res(p, cin, cout):
        norm(p + ".norm1", cin)
        conv(p + ".conv1", cin, cout, 3)
        norm(p + ".norm2", cout)
        conv(p + ".conv2", cout, cout, 3)
        if cin != cout:
            conv(p + ".nin_shortcut", cin, cout, 1)

    def attn(p, c):
        norm(p + ".norm", c)
        for n in ("q", "k", "v", "proj_out"):
            conv(p + "." + n, c, c, 1)

    conv("encoder.conv_in", cfg["in_channels"], ch, 3)
    in_mult = (1,) + tuple(mult)
    block_in = ch
    for i, m in enumerate(mult):
        block_in, block_out = ch * in_mult[i], ch * m
        for j in range(cfg["num_res_blocks"]):
            res(f"encoder.conv_blocks.{i}.res.{j}", block_in, block_out)
            block_in = block_out
            if i == len(mult) - 1:
                attn(f"encoder.conv_blocks.{i}.attn.{j}", block_in)
        if i != len(mult) - 1:
            conv(f"encoder.conv_blocks.{i}.downsample.conv", block_in, block_in, 3)
    res("encoder.mid.0", block_in, block_in)
    attn("encoder.mid.1", block_in)
    res("encoder.mid.2", block_in, block_in)
    norm("encoder.norm_out", block_in)
    conv("encoder.conv_out", block_in, cfg["z_channels"], 3)
    conv("quant_conv", cfg["z_channels"], cfg["e_dim"], 1)
    cb = (torch.rand(cfg["n_codes"], cfg["e_dim"], generator=g) * 2 - 1) / cfg["n_codes"]
    w["quantize.embedding.weight"] = cb / cb.norm(dim=1, keepdim=True).clamp_min(1e-12)
    return w


def main(argv=None):
    """python -m ospo_amd.vq --data-path train.json --out token_cache.npz [--weights vq.safetensors]
    [--path-map OLD=NEW]: the step-5 dataset's chosen / rejected images (ospo/dataclass/train_dataset.py:
    79-97) -> ``dataset.train.token_cache`` (keys "{item_id}/chosen|rejected")."""
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--data-path", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--weights", default=None)
    ap.add_argument("--path-map", action="append", default=[])
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    maps = [m.split("=", 1) for m in a.path_map]

    def remap(p):
        for old, new in maps:
            if p.startswith(old):
                return new + p[len(old):]
        return p
    items = []
    for ex in json.load(open(a.data_path)):
        items.append((f"{ex['item_id']}/chosen", remap(ex["chosen"])))
        items.append((f"{ex['item_id']}/rejected", remap(ex["rejected"])))
    enc = VQEncoder(load_vq_weights(a.weights, a.seed))
    out = build_token_cache(enc, items, a.out, batch=a.batch)
    print(f"[ospo_amd.vq] {len(out)} images -> {a.out}")


if __name__ == "__main__":
    main()
