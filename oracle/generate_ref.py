"""CPU oracle for step-3 text-to-image sampling (BASELINE config 4).

TEST INFRASTRUCTURE ONLY (the checker, never the product; see oracle/simpo_ref.py).

Restates ``JanusProImageGenWrapper.generate_image`` (``ospo/wrapper/image_generation.py:109-171``;
the same loop is ``ospo/inference.py:110-163``) on top of the decoder arithmetic of
``oracle/simpo_ref.py`` (HF 4.38 Llama, eager bf16):

* prompt rows (:124-141): B prompts left-padded with ``pad_id`` to Lp, rows 2b / 2b+1 = prompt b and
  its unconditional copy (``tokens[i, pad_len+1:-1] = pad_id``); attention mask 0 on the padding;
* HF 4.38 ``LlamaModel`` with ``attention_mask`` and ``past_key_values``: position ids are
  ``arange(past_len, past_len + seq)`` -- the padding does not shift them; the 4-D mask adds
  ``finfo(bf16).min`` to masked and future keys;
* per step (:150-169): ``gen_head(h[:, -1])``, ``logit_uncond + cfg_weight * (logit_cond -
  logit_uncond)`` in bf16, ``softmax(logits / temperature)`` (bf16 out), one token per image, its
  ``prepare_gen_img_embeds`` fed to both rows of the pair;
* the draw: ``torch.multinomial`` in the reference; here the inverse CDF of ``ospo_cfg_sample``
  restated bit for bit (fp32 sums of 64-element chunks, then the chunk sums, in order), so given the
  same probabilities and uniform the oracle picks the same token.

Teacher forcing (``forced``) runs the same computation on a given token sequence and returns the
per-step probabilities, which is how the HIP sampler is checked step by step.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from oracle import simpo_ref as O

BF16 = torch.bfloat16
CHUNK = 64


def prompt_rows(prompts: Sequence[Sequence[int]], pad_id: int):
    B = len(prompts)
    Lp = max(len(p) for p in prompts)
    toks = torch.full((2 * B, Lp), pad_id, dtype=torch.long)
    mask = torch.ones(2 * B, Lp, dtype=torch.long)
    for i in range(2 * B):
        ids = torch.tensor(list(prompts[i // 2]), dtype=torch.long)
        pad = Lp - ids.numel()
        toks[i, pad:] = ids
        mask[i, :pad] = 0
        if i % 2 != 0:
            toks[i, pad + 1: Lp - 1] = pad_id
    return toks, mask, Lp


def merge_lora(w, dims):
    """W + s B A for every adapter present (inference.py merges the trained LoRA before sampling)."""
    out = dict(w)
    s = dims.lora_alpha / dims.lora_r
    for k in list(w):
        if k.endswith(".lora_A"):
            base = k[: -len(".lora_A")]
            W = w[base].float() + s * (w[base + ".lora_B"].float() @ w[k].float())
            out[base] = W.to(w[base].dtype)
    return {k: v for k, v in out.items() if ".lora_" not in k}


def sample_inverse_cdf(probs: np.ndarray, u: float) -> int:
    """ospo_cfg_sample's draw, restated: probs fp32 (bf16 values) [V], V <= 256 * 64."""
    V = probs.shape[0]
    p = np.zeros(256 * CHUNK, dtype=np.float32)
    p[:V] = probs.astype(np.float32)
    chunks = p.reshape(256, CHUNK)
    csum = np.add.accumulate(chunks, axis=1, dtype=np.float32)[:, -1]
    tot = np.add.accumulate(csum, dtype=np.float32)[-1]
    target = np.float32(u) * tot
    run, run_last, last = np.float32(0), np.float32(0), 0
    c = 0
    while c < 256:
        if np.float32(run + csum[c]) > target:
            break
        if csum[c] > 0:
            last, run_last = c, run
        run = np.float32(run + csum[c])
        c += 1
    if c == 256:
        c, run = last, run_last
    tok, lastnz = -1, c * CHUNK
    for q in range(CHUNK):
        j = c * CHUNK + q
        if j >= V:
            break
        if chunks[c, q] > 0:
            lastnz = j
        run = np.float32(run + chunks[c, q])
        if run > target:
            tok = j
            break
    return tok if tok >= 0 else lastnz


def guided_probs(logits: torch.Tensor, cfg_weight: float, temperature: float) -> torch.Tensor:
    """image_generation.py:156-160 on bf16 logits [2B, V] -> bf16 probs [B, V]."""
    lc, lu = logits[0::2], logits[1::2]
    lg = lu + cfg_weight * (lc - lu)
    return torch.softmax(lg / temperature, dim=-1)


class _Cache:
    def __init__(self, L):
        self.k = [None] * L
        self.v = [None] * L


def _layer(x, w, i, dims, pos, cache, mask_add):
    """One decoder layer over the new positions ``pos`` (x [R, n, D]) with the KV cache."""
    R, n, D = x.shape
    H, hd = dims.n_heads, dims.head_dim
    pfx = f"layers.{i}."
    h = O.rmsnorm(x, w[pfx + "input_layernorm"], dims.rms_eps)
    q = F.linear(h, w[pfx + "q_proj"]).view(R, n, H, hd).transpose(1, 2)
    k = F.linear(h, w[pfx + "k_proj"]).view(R, n, H, hd).transpose(1, 2)
    v = F.linear(h, w[pfx + "v_proj"]).view(R, n, H, hd).transpose(1, 2)
    cos, sin = O.rope_cos_sin(int(pos[-1]) + 1, hd, dims.rope_theta, x.dtype)
    cos, sin = cos[pos], sin[pos]
    q, k = O.apply_rope(q, cos, sin), O.apply_rope(k, cos, sin)
    cache.k[i] = k if cache.k[i] is None else torch.cat([cache.k[i], k], 2)
    cache.v[i] = v if cache.v[i] is None else torch.cat([cache.v[i], v], 2)
    s = torch.matmul(q, cache.k[i].transpose(-1, -2)) * (1.0 / math.sqrt(hd))
    s = s + mask_add.to(s.dtype)
    p = torch.softmax(s, dim=-1, dtype=torch.float32).to(q.dtype)
    o = torch.matmul(p, cache.v[i]).transpose(1, 2).reshape(R, n, D)
    x = x + F.linear(o, w[pfx + "o_proj"])
    h = O.rmsnorm(x, w[pfx + "post_attention_layernorm"], dims.rms_eps)
    m = F.linear(F.silu(F.linear(h, w[pfx + "gate_proj"])) * F.linear(h, w[pfx + "up_proj"]), w[pfx + "down_proj"])
    return x + m


def generate_ref(prompts: Sequence[Sequence[int]], w, dims, n_img: int, uniforms: torch.Tensor,
                 cfg_weight: float = 5.0, temperature: float = 1.0, pad_id: int = 100015,
                 forced: Optional[torch.Tensor] = None, dtype=BF16):
    """Returns (tokens int64 [B, n_img], probs fp32 [n_img, B, V]).  ``forced`` [B, n_img]: feed these
    tokens instead of the sampled ones (teacher forcing); ``tokens`` are still the oracle's own draws."""
    w = merge_lora({k: (v.to(dtype) if v.is_floating_point() else v) for k, v in w.items()}, dims)
    B = len(prompts)
    toks, amask, Lp = prompt_rows(prompts, pad_id)
    R = 2 * B
    minv = torch.finfo(dtype).min
    cache = _Cache(dims.n_layers)
    x = F.embedding(toks, w["embed_tokens"])
    pos = torch.arange(Lp)
    key_ok = amask.bool()                                       # [R, T]
    causal = torch.ones(Lp, Lp, dtype=torch.bool).tril()
    allowed = causal[None] & key_ok[:, None, :]                 # [R, Lp, Lp]
    out_tok = torch.zeros(B, n_img, dtype=torch.long)
    out_p = torch.zeros(n_img, B, dims.img_vocab, dtype=torch.float32)
    with torch.no_grad():
        for step in range(n_img):
            mask_add = torch.where(allowed, torch.zeros(()), torch.full((), minv))[:, None]  # [R, 1, n, T]
            for i in range(dims.n_layers):
                x = _layer(x, w, i, dims, pos, cache, mask_add)
            hlast = O.rmsnorm(x[:, -1], w["norm"], dims.rms_eps)
            logits = O.gen_head(hlast, w)
            probs = guided_probs(logits, cfg_weight, temperature)
            out_p[step] = probs.float()
            for b in range(B):
                out_tok[b, step] = sample_inverse_cdf(probs[b].float().numpy(), float(uniforms[step, b]))
            nxt = (forced[:, step] if forced is not None else out_tok[:, step]).long()
            nxt2 = torch.stack([nxt, nxt], 1).reshape(-1)
            x = O.prepare_gen_img_embeds(nxt2, w).unsqueeze(1)
            T = int(pos[-1]) + 2
            pos = torch.tensor([T - 1])
            key_ok = torch.cat([key_ok, torch.ones(R, 1, dtype=torch.bool)], 1)
            allowed = key_ok[:, None, :]
    return out_tok, out_p
