"""CPU oracle for the Janus-Pro SimPO training step (OSPO step 5).

TEST INFRASTRUCTURE ONLY.  This module is the checker, never the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it.  The product path (``ospo_amd``) never imports or calls it
and fails loudly when its HIP library is missing.

It is a plain-PyTorch (CPU) restatement of the reference algorithm, written
from the reference's behaviour, function by function:

* preprocess_batch            -> ``/root/reference/ospo/wrapper/train.py:219-279``
* concatenated_inputs         -> ``ospo/wrapper/train.py:282-314`` (+ trl
  ``pad_to_length`` semantics: pad the last dim only when shorter, a no-op on
  this path)
* concatenated_forward        -> ``ospo/wrapper/train.py:345-372``
* get_batch_logps             -> ``ospo/wrapper/train.py:375-396``
* simpo_loss                  -> ``ospo/wrapper/train.py:317-342``
* get_batch_loss_metrics      -> ``ospo/wrapper/train.py:399-445``
* LlamaForCausalLM decoder    -> HF transformers 4.38.2 (upstream, not in the
  reference tree; called at ``janus/models/modeling_vlm.py:219``): RMSNorm
  (fp32 variance, eps 1e-6), rotate-half RoPE (theta 1e4), causal attention
  with fp32 softmax, SwiGLU MLP, final RMSNorm == ``hidden_states[-1]``.
* LoRA linear                 -> peft 0.7.1 ``lora.Linear.forward`` (upstream,
  called from ``ospo/utils/model.py:50-60``): ``y = base(x) + B(A(drop(x)))*s``.
* gen_head (vision_head)      -> ``janus/models/modeling_vlm.py:36-51``
* prepare_gen_img_embeds      -> ``janus/models/modeling_vlm.py:263-264`` with
  ``MlpProjector`` mlp_gelu depth 2 (``janus/models/projector.py:39-45``).

Precision modes
---------------
``dtype=torch.float32``: everything fp32 -- must match the reference run in
fp32 (``train.py:53-54`` precision==32 branch) to fp32 round-off.
``dtype=torch.bfloat16``: the reference CPU bf16 path (bf16 weights and
activations, each op rounded to bf16 as eager PyTorch does), EXCEPT that
``log_softmax`` runs in fp32 on the bf16 logits -- what the GPU reference does
under autocast and what SURVEY §7 ("Hard parts") prescribes, because the CPU
bf16 log_softmax alone is off by ~2.5e-3 relative.

Parity pinning: ``tests/golden/make_golden.py`` runs the reference's own
``train.py`` functions (with dependency stubs) in this container and writes
``tests/golden/*.npz``; ``tests/test_oracle_golden.py`` checks this module
against them.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

LABEL_PAD = -100
PROJS_ATTN = ("q_proj", "k_proj", "v_proj", "o_proj")
PROJS_MLP = ("gate_proj", "up_proj", "down_proj")
PROJS = PROJS_ATTN + PROJS_MLP


@dataclass
class JanusDims:
    """Shapes of a Janus-Pro-like model (7B: L30 D4096 F11008 H32)."""
    n_layers: int = 30
    d_model: int = 4096
    d_ff: int = 11008
    n_heads: int = 32
    head_dim: int = 128
    vocab: int = 102400
    img_vocab: int = 16384
    img_embed: int = 8        # gen_embed dim (VQ codebook embed dim)
    gen_head_dim: int = 4096  # image_token_embed
    rope_theta: float = 10000.0
    rms_eps: float = 1e-6
    lora_r: int = 16
    lora_alpha: int = 32
    lora_dropout: float = 0.0

    @property
    def lora_scale(self) -> float:
        return self.lora_alpha / self.lora_r

    def proj_shape(self, p: str) -> Tuple[int, int]:
        d, f = self.d_model, self.d_ff
        return {"q_proj": (d, d), "k_proj": (d, d), "v_proj": (d, d), "o_proj": (d, d),
                "gate_proj": (f, d), "up_proj": (f, d), "down_proj": (d, f)}[p]


JANUS_PRO_7B = JanusDims()
JANUS_PRO_1B = JanusDims(n_layers=24, d_model=2048, d_ff=5632, n_heads=16, gen_head_dim=2048)


# --------------------------------------------------------------------------
# weights
# --------------------------------------------------------------------------
def init_weights(dims: JanusDims, seed: int = 0, dtype=torch.bfloat16, std: float = 0.02,
                 lora_seed: int = 1, lora_b_std: float = 1e-3) -> Dict[str, torch.Tensor]:
    """Seeded synthetic weights (HF init std 0.02; norms = 1; biases small).

    LoRA A is kaiming-uniform (peft default), LoRA B ~ N(0, lora_b_std) so that
    every gradient path is live."""
    g = torch.Generator().manual_seed(seed)

    def n(*shape, s=std):
        return (torch.randn(*shape, generator=g) * s).to(dtype)

    w: Dict[str, torch.Tensor] = {}
    D, Fd = dims.d_model, dims.d_ff
    w["embed_tokens"] = n(dims.vocab, D)
    for i in range(dims.n_layers):
        w[f"layers.{i}.input_layernorm"] = (1.0 + torch.randn(D, generator=g) * 0.05).to(dtype)
        w[f"layers.{i}.post_attention_layernorm"] = (1.0 + torch.randn(D, generator=g) * 0.05).to(dtype)
        for p in PROJS:
            w[f"layers.{i}.{p}"] = n(*dims.proj_shape(p))
    w["norm"] = (1.0 + torch.randn(D, generator=g) * 0.05).to(dtype)
    w["gen_head.w1"] = n(dims.gen_head_dim, D)
    w["gen_head.b1"] = n(dims.gen_head_dim)
    w["gen_head.w2"] = n(dims.img_vocab, dims.gen_head_dim)
    w["gen_head.b2"] = n(dims.img_vocab)
    w["gen_aligner.w1"] = n(D, dims.img_embed, s=0.3)
    w["gen_aligner.b1"] = n(D)
    w["gen_aligner.w2"] = n(D, D)
    w["gen_aligner.b2"] = n(D)
    w["gen_embed"] = n(dims.img_vocab, dims.img_embed, s=1.0)
    w.update(init_lora(dims, seed=lora_seed, dtype=dtype, b_std=lora_b_std))
    return w


def init_lora(dims: JanusDims, seed: int = 1, dtype=torch.bfloat16, b_std: float = 1e-3):
    g = torch.Generator().manual_seed(seed)
    w = {}
    r = dims.lora_r
    for i in range(dims.n_layers):
        for p in PROJS:
            out_f, in_f = dims.proj_shape(p)
            bound = 1.0 / math.sqrt(in_f)  # kaiming_uniform_(a=sqrt(5)) bound
            w[f"layers.{i}.{p}.lora_A"] = ((torch.rand(r, in_f, generator=g) * 2 - 1) * bound).to(dtype)
            w[f"layers.{i}.{p}.lora_B"] = (torch.randn(out_f, r, generator=g) * b_std).to(dtype)
    return w


def lora_names(dims: JanusDims) -> List[str]:
    names = []
    for i in range(dims.n_layers):
        for p in PROJS:
            names += [f"layers.{i}.{p}.lora_A", f"layers.{i}.{p}.lora_B"]
    return names


# --------------------------------------------------------------------------
# model pieces
# --------------------------------------------------------------------------
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """HF LlamaRMSNorm: fp32 variance, normalise, cast back, times weight."""
    dt = x.dtype
    h = x.to(torch.float32)
    var = h.pow(2).mean(-1, keepdim=True)
    h = h * torch.rsqrt(var + eps)
    return w * h.to(dt)


def rope_cos_sin(T: int, head_dim: int, theta: float, dtype) -> Tuple[torch.Tensor, torch.Tensor]:
    """HF LlamaRotaryEmbedding (default rope): fp32 freqs, cos/sin cast to x dtype."""
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    pos = torch.arange(T, dtype=torch.float32)
    freqs = torch.outer(pos, inv_freq)
    emb = torch.cat([freqs, freqs], dim=-1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


def rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat([-x[..., h:], x[..., :h]], dim=-1)


def apply_rope(x, cos, sin):
    return x * cos + rotate_half(x) * sin


def lora_linear(x, W, A, B, scale, dropout_p: float = 0.0, training: bool = True, mask=None, mx8: bool = False):
    """peft 0.7.1 lora.Linear.forward: base(x) + lora_B(lora_A(dropout(x))) * scaling.
    ``mask`` (bool, x's shape): an explicit keep mask (kept -> x / (1 - p) in x's dtype), so the
    HIP path's counter-based masks can be replayed; without it torch's F.dropout draws one.
    ``mx8``: the frozen base product in MXFP8 (BASELINE config 5, oracle/mx8_ref.py)."""
    if mx8:
        from oracle.mx8_ref import mx8_linear
        y = mx8_linear(x, W)
    else:
        y = F.linear(x, W)
    if A is None:
        return y
    if dropout_p > 0 and training and mask is not None:
        xd = torch.where(mask, (x.float() / (1.0 - dropout_p)).to(x.dtype), torch.zeros((), dtype=x.dtype))
    else:
        xd = F.dropout(x, p=dropout_p, training=training) if dropout_p > 0 else x
    return y + F.linear(F.linear(xd, A), B) * scale


def attention(q, k, v, scale):
    """Causal attention, eager HF style: scores in x dtype, fp32 softmax, cast back."""
    T = q.shape[-2]
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    mask = torch.full((T, T), float("-inf")).triu(1)
    s = s + mask.to(s.dtype)
    p = torch.softmax(s, dim=-1, dtype=torch.float32).to(q.dtype)
    return torch.matmul(p, v)


_GROUP = {"q_proj": "qkv", "k_proj": "qkv", "v_proj": "qkv", "o_proj": "o", "gate_proj": "gu", "up_proj": "gu",
          "down_proj": "down"}


def decoder_layer(x, w, i, dims: JanusDims, cos, sin, lora: bool = True, training=True, masks=None, mx8=False):
    S, T, D = x.shape
    H, hd = dims.n_heads, dims.head_dim
    s = dims.lora_scale
    pfx = f"layers.{i}."

    def lin(h, p):
        A = w.get(pfx + p + ".lora_A") if lora else None
        B = w.get(pfx + p + ".lora_B") if lora else None
        mk = masks.get((i, _GROUP[p])) if masks else None
        if mk is not None:
            mk = mk.reshape(h.shape)
        return lora_linear(h, w[pfx + p], A, B, s, dims.lora_dropout, training, mk, mx8)

    res = x
    h = rmsnorm(x, w[pfx + "input_layernorm"], dims.rms_eps)
    q = lin(h, "q_proj").view(S, T, H, hd).transpose(1, 2)
    k = lin(h, "k_proj").view(S, T, H, hd).transpose(1, 2)
    v = lin(h, "v_proj").view(S, T, H, hd).transpose(1, 2)
    q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
    o = attention(q, k, v, 1.0 / math.sqrt(hd)).transpose(1, 2).reshape(S, T, D)
    x = res + lin(o, "o_proj")
    res = x
    h = rmsnorm(x, w[pfx + "post_attention_layernorm"], dims.rms_eps)
    m = lin(F.silu(lin(h, "gate_proj")) * lin(h, "up_proj"), "down_proj")
    return res + m


def llama_hidden(inputs_embeds, w, dims: JanusDims, lora=True, training=True, masks=None, mx8=False):
    """LlamaModel forward over inputs_embeds -> final-normed hidden state
    (== ``outputs.hidden_states[-1]`` at train.py:356).  masks: {(layer, group): keep mask}."""
    T = inputs_embeds.shape[1]
    cos, sin = rope_cos_sin(T, dims.head_dim, dims.rope_theta, inputs_embeds.dtype)
    x = inputs_embeds
    for i in range(dims.n_layers):
        x = decoder_layer(x, w, i, dims, cos, sin, lora, training, masks, mx8)
    return rmsnorm(x, w["norm"], dims.rms_eps)


def gen_head(h, w):
    """vision_head (modeling_vlm.py:36-51): Linear -> GELU(erf) -> Linear."""
    z = F.gelu(F.linear(h, w["gen_head.w1"], w["gen_head.b1"]))
    return F.linear(z, w["gen_head.w2"], w["gen_head.b2"])


def prepare_gen_img_embeds(ids, w):
    """gen_aligner(gen_embed(ids)); MlpProjector mlp_gelu depth 2."""
    e = F.embedding(ids, w["gen_embed"])
    e = F.gelu(F.linear(e, w["gen_aligner.w1"], w["gen_aligner.b1"]))
    return F.linear(e, w["gen_aligner.w2"], w["gen_aligner.b2"])


# --------------------------------------------------------------------------
# the wrapper's algorithm
# --------------------------------------------------------------------------
def preprocess_batch(text_tokens: Sequence[torch.Tensor], chosen_ids: torch.Tensor,
                     rejected_ids: torch.Tensor, w, dtype):
    """train.py:219-279 with VQ encode replaced by given token ids.

    text_tokens: list of int [1, Lt_i]; chosen_ids / rejected_ids: int64 [B, N].
    Text rows are right-padded with ZERO embeddings to the batch max; text
    labels are -100; no attention mask reaches the model (train.py:272,276)."""
    B = len(text_tokens)
    embs = [F.embedding(t.long(), w["embed_tokens"]) for t in text_tokens]
    Lt = max(e.shape[1] for e in embs)
    D = embs[0].shape[-1]
    txt = torch.zeros(B, Lt, D, dtype=dtype)
    for i, e in enumerate(embs):
        txt[i, : e.shape[1]] = e[0]
    txt_lab = torch.full((B, Lt), LABEL_PAD, dtype=torch.long)
    c_img = prepare_gen_img_embeds(chosen_ids.long(), w)
    r_img = prepare_gen_img_embeds(rejected_ids.long(), w)
    return {
        "chosen_inputs_embeds": torch.cat([txt, c_img], 1),
        "chosen_labels": torch.cat([txt_lab, chosen_ids.long()], 1),
        "rejected_inputs_embeds": torch.cat([txt, r_img], 1),
        "rejected_labels": torch.cat([txt_lab, rejected_ids.long()], 1),
    }


def concatenated_inputs(batch):
    """train.py:282-314: cat chosen then rejected along dim 0 (pad_to_length no-op)."""
    return {
        "concatenated_inputs_embeds": torch.cat([batch["chosen_inputs_embeds"], batch["rejected_inputs_embeds"]], 0),
        "concatenated_labels": torch.cat([batch["chosen_labels"], batch["rejected_labels"]], 0),
    }


def get_batch_logps(logits, labels, average_log_prob=True, label_pad_token_id=LABEL_PAD):
    """train.py:375-396; log_softmax evaluated in fp32 (see module doc)."""
    if logits.shape[:-1] != labels.shape:
        raise ValueError("Logits (batch and sequence length dim) and labels must have the same shape.")
    labels = labels[:, 1:].clone()
    logits = logits[:, :-1, :]
    loss_mask = labels != label_pad_token_id
    labels[labels == label_pad_token_id] = 0
    lp = torch.gather(logits.float().log_softmax(-1), dim=2, index=labels.unsqueeze(2)).squeeze(2)
    if average_log_prob:
        return (lp * loss_mask).sum(-1) / loss_mask.sum(-1)
    return (lp * loss_mask).sum(-1)


def simpo_loss(c, r, beta=10.0, gamma_beta_ratio=0.5, label_smoothing=0.0, loss_type="sigmoid"):
    """train.py:317-342."""
    logits = (c - r) - gamma_beta_ratio
    if loss_type == "sigmoid":
        losses = -F.logsigmoid(beta * logits) * (1 - label_smoothing) - F.logsigmoid(-beta * logits) * label_smoothing
    elif loss_type == "hinge":
        losses = torch.relu(1 - beta * logits)
    else:
        raise ValueError(f"Unknown loss type: {loss_type}. Should be one of ['sigmoid', 'hinge']")
    return losses, beta * c.detach(), beta * r.detach()


@dataclass
class StepOut:
    loss: torch.Tensor
    chosen_logps: torch.Tensor
    rejected_logps: torch.Tensor
    losses: torch.Tensor
    metrics: Dict[str, float] = field(default_factory=dict)
    lora_grads: Optional[Dict[str, torch.Tensor]] = None


def simpo_step(text_tokens, chosen_ids, rejected_ids, w, dims: JanusDims, dtype=torch.bfloat16,
               beta=10.0, gamma_beta_ratio=0.5, label_smoothing=0.0, loss_type="sigmoid",
               backward: bool = True, training: bool = True, dropout_masks=None, mx8: bool = False,
               sft_weight: float = 0.0) -> StepOut:
    """One SimPO step: preprocess -> concatenated forward -> logps -> loss
    (train.py:399-445, + sft_weight * CE on the chosen logits, :421-430) -> backward to the
    LoRA tensors (autograd)."""
    w = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in w.items()}
    lnames = [k for k in w if ".lora_" in k]
    if backward:
        for k in lnames:
            w[k] = w[k].detach().clone().requires_grad_(True)
    with torch.no_grad():
        batch = preprocess_batch(text_tokens, chosen_ids, rejected_ids, w, dtype)
    cb = concatenated_inputs(batch)
    B = chosen_ids.shape[0]
    with torch.set_grad_enabled(backward):
        h = llama_hidden(cb["concatenated_inputs_embeds"], w, dims, lora=True, training=training,
                         masks=dropout_masks, mx8=mx8)
        logits = gen_head(h, w)
        logps = get_batch_logps(logits, cb["concatenated_labels"])
        c, r = logps[:B], logps[B:]
        losses, cr, rr = simpo_loss(c, r, beta, gamma_beta_ratio, label_smoothing, loss_type)
        loss = losses.mean()
        sft_loss = None
        if sft_weight > 0.0:  # train.py:421-428: CrossEntropyLoss (ignore -100) on logits[:, :-1] vs labels[:, 1:]
            cl = logits[:B, :-1, :].float()
            lab = cb["concatenated_labels"][:B, 1:]
            sft_loss = torch.nn.functional.cross_entropy(cl.reshape(-1, cl.shape[-1]), lab.reshape(-1),
                                                         ignore_index=LABEL_PAD)
            loss = sft_weight * sft_loss + loss
    metrics = {
        "rewards/chosen": cr.mean().item(), "rewards/rejected": rr.mean().item(),
        "rewards/accuracies": (cr > rr).float().mean().item(),
        "rewards/margins": (cr - rr).mean().item(),
        "logps/chosen": c.detach().mean().item(), "logps/rejected": r.detach().mean().item(),
        "logits/chosen": logits[:B].detach().float().mean().item(),
        "logits/rejected": logits[B:].detach().float().mean().item(),
    }
    if sft_loss is not None:
        metrics["sft_loss"] = sft_loss.item()
        # train.py:422 rebinds policy_chosen_logits to [..., :-1, :] before the logging at :442
        metrics["logits/chosen"] = logits[:B, :-1].detach().float().mean().item()
    grads = None
    if backward:
        loss.backward()
        grads = {k: w[k].grad.detach().clone() for k in lnames}
    return StepOut(loss.detach(), c.detach(), r.detach(), losses.detach(), metrics, grads)


# --------------------------------------------------------------------------
# optimizer semantics (PL clip 1.0 -> torch AdamW on the LoRA tensors)
# --------------------------------------------------------------------------
def clip_and_adamw(params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor], state: dict,
                   lr=4e-5, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.0, max_norm=1.0):
    """``compute_total_grad_norm`` (train.py:459-469) + PL ``gradient_clip_val``
    (utils/train.py:30 -> torch clip_grad_norm_) + ``AdamW`` (train.py:108-115).
    Returns the pre-clip total norm.  Uses torch.optim.AdamW itself so the
    update is the reference library's own arithmetic."""
    names = sorted(params)
    ps = [params[k] for k in names]
    for p, k in zip(ps, names):
        p.grad = grads[k].to(p.dtype).clone()
    total = torch.sqrt(sum((p.grad.float() ** 2).sum() for p in ps))
    torch.nn.utils.clip_grad_norm_(ps, max_norm)
    if "opt" not in state:
        state["opt"] = torch.optim.AdamW(ps, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                         foreach=False)
    state["opt"].step()
    return total.item()
