"""Model assembly (mirrors ospo/utils/model.py:13-71).

``get_model(mode='train', config=...)`` -> ``(model, chat_processor, image_processor, tokenizer)``
like the reference.  ``model`` is a ``JanusProPolicy``: the frozen Janus-Pro
generation path (LLM + gen_head + gen_aligner + gen_embed) resident on the GPU
with peft-style LoRA on q,k,v,o,gate,up,down (``LoraConfig(r, alpha, targets,
dropout)``, model.py:50-57) inside ``SimPOEngine``.

Weights: a Janus-Pro HF checkpoint directory (``config.model.model_path`` with
``*.safetensors``; safe loader only) when present; otherwise -- as in this
offline container -- random-init weights of the named architecture
(``config.model.arch``: janus-pro-7b | janus-pro-1b), with a log line saying so.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional

import torch

from .config import get
from .data import load_tokenizer
from .engine import JANUS_PRO_1B, JANUS_PRO_7B, ModelDims, SimPOEngine, synthetic_weights

TARGETS = ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"]


def hf_to_ours(k: str) -> Optional[str]:
    """Janus-Pro MultiModalityCausalLM state-dict key -> engine weight name."""
    if k.startswith("language_model.model.layers."):
        parts = k.split(".")
        i, leaf = parts[3], parts[-2]
        if leaf in ("input_layernorm", "post_attention_layernorm"):
            return f"layers.{i}.{leaf}"
        if leaf in TARGETS:
            return f"layers.{i}.{leaf}"
        return None
    table = {
        "language_model.model.embed_tokens.weight": "embed_tokens",
        "language_model.model.norm.weight": "norm",
        "gen_head.output_mlp_projector.weight": "gen_head.w1", "gen_head.output_mlp_projector.bias": "gen_head.b1",
        "gen_head.vision_head.weight": "gen_head.w2", "gen_head.vision_head.bias": "gen_head.b2",
        "gen_aligner.layers.0.weight": "gen_aligner.w1", "gen_aligner.layers.0.bias": "gen_aligner.b1",
        "gen_aligner.layers.2.weight": "gen_aligner.w2", "gen_aligner.layers.2.bias": "gen_aligner.b2",
        "gen_embed.weight": "gen_embed",
    }
    return table.get(k)


def load_janus_checkpoint(model_path: str) -> Optional[Dict[str, torch.Tensor]]:
    files = sorted(glob.glob(os.path.join(model_path or "", "*.safetensors")))
    if not files:
        return None
    from safetensors.torch import load_file
    w = {}
    for f in files:
        for k, v in load_file(f).items():
            ours = hf_to_ours(k)
            if ours is not None:
                w[ours] = v.to(torch.bfloat16)
    return w


def dims_from_checkpoint(model_path: str) -> Optional[ModelDims]:
    p = os.path.join(model_path or "", "config.json")
    if not os.path.exists(p):
        return None
    c = json.load(open(p))
    lc = c.get("language_config", c)
    ghp = c.get("gen_head_config", {}).get("params", {})
    return ModelDims(n_layers=lc["num_hidden_layers"], d_model=lc["hidden_size"], d_ff=lc["intermediate_size"],
                     n_heads=lc["num_attention_heads"], head_dim=lc["hidden_size"] // lc["num_attention_heads"],
                     vocab=lc["vocab_size"], img_vocab=ghp.get("image_token_size", 16384),
                     img_embed=c.get("gen_vision_config", {}).get("params", {}).get("n_embed", 8),
                     gen_head_dim=ghp.get("image_token_embed", lc["hidden_size"]),
                     rope_theta=lc.get("rope_theta", 10000.0), rms_eps=lc.get("rms_norm_eps", 1e-6))


class JanusProPolicy:
    """The trainable Janus-Pro generation policy (LoRA adapters on the LLM)."""

    def __init__(self, engine: SimPOEngine, lora_cfg: dict, synthetic: bool):
        self.engine = engine
        self.lora_cfg = lora_cfg
        self.synthetic = synthetic
        # flat LoRA params as an autograd leaf: PolicyLogps hangs the backward on it
        self.lora_anchor = torch.zeros(1, device=engine.device, requires_grad=True)

    @property
    def device(self):
        return self.engine.device

    def named_lora_parameters(self):
        return self.engine.lora_tensors()

    def train(self):
        return self


def get_model(mode: str = "train", dtype=torch.bfloat16, config=None, device=None, max_pairs: Optional[int] = None,
              max_text_len: int = 128, n_img_tokens: int = 576, seed: int = 0):
    if mode not in ("generate", "train"):
        raise ValueError(f"Invalid mode: {mode}. Choose either 'generate' or 'train'.")
    if mode == "generate":
        raise NotImplementedError("step-3 generation is not on the built path (SURVEY §8f rank 2)")
    if dtype != torch.bfloat16:
        raise NotImplementedError("the MI355X path trains in bf16 (configs/step5.yaml precision: bf16)")
    if not (get(config, "use_lora", False) or get(config, "use_peft", False)):
        raise NotImplementedError("only the LoRA (use_peft/use_lora: true) path is built (SURVEY §2)")
    targets = list(get(config, "lora.target_modules", TARGETS))
    if sorted(targets) != sorted(TARGETS):
        raise NotImplementedError(f"LoRA target_modules must be {TARGETS}")
    r = int(get(config, "lora.lora_rank", 32))
    alpha = int(get(config, "lora.lora_alpha", 64))
    dropout = float(get(config, "lora.lora_dropout", 0.0) or 0.0)
    if dropout > 0 and get(config, "lora.ignore_dropout", False):
        print(f"[ospo_amd] lora_dropout={dropout} ignored (lora.ignore_dropout=true): adapters run without dropout")
        dropout = 0.0
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    model_path = get(config, "model.model_path")
    w = load_janus_checkpoint(model_path)
    dims = dims_from_checkpoint(model_path)
    synthetic = w is None
    if dims is None:
        arch = str(get(config, "model.arch", "janus-pro-7b")).lower()
        base = {"janus-pro-7b": JANUS_PRO_7B, "janus-pro-1b": JANUS_PRO_1B}.get(arch)
        if base is None:
            raise ValueError(f"unknown model.arch {arch}")
        over = get(config, "model.override", {}) or {}
        dims = ModelDims(**{**base.__dict__, **over})
    dims = ModelDims(**{**dims.__dict__, "lora_r": r, "lora_alpha": alpha})
    if synthetic:
        print(f"[ospo_amd] no Janus-Pro checkpoint at {model_path!r}: random-init {dims.n_layers}-layer "
              f"d={dims.d_model} weights (synthetic)")
        w = synthetic_weights(dims, device, seed=seed, lora_seed=seed + 1)
    else:
        # peft init: lora_A kaiming-uniform, lora_B zeros (ospo/utils/model.py:50-60)
        import math
        g = torch.Generator().manual_seed(seed + 1)
        for i in range(dims.n_layers):
            for p in TARGETS:
                out_f, in_f = w[f"layers.{i}.{p}"].shape
                b = 1.0 / math.sqrt(in_f)
                w[f"layers.{i}.{p}.lora_A"] = ((torch.rand(r, in_f, generator=g) * 2 - 1) * b).to(torch.bfloat16)
                w[f"layers.{i}.{p}.lora_B"] = torch.zeros(out_f, r, dtype=torch.bfloat16)
    bs = max_pairs or int(get(config, "dataset.train.batch_size", 4))
    # BASELINE config 5: MXFP8 frozen decoder Linears (model.linear_dtype: mx8, or experiment.precision: fp8)
    linear_dtype = str(get(config, "model.linear_dtype", "bf16") or "bf16").lower()
    if str(get(config, "experiment.precision", "bf16")).lower() in ("fp8", "mx8"):
        linear_dtype = "mx8"
    engine = SimPOEngine(dims, w, device=device, max_pairs=bs, max_text_len=max_text_len, n_img_tokens=n_img_tokens,
                         lora_dropout=dropout, dropout_seed=seed, linear_dtype=linear_dtype)
    del w
    tokenizer = load_tokenizer(get(config, "model.tokenizer_path"), vocab=dims.vocab)
    lora_cfg = {"lora_rank": r, "lora_alpha": alpha, "lora_dropout": dropout, "target_modules": targets}
    return JanusProPolicy(engine, lora_cfg, synthetic), None, None, tokenizer
