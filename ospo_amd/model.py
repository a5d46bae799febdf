"""Model assembly (mirrors ospo/utils/model.py:13-71).

``get_model(mode='train', config=...)`` -> ``(model, chat_processor, image_processor, tokenizer)``
like the reference.  ``model`` is a ``JanusProPolicy``: the frozen Janus-Pro
generation path (LLM + gen_head + gen_aligner + gen_embed) resident on the GPU
with peft-style LoRA on q,k,v,o,gate,up,down (``LoraConfig(r, alpha, targets,
dropout)``, model.py:50-57) inside ``SimPOEngine``.

Weights: a Janus-Pro HF checkpoint directory (``config.model.model_path``:
``*.safetensors`` or ``pytorch_model*.bin`` shards, loaded with loaders that execute
nothing from the file); a missing weight is an error.  Random-init weights of the
named architecture (``config.model.arch``: janus-pro-7b | janus-pro-1b) only with
``model.synthetic: true`` -- what this offline container runs.
"""
from __future__ import annotations

import glob
import json
import os
import sys
from typing import Dict, Optional

import torch

from .config import get
from .data import ChatProcessor, VLMImageProcessor, load_tokenizer
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


def _checkpoint_files(model_path: str):
    """The weight shards of an HF checkpoint directory: *.safetensors, else pytorch_model*.bin."""
    st = sorted(glob.glob(os.path.join(model_path, "*.safetensors")))
    return st if st else sorted(glob.glob(os.path.join(model_path, "pytorch_model*.bin")))


def _iter_state(path: str):
    """Tensors of one shard through loaders that execute nothing from the file."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        yield from load_file(path).items()
    else:
        yield from torch.load(path, map_location="cpu", weights_only=True, mmap=True).items()


def expected_weight_names(dims: ModelDims):
    names = ["embed_tokens", "norm", "gen_head.w1", "gen_head.b1", "gen_head.w2", "gen_head.b2", "gen_aligner.w1",
             "gen_aligner.b1", "gen_aligner.w2", "gen_aligner.b2", "gen_embed"]
    for i in range(dims.n_layers):
        names += [f"layers.{i}.{leaf}" for leaf in ["input_layernorm", "post_attention_layernorm"] + TARGETS]
    return names


def load_janus_checkpoint(model_path: str, dims: Optional[ModelDims] = None):
    """(frozen weights under engine names, VQ weights ``encoder.* / quant_conv.* / quantize.*``)
    from a Janus-Pro HF checkpoint directory (safetensors or .bin shards).  Raises when the
    directory holds no shards or misses a weight the path needs."""
    files = _checkpoint_files(model_path)
    if not files:
        raise FileNotFoundError(f"{model_path}: no *.safetensors or pytorch_model*.bin shards")
    w, vq = {}, {}
    for f in files:
        for k, v in _iter_state(f):
            ours = hf_to_ours(k)
            if ours is not None:
                w[ours] = v.to(torch.bfloat16)
            elif k.startswith("gen_vision_model."):
                k2 = k[len("gen_vision_model."):]
                if k2.startswith(("encoder.", "quant_conv.", "quantize.embedding")):
                    vq[k2] = v.float()
    if dims is not None:
        missing = [n for n in expected_weight_names(dims) if n not in w]
        if missing:
            raise KeyError(f"{model_path}: {len(missing)} weights missing, e.g. {missing[:4]}")
    return w, vq


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
    """The trainable Janus-Pro generation policy (LoRA adapters on the LLM) and its frozen VQ
    tokenizer (``gen_vision_model.encode``, run on the GPU by ``ospo_amd.vq.VQEncoder``)."""

    def __init__(self, engine: SimPOEngine, lora_cfg: dict, synthetic: bool, vq_weights=None, vq_seed: int = 0):
        self.engine = engine
        self.lora_cfg = lora_cfg
        self.synthetic = synthetic
        self._vq_weights, self._vq_seed, self._vq = vq_weights, vq_seed, None
        # flat LoRA params as an autograd leaf: PolicyLogps hangs the backward on it
        self.lora_anchor = torch.zeros(1, device=engine.device, requires_grad=True)

    @property
    def device(self):
        return self.engine.device

    @property
    def gen_vision_model(self):
        """The VQ-16 encoder, built on first use (checkpoint ``gen_vision_model.*`` weights, or the
        seeded synthetic ones of a synthetic model)."""
        if self._vq is None:
            from .vq import VQEncoder, synthetic_vq_weights
            if self._vq_weights is None and not self.synthetic:
                raise RuntimeError("the checkpoint has no gen_vision_model weights: pixel batches cannot be encoded")
            w = self._vq_weights if self._vq_weights is not None else synthetic_vq_weights(self._vq_seed)
            self._vq = VQEncoder(w, device=self.engine.device)
            self._vq_weights = None
        return self._vq

    def vq_encode(self, pixels: torch.Tensor) -> torch.Tensor:
        """f32 [n, 3, 384, 384] -> int32 [n, 576] VQ ids on the device (fp32 encode: the ids of the
        reference's vq_model.py run in fp32, not of its bf16 run)."""
        return self.gen_vision_model.encode(pixels)

    def named_lora_parameters(self):
        return self.engine.lora_tensors()

    def train(self):
        return self


def get_model(mode: str = "train", dtype=torch.bfloat16, config=None, device=None, max_pairs: Optional[int] = None,
              max_text_len: int = 128, n_img_tokens: int = 576, seed: int = 0):
    """ospo/utils/model.py:13-71.  Weights come from ``model.model_path`` (an HF Janus-Pro
    checkpoint directory: safetensors or .bin shards); random-init weights of ``model.arch`` only
    when ``model.synthetic: true`` is set (no checkpoint exists offline).  Returns
    ``(model, chat_processor, image_processor, tokenizer)`` like the reference."""
    if mode not in ("generate", "train"):
        raise ValueError(f"Invalid mode: {mode}. Choose either 'generate' or 'train'.")
    if mode == "generate":
        raise NotImplementedError("step-3 generation runs through ospo_amd.generate.T2IGenerator")
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
    synthetic = bool(get(config, "model.synthetic", False))
    vq_w = None
    if synthetic:
        arch = str(get(config, "model.arch", "janus-pro-7b")).lower()
        base = {"janus-pro-7b": JANUS_PRO_7B, "janus-pro-1b": JANUS_PRO_1B}.get(arch)
        if base is None:
            raise ValueError(f"unknown model.arch {arch}")
        over = get(config, "model.override", {}) or {}
        dims = ModelDims(**{**base.__dict__, **over, "lora_r": r, "lora_alpha": alpha})
        print(f"[ospo_amd] model.synthetic: random-init {dims.n_layers}-layer d={dims.d_model} weights", file=sys.stderr)
        w = synthetic_weights(dims, device, seed=seed, lora_seed=seed + 1)
    else:
        if not model_path or not os.path.isdir(model_path):
            raise FileNotFoundError(f"model.model_path {model_path!r} is not a checkpoint directory "
                                    "(set model.synthetic: true for random-init weights)")
        dims = dims_from_checkpoint(model_path)
        if dims is None:
            raise FileNotFoundError(f"{model_path}: no config.json")
        dims = ModelDims(**{**dims.__dict__, "lora_r": r, "lora_alpha": alpha})
        w, vq_w = load_janus_checkpoint(model_path, dims)
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
    # the reference loads tokenizer + processor from model_path (ospo/utils/model.py:26-28)
    tok_path = get(config, "model.tokenizer_path") or (None if synthetic else model_path)
    tokenizer = load_tokenizer(tok_path, vocab=dims.vocab)
    lora_cfg = {"lora_rank": r, "lora_alpha": alpha, "lora_dropout": dropout, "target_modules": targets}
    model = JanusProPolicy(engine, lora_cfg, synthetic, vq_weights=vq_w, vq_seed=seed)
    return model, ChatProcessor(tokenizer), VLMImageProcessor(), tokenizer
