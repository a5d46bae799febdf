"""Generate golden vectors from the REFERENCE's own SimPO code (this container only).

Run:  python tests/golden/make_golden.py          (needs /root/reference)

What runs is the reference's ``ospo/wrapper/train.py`` (``JanusProTrainWrapper``:
``preprocess_batch`` -> ``get_batch_loss_metrics`` -> ``get_batch_logps`` ->
``simpo_loss``), the reference's ``janus/models/projector.py`` (``MlpProjector``)
and ``vision_head`` (``janus/models/modeling_vlm.py:36-51``, exec'd from its source
because the module itself does not import under transformers 5.15),
over the container's ``transformers.LlamaForCausalLM`` (eager attention) with a
restated peft-0.7.1 LoRA linear.  Third-party packages absent from the container
(pytorch_lightning, pyrootutils, omegaconf, attrdict, trl) are replaced by stubs
that do not touch arithmetic; trl's ``pad_to_length`` is restated with trl
semantics (pad the last dim only when it is shorter).

VQ encode is bypassed: the "image tensors" handed to ``preprocess_batch`` carry
the token ids and a fake ``gen_vision_model.encode`` returns them as
``output[2][2]`` (the int path of train.py:253-258 is exercised unchanged).

Outputs (``tests/golden/*.npz``, data only -- never reference source):
  logps_kat.npz        get_batch_logps / simpo_loss known-answer vectors
  step_tiny_weights.npz  D=256 L=2 model weights (bf16 bits), shared by:
  step_tiny_fp32.npz   2 ragged pairs, N=64, reference run in fp32
  step_tiny_bf16.npz   same inputs, bf16 model (reference CPU bf16 path)
  step_tiny_sft_fp32.npz  the tiny fp32 step with algo.sft_weight = 0.5 (CE on the
                       chosen logits, train.py:421-430)
  step_1b2l_bf16.npz   Janus-Pro-1B dims, 2 layers, 4 pairs from train.json
                       (synthetic prompt ids), N=64; weights regenerated from a
                       seed by ``oracle.simpo_ref.init_weights`` (checksum kept)
"""
from __future__ import annotations

import ast
import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import simpo_ref as O  # noqa: E402


# ----------------------------------------------------------------------------- stubs
class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    __setattr__ = dict.__setitem__

    @classmethod
    def from_nested(cls, d):
        return cls({k: cls.from_nested(v) for k, v in d.items()}) if isinstance(d, dict) else d


def install_stubs():
    pl = types.ModuleType("pytorch_lightning")

    class LightningModule(nn.Module):
        logged: dict = {}

        @property
        def device(self):
            return torch.device("cpu")

        def log(self, k, v, **kw):
            LightningModule.logged[k] = float(v)

        def log_dict(self, d, **kw):
            for k, v in d.items():
                self.log(k, v)

    pl.LightningModule = LightningModule
    pl.Trainer = object
    pl.seed_everything = lambda *a, **k: None
    strat = types.ModuleType("pytorch_lightning.strategies")
    strat.DDPStrategy = object
    pl.strategies = strat
    sys.modules["pytorch_lightning"] = pl
    sys.modules["pytorch_lightning.strategies"] = strat
    pr = types.ModuleType("pyrootutils")
    pr.setup_root = lambda *a, **k: None
    sys.modules["pyrootutils"] = pr
    oc = types.ModuleType("omegaconf")
    oc.OmegaConf = object
    sys.modules["omegaconf"] = oc
    ad = types.ModuleType("attrdict")
    ad.AttrDict = AttrDict
    sys.modules["attrdict"] = ad
    trl = types.ModuleType("trl")
    trl_tr = types.ModuleType("trl.trainer")
    trl_ut = types.ModuleType("trl.trainer.utils")

    def pad_to_length(tensor, length, pad_value, dim=-1):
        if tensor.size(dim) >= length:
            return tensor
        pad_size = list(tensor.shape)
        pad_size[dim] = length - tensor.size(dim)
        return torch.cat([tensor, pad_value * torch.ones(*pad_size, dtype=tensor.dtype, device=tensor.device)], dim=dim)

    trl_ut.pad_to_length = pad_to_length
    for n, m in (("trl", trl), ("trl.trainer", trl_tr), ("trl.trainer.utils", trl_ut)):
        sys.modules[n] = m
    return LightningModule


def load_ref_module(name, relpath):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_vision_head():
    src = open(os.path.join(REF, "janus/models/modeling_vlm.py")).read()
    tree = ast.parse(src)
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "vision_head"][0]
    ns = {"torch": torch}
    exec(compile(ast.Module(body=[cls], type_ignores=[]), "modeling_vlm.py", "exec"), ns)
    return ns["vision_head"]


# ----------------------------------------------------------------------------- model
class LoraLinear(nn.Module):
    """peft 0.7.1 lora.Linear (non-merged forward), restated."""

    def __init__(self, base: nn.Linear, r, alpha):
        super().__init__()
        self.base_layer = base
        self.lora_A = nn.Linear(base.in_features, r, bias=False)
        self.lora_B = nn.Linear(r, base.out_features, bias=False)
        self.scaling = alpha / r

    def forward(self, x):
        prev = x.dtype
        result = self.base_layer(x)
        x = x.to(self.lora_A.weight.dtype)
        result = result + self.lora_B(self.lora_A(x)) * self.scaling
        return result.to(prev)


class LMWrap(nn.Module):
    """Mirrors the peft attribute chain: language_model.model -> LlamaForCausalLM."""

    def __init__(self, llama):
        super().__init__()
        self.model = llama

    def get_input_embeddings(self):
        return self.model.get_input_embeddings()


class FakeVQ(nn.Module):
    def __init__(self):
        super().__init__()
        self.dummy = nn.Parameter(torch.zeros(1), requires_grad=False)

    def encode(self, x):
        return None, (None, None, None), (None, None, x.view(-1).long())


class JanusLike(nn.Module):
    def __init__(self, dims: O.JanusDims, w, dtype, MlpProjector, vision_head):
        super().__init__()
        from transformers import LlamaConfig, LlamaForCausalLM
        cfg = LlamaConfig(vocab_size=dims.vocab, hidden_size=dims.d_model, intermediate_size=dims.d_ff,
                          num_hidden_layers=dims.n_layers, num_attention_heads=dims.n_heads,
                          num_key_value_heads=dims.n_heads, rms_norm_eps=dims.rms_eps,
                          max_position_embeddings=4096, rope_theta=dims.rope_theta,
                          attn_implementation="eager", tie_word_embeddings=False)
        llama = LlamaForCausalLM(cfg)
        sd = llama.state_dict()
        with torch.no_grad():
            sd["model.embed_tokens.weight"].copy_(w["embed_tokens"])
            sd["model.norm.weight"].copy_(w["norm"])
            for i in range(dims.n_layers):
                for nm in ("input_layernorm", "post_attention_layernorm"):
                    sd[f"model.layers.{i}.{nm}.weight"].copy_(w[f"layers.{i}.{nm}"])
                for p in O.PROJS:
                    grp = "self_attn" if p in O.PROJS_ATTN else "mlp"
                    sd[f"model.layers.{i}.{grp}.{p}.weight"].copy_(w[f"layers.{i}.{p}"])
        llama.load_state_dict(sd)
        for i in range(dims.n_layers):
            layer = llama.model.layers[i]
            for p in O.PROJS:
                grp = layer.self_attn if p in O.PROJS_ATTN else layer.mlp
                ll = LoraLinear(getattr(grp, p), dims.lora_r, dims.lora_alpha)
                with torch.no_grad():
                    ll.lora_A.weight.copy_(w[f"layers.{i}.{p}.lora_A"])
                    ll.lora_B.weight.copy_(w[f"layers.{i}.{p}.lora_B"])
                setattr(grp, p, ll)
        self.language_model = LMWrap(llama)
        self.gen_head = vision_head(AttrDict(n_embed=dims.d_model, image_token_embed=dims.gen_head_dim,
                                             image_token_size=dims.img_vocab))
        self.gen_aligner = MlpProjector(AttrDict(projector_type="mlp_gelu", input_dim=dims.img_embed,
                                                 n_embed=dims.d_model, depth=2))
        self.gen_embed = nn.Embedding(dims.img_vocab, dims.img_embed)
        with torch.no_grad():
            self.gen_head.output_mlp_projector.weight.copy_(w["gen_head.w1"])
            self.gen_head.output_mlp_projector.bias.copy_(w["gen_head.b1"])
            self.gen_head.vision_head.weight.copy_(w["gen_head.w2"])
            self.gen_head.vision_head.bias.copy_(w["gen_head.b2"])
            self.gen_aligner.layers[0].weight.copy_(w["gen_aligner.w1"])
            self.gen_aligner.layers[0].bias.copy_(w["gen_aligner.b1"])
            self.gen_aligner.layers[2].weight.copy_(w["gen_aligner.w2"])
            self.gen_aligner.layers[2].bias.copy_(w["gen_aligner.b2"])
            self.gen_embed.weight.copy_(w["gen_embed"])
        self.to(dtype)
        self.gen_vision_model = FakeVQ()  # stays fp32 so the ids survive the dtype cast at train.py:247-251
        for n, p in self.named_parameters():
            p.requires_grad_(".lora_" in n)

    @property
    def dtype(self):
        return self.gen_embed.weight.dtype

    def prepare_gen_img_embeds(self, image_ids):  # modeling_vlm.py:263-264
        return self.gen_aligner(self.gen_embed(image_ids))


# ----------------------------------------------------------------------------- runners
def run_reference_step(dims, w, dtype, text_tokens, chosen_ids, rejected_ids, algo):
    install_stubs()
    sys.path.insert(0, REF)
    train_mod = load_ref_module("ospo_ref_train", "ospo/wrapper/train.py")
    proj_mod = load_ref_module("janus_ref_projector", "janus/models/projector.py")
    vision_head = load_vision_head()
    model = JanusLike(dims, w, dtype, proj_mod.MlpProjector, vision_head)
    model.language_model.model.config.output_hidden_states = True  # train.py:50
    model.train()
    cfg = AttrDict.from_nested({"algo": algo, "tokenizer": {"label_pad_token_id": -100, "max_length": 2048,
                                                             "max_prompt_length": 1024}})
    tok = types.SimpleNamespace(pad_token_id=100002)
    wrapper = train_mod.JanusProTrainWrapper(cfg, model, None, None, tok)
    B = len(text_tokens)
    batch = ([f"{i:07d}" for i in range(B)], list(text_tokens),
             [chosen_ids[i:i + 1].float() for i in range(B)], [rejected_ids[i:i + 1].float() for i in range(B)])
    sys.modules["pytorch_lightning"].LightningModule.logged.clear()
    pre = wrapper.preprocess_batch(batch)
    # capture per-seq logps through the reference's own concatenated_forward
    c, r, cl, rl, _ = wrapper.concatenated_forward(pre)
    loss = wrapper.get_batch_loss_metrics(pre)
    loss.backward()
    logged = dict(sys.modules["pytorch_lightning"].LightningModule.logged)
    grads = {}
    for n, p in model.named_parameters():
        if ".lora_" in n:
            # model.layers.{i}.self_attn.q_proj.lora_A.weight -> layers.{i}.q_proj.lora_A
            parts = n.split(".")
            i = parts[parts.index("layers") + 1]
            proj = [x for x in parts if x.endswith("_proj")][0]
            ab = "lora_A" if "lora_A" in parts else "lora_B"
            # concatenated_forward above ran a second graph; grads accumulate from
            # get_batch_loss_metrics' backward only (c/r graph never backpropagated)
            grads[f"layers.{i}.{proj}.{ab}"] = p.grad.detach().float().clone()
    return {"chosen_logps": c.detach().float(), "rejected_logps": r.detach().float(),
            "loss": loss.detach().float(), "logged": logged, "grads": grads,
            "inputs_embeds": pre["chosen_inputs_embeds"].detach().float()}


def bf16_bits(t):
    return t.to(torch.bfloat16).view(torch.int16).numpy().astype(np.uint16)


def synth_prompt_ids(prompt: str, vocab: int):
    """Deterministic synthetic ids for the DeepSeek SFT prompt (tokenizer absent):
    BOS + one id per whitespace piece of "User: {p}\\n\\nAssistant:" + <begin_of_image>."""
    text = f"User: {prompt}\n\nAssistant:"
    ids = [vocab - 2]  # BOS stand-in
    for piece in text.split():
        ids.append(int(hashlib.md5(piece.encode()).hexdigest(), 16) % (vocab - 3))
    ids.append(vocab - 1)  # <begin_of_image> stand-in
    return torch.tensor([ids], dtype=torch.int32)


def weights_checksum(w):
    h = hashlib.sha256()
    for k in sorted(w):
        h.update(k.encode())
        h.update(w[k].float().numpy().tobytes())
    return h.hexdigest()


def save_step(path, dims, w, text_tokens, chosen, rejected, out, algo, store_weights=True, seed=None):
    d = {}
    Lt = [t.shape[1] for t in text_tokens]
    maxL = max(Lt)
    tt = np.full((len(text_tokens), maxL), -1, dtype=np.int32)
    for i, t in enumerate(text_tokens):
        tt[i, : t.shape[1]] = t[0].numpy()
    d["text_tokens"] = tt
    d["text_lens"] = np.array(Lt, dtype=np.int32)
    d["chosen_ids"] = chosen.numpy().astype(np.int32)
    d["rejected_ids"] = rejected.numpy().astype(np.int32)
    d["dims"] = np.array(json.dumps(dims.__dict__))
    d["algo"] = np.array(json.dumps(algo))
    if store_weights:
        for k, v in w.items():
            d["w::" + k] = v.float().numpy() if v.dtype == torch.float32 else bf16_bits(v)
        d["weights_dtype"] = np.array("float32" if next(iter(w.values())).dtype == torch.float32 else "bfloat16")
    else:
        d["weights_seed"] = np.array(seed)
        d["weights_sha256"] = np.array(weights_checksum(w))
    d["out::chosen_logps"] = out["chosen_logps"].numpy()
    d["out::rejected_logps"] = out["rejected_logps"].numpy()
    d["out::loss"] = out["loss"].numpy()
    d["out::logged"] = np.array(json.dumps(out["logged"]))
    for k, v in out["grads"].items():
        d["grad::" + k] = v.numpy()
    np.savez_compressed(path, **d)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


def make_logps_kat():
    install_stubs()
    sys.path.insert(0, REF)
    train_mod = load_ref_module("ospo_ref_train", "ospo/wrapper/train.py")
    g = torch.Generator().manual_seed(123)
    S, T, V = 4, 24, 16384
    logits = (torch.randn(S, T, V, generator=g) * 2.0).to(torch.bfloat16)
    labels = torch.randint(0, V, (S, T), generator=g)
    lt = [5, 8, 3, 8]
    for s in range(S):
        labels[s, : lt[s]] = -100
    w = train_mod.JanusProTrainWrapper.__new__(train_mod.JanusProTrainWrapper)
    nn.Module.__init__(w)
    w.label_pad_token_id = -100
    avg = w.get_batch_logps(logits.float(), labels, average_log_prob=True)
    tot = w.get_batch_logps(logits.float(), labels, average_log_prob=False)
    c = torch.linspace(-9.8, -9.2, 6)
    r = torch.linspace(-9.5, -9.6, 6)
    combos = [(10.0, 0.5, 0.0, "sigmoid"), (2.0, 0.0, 0.1, "sigmoid"), (10.0, 0.5, 0.0, "hinge"),
              (1.0, 0.3, 0.0, "hinge")]
    d = {"logits_bf16": bf16_bits(logits), "labels": labels.numpy().astype(np.int64),
         "logps_avg": avg.numpy(), "logps_sum": tot.numpy(), "c": c.numpy(), "r": r.numpy()}
    for j, (beta, gbr, ls, lt_) in enumerate(combos):
        w.beta, w.gamma_beta_ratio, w.label_smoothing, w.loss_type = beta, gbr, ls, lt_
        losses, cr, rr = w.simpo_loss(c, r)
        d[f"simpo{j}::params"] = np.array(json.dumps([beta, gbr, ls, lt_]))
        d[f"simpo{j}::losses"] = losses.numpy()
        d[f"simpo{j}::chosen_rewards"] = cr.numpy()
        d[f"simpo{j}::rejected_rewards"] = rr.numpy()
    p = os.path.join(HERE, "logps_kat.npz")
    np.savez_compressed(p, **d)
    print("wrote", p, os.path.getsize(p) // 1024, "KiB")


TINY = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, head_dim=128, vocab=512,
                   img_vocab=2048, img_embed=8, gen_head_dim=256, lora_r=16, lora_alpha=32)
ALGO = {"beta": 10.0, "gamma_beta_ratio": 0.5, "sft_weight": 0.0, "label_smoothing": 0.0, "loss_type": "sigmoid"}


def make_tiny():
    g = torch.Generator().manual_seed(7)
    text = [torch.randint(0, TINY.vocab, (1, 5), generator=g, dtype=torch.int32),
            torch.randint(0, TINY.vocab, (1, 8), generator=g, dtype=torch.int32)]
    N = 64
    chosen = torch.randint(0, TINY.img_vocab, (2, N), generator=g)
    rejected = torch.randint(0, TINY.img_vocab, (2, N), generator=g)
    # one bf16-representable weight set, stored once, used by both precisions
    w = O.init_weights(TINY, seed=0, dtype=torch.bfloat16, lora_b_std=2e-2)
    p = os.path.join(HERE, "step_tiny_weights.npz")
    np.savez_compressed(p, **{k: bf16_bits(v) for k, v in w.items()})
    print("wrote", p, os.path.getsize(p) // 1024, "KiB")
    for dt, nm in ((torch.float32, "fp32"), (torch.bfloat16, "bf16")):
        wd = {k: v.to(dt) for k, v in w.items()}
        out = run_reference_step(TINY, wd, dt, text, chosen, rejected, ALGO)
        save_step(os.path.join(HERE, f"step_tiny_{nm}.npz"), TINY, wd, text, chosen, rejected, out, ALGO,
                  store_weights=False, seed=0)


def make_tiny_sft():
    """The make_tiny inputs and weights, fp32, with sft_weight = 0.5."""
    g = torch.Generator().manual_seed(7)
    text = [torch.randint(0, TINY.vocab, (1, 5), generator=g, dtype=torch.int32),
            torch.randint(0, TINY.vocab, (1, 8), generator=g, dtype=torch.int32)]
    N = 64
    chosen = torch.randint(0, TINY.img_vocab, (2, N), generator=g)
    rejected = torch.randint(0, TINY.img_vocab, (2, N), generator=g)
    w = O.init_weights(TINY, seed=0, dtype=torch.bfloat16, lora_b_std=2e-2)
    wd = {k: v.to(torch.float32) for k, v in w.items()}
    algo = dict(ALGO, sft_weight=0.5)
    out = run_reference_step(TINY, wd, torch.float32, text, chosen, rejected, algo)
    save_step(os.path.join(HERE, "step_tiny_sft_fp32.npz"), TINY, wd, text, chosen, rejected, out, algo,
              store_weights=False, seed=0)


ONEB_2L = O.JanusDims(n_layers=2, d_model=2048, d_ff=5632, n_heads=16, head_dim=128, vocab=102400,
                      img_vocab=16384, img_embed=8, gen_head_dim=2048, lora_r=16, lora_alpha=32)


def make_1b():
    data = json.load(open(os.path.join(REF, "examples/step4/train.json")))
    items = [x for x in data if x["item_id"] in ("0000000", "0000001", "0000002", "0000003")]
    text = [synth_prompt_ids(x["prompt"], ONEB_2L.vocab) for x in items]
    N = 64
    g = torch.Generator().manual_seed(11)
    chosen = torch.randint(0, ONEB_2L.img_vocab, (len(items), N), generator=g)
    rejected = torch.randint(0, ONEB_2L.img_vocab, (len(items), N), generator=g)
    w = O.init_weights(ONEB_2L, seed=5, dtype=torch.bfloat16, lora_b_std=1e-2)
    out = run_reference_step(ONEB_2L, w, torch.bfloat16, text, chosen, rejected, ALGO)
    save_step(os.path.join(HERE, "step_1b2l_bf16.npz"), ONEB_2L, w, text, chosen, rejected, out, ALGO,
              store_weights=False, seed=5)


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["kat", "tiny", "sft", "1b"]
    for name, fn in (("kat", make_logps_kat), ("tiny", make_tiny), ("sft", make_tiny_sft), ("1b", make_1b)):
        if name in which:
            fn()
