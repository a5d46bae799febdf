"""Golden vectors of step-3 image generation from the REFERENCE's own loop (this container only).

Run:  python tests/golden/make_golden_generate.py          (needs /root/reference)

Runs ``JanusProImageGenWrapper.generate_image`` of the reference's ``ospo/wrapper/image_generation.py``
(:109-191: prompt rows with left padding and the unconditional copies, the KV-cache loop, CFG,
``softmax(logits / temperature)``, ``torch.multinomial``, ``prepare_gen_img_embeds``, then
``gen_vision_model.decode_code`` and the uint8 PNGs it saves) on a tiny Janus-like model in fp32 on
the CPU: the container's ``transformers.LlamaForCausalLM`` (eager attention), the reference's
``MlpProjector`` (janus/models/projector.py), ``vision_head`` (exec'd from modeling_vlm.py, as
make_golden.py) and the reference's own ``VQModel`` (janus/models/vq_model.py) with the seeded
weights of ``oracle.vq_ref``.  Absent packages (pytorch_lightning, pyrootutils) are stubbed;
``Tensor.cuda`` is the identity during the run (the loop moves its token buffer to CUDA); the
tokenizer maps a prompt string of integers to those ids (no Janus tokenizer offline).  Each
step's gen_head output is recorded (the loop does not expose it), so the golden holds the
per-step guided probabilities the reference sampled from.

Output ``tests/golden/generate_golden.npz`` (data only): prompts (ids), the weight seeds, the
sampled tokens, the probabilities [B, V] of 8 of the steps (fp16) and every step's max probability,
the saved uint8 images.
"""
from __future__ import annotations

import ast
import importlib.util
import os
import sys
import tempfile
import types

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import simpo_ref as O  # noqa: E402
from oracle import vq_ref as V  # noqa: E402

DIMS = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=16384, gen_head_dim=256,
                   lora_r=16, lora_alpha=32)
W_SEED, VQ_SEED, VQ_DEC_SEED, GEN_SEED = 29, 3, 4, 1234
N_IMG, IMG = 64, 128  # 8 x 8 tokens -> 128 px
PROMPTS = [[101, 7, 33, 250, 12, 9], [88, 300, 4], [17, 17, 42, 99, 501, 2, 60, 3]]
PAD_ID, CFG, TEMP = 5, 5.0, 1.0
STEPS = [0, 1, 2, 3, 15, 31, 47, 63]  # steps whose full probability vectors are kept


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def install_stubs():
    pl = types.ModuleType("pytorch_lightning")

    class LightningModule(nn.Module):
        @property
        def device(self):
            return torch.device("cpu")

    pl.LightningModule = LightningModule
    pl.seed_everything = lambda *a, **k: None
    sys.modules["pytorch_lightning"] = pl
    pr = types.ModuleType("pyrootutils")
    pr.setup_root = lambda *a, **k: None
    sys.modules["pyrootutils"] = pr
    pv = types.ModuleType("janus.models.processing_vlm")
    pv.VLChatProcessorOutput = pv.BatchedVLChatProcessorOutput = object
    for name in ("janus", "janus.models", "ospo", "ospo.utils"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["janus.models.processing_vlm"] = pv
    common = types.ModuleType("ospo.utils.common")  # set_seed as common.py:60-65 (PL part stubbed)

    def set_seed(seed):
        import random
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
    common.set_seed = set_seed
    common.save_json = lambda *a, **k: None
    sys.modules["ospo.utils.common"] = common
    ad = types.ModuleType("attrdict")
    ad.AttrDict = AttrDict
    sys.modules["attrdict"] = ad


def load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def vision_head_cls():
    src = open(os.path.join(REF, "janus/models/modeling_vlm.py")).read()
    cls = [n for n in ast.parse(src).body if isinstance(n, ast.ClassDef) and n.name == "vision_head"][0]
    ns = {"torch": torch}
    exec(compile(ast.Module(body=[cls], type_ignores=[]), "modeling_vlm.py", "exec"), ns)
    return ns["vision_head"]


class Tok:
    vocab = {"<begin_of_image>": 1, "<end_of_image>": 2, "<image_placeholder>": 3, "<｜▁pad▁｜>": PAD_ID}

    def encode(self, text):
        return [int(t) for t in text.split()]


def main():
    install_stubs()
    sys.path.insert(0, REF)
    load("ospo.constant", "ospo/constant.py")
    load("ospo.utils.processor", "ospo/utils/processor.py")
    gen_mod = load("ospo_ref_image_generation", "ospo/wrapper/image_generation.py")
    proj = load("janus_ref_projector", "janus/models/projector.py")
    vqm = load("janus_ref_vq_model", "janus/models/vq_model.py")
    from transformers import LlamaConfig, LlamaForCausalLM

    w = O.init_weights(DIMS, seed=W_SEED, dtype=torch.float32, lora_b_std=1e-2)
    from oracle.generate_ref import merge_lora
    wm = merge_lora(w, DIMS)  # inference.py merges the adapter before sampling
    cfg = LlamaConfig(vocab_size=DIMS.vocab, hidden_size=DIMS.d_model, intermediate_size=DIMS.d_ff,
                      num_hidden_layers=DIMS.n_layers, num_attention_heads=DIMS.n_heads,
                      num_key_value_heads=DIMS.n_heads, rms_norm_eps=DIMS.rms_eps, max_position_embeddings=4096,
                      rope_theta=DIMS.rope_theta, attn_implementation="eager", tie_word_embeddings=False)
    llama = LlamaForCausalLM(cfg)
    sd = llama.state_dict()
    with torch.no_grad():
        sd["model.embed_tokens.weight"].copy_(wm["embed_tokens"])
        sd["model.norm.weight"].copy_(wm["norm"])
        for i in range(DIMS.n_layers):
            for nm in ("input_layernorm", "post_attention_layernorm"):
                sd[f"model.layers.{i}.{nm}.weight"].copy_(wm[f"layers.{i}.{nm}"])
            for p in O.PROJS:
                grp = "self_attn" if p in O.PROJS_ATTN else "mlp"
                sd[f"model.layers.{i}.{grp}.{p}.weight"].copy_(wm[f"layers.{i}.{p}"])
    llama.load_state_dict(sd)
    model = nn.Module()
    model.language_model = llama
    model.gen_head = vision_head_cls()(AttrDict(n_embed=DIMS.d_model, image_token_embed=DIMS.gen_head_dim,
                                                image_token_size=DIMS.img_vocab))
    model.gen_aligner = proj.MlpProjector(AttrDict(projector_type="mlp_gelu", input_dim=DIMS.img_embed,
                                                   n_embed=DIMS.d_model, depth=2))
    model.gen_embed = nn.Embedding(DIMS.img_vocab, DIMS.img_embed)
    with torch.no_grad():
        model.gen_head.output_mlp_projector.weight.copy_(wm["gen_head.w1"])
        model.gen_head.output_mlp_projector.bias.copy_(wm["gen_head.b1"])
        model.gen_head.vision_head.weight.copy_(wm["gen_head.w2"])
        model.gen_head.vision_head.bias.copy_(wm["gen_head.b2"])
        model.gen_aligner.layers[0].weight.copy_(wm["gen_aligner.w1"])
        model.gen_aligner.layers[0].bias.copy_(wm["gen_aligner.b1"])
        model.gen_aligner.layers[2].weight.copy_(wm["gen_aligner.w2"])
        model.gen_aligner.layers[2].bias.copy_(wm["gen_aligner.b2"])
        model.gen_embed.weight.copy_(wm["gen_embed"])
    model.prepare_gen_img_embeds = lambda ids: model.gen_aligner(model.gen_embed(ids))  # modeling_vlm.py:263-264
    vq = vqm.VQModel(vqm.ModelArgs()).eval()
    vw = V.init_vq_weights(VQ_SEED)
    vw.update(V.init_vq_decoder_weights(VQ_DEC_SEED))
    missing, unexpected = vq.load_state_dict(vw, strict=False)
    assert not unexpected and all(k.startswith("quantize.codebook_used") for k in missing), (missing, unexpected)
    model.gen_vision_model = vq
    model.eval()
    recorded = []

    class Recorder(nn.Module):
        def __init__(self, inner):
            super().__init__()
            self.inner = inner

        def forward(self, h):
            out = self.inner(h)
            recorded.append(out.detach().clone())
            return out
    model.gen_head = Recorder(model.gen_head)

    proc = types.SimpleNamespace(tokenizer=Tok(), pad_id=PAD_ID, image_start_tag="<begin_of_image>")
    wrapper = gen_mod.JanusProImageGenWrapper(AttrDict(generation_config=AttrDict(cfg_weight=CFG, temperature=TEMP)),
                                              model, Tok(), proc)
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    tmp = tempfile.mkdtemp()
    paths = [os.path.join(tmp, f"{i:02d}.png") for i in range(len(PROMPTS))]
    try:
        with torch.no_grad():
            wrapper.generate_image([" ".join(map(str, p)) for p in PROMPTS], paths, seed=GEN_SEED,
                                   image_token_num_per_image=N_IMG, img_size=IMG, patch_size=16)
    finally:
        torch.Tensor.cuda = cuda
    B = len(PROMPTS)
    assert len(recorded) == N_IMG
    probs = []
    for lg in recorded:  # image_generation.py:156-160, recomputed from the recorded head output
        l2 = lg[1::2] + CFG * (lg[0::2] - lg[1::2])
        probs.append(torch.softmax(l2 / TEMP, dim=-1))
    probs = torch.stack(probs)  # [n, B, V]
    # the sampled tokens: the loop's only random op is torch.multinomial, so replaying its calls on the
    # recorded probabilities after set_seed(seed) gives its draws (checked below against the saved PNGs)
    torch.manual_seed(GEN_SEED)
    import random
    random.seed(GEN_SEED)
    np.random.seed(GEN_SEED)
    toks = torch.stack([torch.multinomial(p, num_samples=1).squeeze(-1) for p in probs], 1)  # same RNG stream
    from PIL import Image
    imgs = np.stack([np.asarray(Image.open(p)) for p in paths])
    out = {"prompts_flat": np.array(sum(PROMPTS, []), dtype=np.int64),
           "prompt_lens": np.array([len(p) for p in PROMPTS], dtype=np.int64),
           "seeds": np.array([W_SEED, VQ_SEED, VQ_DEC_SEED, GEN_SEED], dtype=np.int64),
           "pad_cfg_temp": np.array([PAD_ID, CFG, TEMP], dtype=np.float64),
           "tokens": toks.numpy().astype(np.int64), "prob_steps": np.array(STEPS, dtype=np.int64),
           "probs_f16": probs[STEPS].numpy().astype(np.float16),
           "probs_max": probs.amax(-1).numpy().astype(np.float32), "images_u8": imgs}
    # the replayed draws must be the loop's: they decode to the saved images
    dec = vq.decode_code(toks.int(), shape=[B, 8, IMG // 16, IMG // 16]).detach().numpy().transpose(0, 2, 3, 1)
    dec = np.clip((dec + 1) / 2 * 255, 0, 255)
    u8 = np.zeros(dec.shape, dtype=np.uint8)
    u8[:] = dec
    assert np.array_equal(u8, imgs), "replayed multinomial draws differ from the loop's"
    np.savez_compressed(os.path.join(HERE, "generate_golden.npz"), **out)
    print("wrote generate_golden.npz", toks.shape, imgs.shape)


if __name__ == "__main__":
    main()
