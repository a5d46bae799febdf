"""CPU: the step-3 sampling oracle (oracle/generate_ref.py) and the VQ decoder oracle against the
reference's own generate_image loop (ospo/wrapper/image_generation.py:109-181, run in fp32 on a tiny
Janus-like model by tests/golden/make_golden_generate.py): teacher-forced on the reference's sampled
tokens, the oracle reproduces the probabilities the reference sampled from, and decoding those tokens
reproduces the PNGs the reference saved."""
import os

import numpy as np
import torch

from oracle import generate_ref as G
from oracle import simpo_ref as O
from oracle import vq_ref as V

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "generate_golden.npz")
DIMS = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=16384, gen_head_dim=256,
                   lora_r=16, lora_alpha=32)


def _case():
    z = np.load(GOLD)
    lens = z["prompt_lens"].tolist()
    flat = z["prompts_flat"].tolist()
    prompts, o = [], 0
    for L in lens:
        prompts.append(flat[o:o + L])
        o += L
    w_seed, vq_seed, vq_dec_seed, _ = z["seeds"].tolist()
    pad, cfg, temp = z["pad_cfg_temp"].tolist()
    return z, prompts, int(w_seed), int(vq_seed), int(vq_dec_seed), int(pad), cfg, temp


def test_generate_oracle_matches_reference_loop():
    z, prompts, w_seed, _, _, pad, cfg, temp = _case()
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    w = O.init_weights(DIMS, seed=w_seed, dtype=torch.float32, lora_b_std=1e-2)
    tok = torch.from_numpy(z["tokens"])
    n = tok.shape[1]
    u = torch.rand(n, len(prompts))
    _, p = G.generate_ref(prompts, w, DIMS, n, u, cfg, temp, pad_id=pad, forced=tok, dtype=torch.float32)
    steps = z["prob_steps"].tolist()
    ref = torch.from_numpy(z["probs_f16"].astype(np.float32))
    l1 = (p[steps] - ref).abs().sum(-1)
    assert float(l1.max()) < 2e-3, l1  # fp16 storage of the reference probabilities dominates
    assert float((p.amax(-1) - torch.from_numpy(z["probs_max"])).abs().max()) < 1e-5
    # the reference's draws are in the support of the oracle's distributions
    assert bool((p.gather(2, tok.t().unsqueeze(-1)) > 0).all())


def test_vq_decode_oracle_reproduces_reference_images():
    z, _, _, vq_seed, vq_dec_seed, _, _, _ = _case()
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    w = V.init_vq_weights(vq_seed)
    w.update(V.init_vq_decoder_weights(vq_dec_seed))
    dec = V.decode_code_ref(torch.from_numpy(z["tokens"]), w, 8, 8)
    u8 = V.to_uint8_images(dec)
    diff = np.abs(u8.astype(np.int16) - z["images_u8"].astype(np.int16))
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3
