"""Loaders for the golden fixtures in tests/golden (data only; see make_golden.py)."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from oracle import simpo_ref as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bits_to_bf16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(a.astype(np.uint16).view(np.int16).copy()).view(torch.bfloat16)


def load(name: str):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def exists(name: str) -> bool:
    return os.path.exists(os.path.join(GOLDEN, name))


def dims_of(z) -> O.JanusDims:
    return O.JanusDims(**json.loads(str(z["dims"])))


def step_inputs(z):
    tt, lens = z["text_tokens"], z["text_lens"]
    text = [torch.from_numpy(tt[i, : lens[i]].copy()).view(1, -1) for i in range(len(lens))]
    chosen = torch.from_numpy(z["chosen_ids"].astype(np.int64))
    rejected = torch.from_numpy(z["rejected_ids"].astype(np.int64))
    return text, chosen, rejected


def step_weights(z, name: str, dims: O.JanusDims):
    """Weights for a step fixture: the shared tiny weight file, or regenerated
    from the recorded seed (checked against the recorded sha256)."""
    if name.startswith("step_tiny"):
        wz = load("step_tiny_weights.npz")
        return {k: bits_to_bf16(wz[k]) for k in wz.files}
    w = O.init_weights(dims, seed=int(z["weights_seed"]), dtype=torch.bfloat16, lora_b_std=1e-2)
    return w


def step_outputs(z):
    out = {k[5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("out::") and k != "out::logged"}
    out["logged"] = json.loads(str(z["out::logged"]))
    out["grads"] = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("grad::")}
    return out


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def golden_vq_pixels(z, i):
    """f32 [1, 3, s, s] pixels of vq_golden image i made by ospo_amd.data.VLMImageProcessor from the
    stored uint8 image -- byte-identical to the reference processor's tensor the golden ids were
    encoded from (its sha256 is in the golden)."""
    import hashlib
    from PIL import Image
    from ospo_amd.data import VLMImageProcessor
    u8 = z[f"img{i}_u8"]
    x = VLMImageProcessor(image_size=u8.shape[0])([Image.fromarray(u8)])["pixel_values"]
    assert hashlib.sha256(x.numpy().tobytes()).hexdigest() == str(z[f"img{i}_px_sha256"])
    return x
