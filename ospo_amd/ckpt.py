"""Lightning-layout checkpoints (ospo/utils/train.py:11-17).

``{save_path}/{exp_name}/version_N/step=NNNNNN.ckpt`` next to ``config.yaml``
(JSON text, ospo/utils/common.py:102-108).  The .ckpt is a torch file with the
PL 1.9 keys (state_dict, optimizer_states, lr_schedulers, epoch, global_step,
pytorch-lightning_version, loops, callbacks).  ``state_dict`` carries the LoRA
adapters under their peft names (``model.language_model.base_model.model.model
.layers.{i}.{self_attn|mlp}.{proj}.lora_{A|B}.default.weight``) -- the keys
ospo/inference.py:274-278 loads with strict=False; the frozen 7B base is not
re-written (it is the unchanged pretrained checkpoint).
"""
from __future__ import annotations

import os
import re
from typing import Optional

import torch

from .lora import peft_key


def next_version_dir(save_path: str, exp_name: str) -> str:
    root = os.path.join(save_path, exp_name)
    os.makedirs(root, exist_ok=True)
    vs = [int(m.group(1)) for d in os.listdir(root) if (m := re.fullmatch(r"version_(\d+)", d))]
    return os.path.join(root, f"version_{max(vs) + 1 if vs else 0}")


def save_checkpoint(path: str, engine, optimizer, scheduler, epoch: int, global_step: int):
    sd = {peft_key(n): t.detach().cpu().clone() for n, t in engine.lora_tensors().items()}
    ckpt = {
        "epoch": epoch, "global_step": global_step, "pytorch-lightning_version": "1.9.4",
        "state_dict": sd,
        "optimizer_states": [optimizer.state_dict()],
        "lr_schedulers": [scheduler.state_dict()],
        "loops": {}, "callbacks": {},
    }
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save(ckpt, path)
    return path


def load_checkpoint(path: str, engine, optimizer=None, scheduler=None) -> dict:
    """Restore adapters (+ optimizer / scheduler) -- PL resume (step5.py:46-48)."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    sd = ckpt["state_dict"]
    tensors = {}
    for n, t in engine.lora_tensors().items():
        k = peft_key(n)
        if k not in sd:
            raise KeyError(f"checkpoint {path} lacks {k}")
        tensors[n] = sd[k].to(t.dtype)
    flat = torch.zeros(engine.layout.numel, dtype=engine.lora.dtype)
    engine.layout.to_flat(tensors, flat)
    engine.lora.copy_(flat)
    engine.pack_lora()
    if optimizer is not None and ckpt.get("optimizer_states"):
        optimizer.load_state_dict(ckpt["optimizer_states"][0])
    if scheduler is not None and ckpt.get("lr_schedulers"):
        scheduler.load_state_dict(ckpt["lr_schedulers"][0])
    return ckpt


def step_ckpt_name(global_step: int) -> str:
    return f"step={global_step:06d}.ckpt"
