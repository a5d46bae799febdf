"""Flat LoRA parameter layout (peft 0.7.1 adapters on q,k,v,o,gate,up,down).

All trainable state lives in ONE contiguous buffer per kind (bf16 params, fp32
grads, bf16 AdamW moments) so the optimizer is one fused kernel and the DP
all-reduce is one bucketed collective over contiguous per-layer slices.

Per layer (D = hidden, F = intermediate, r = rank), in this order:
    A_qkv [3r, D]  = lora_A of q | k | v      (peft lora_A.weight is [r, in])
    A_o   [r,  D]
    A_gu  [2r, D]  = gate | up
    A_d   [r,  F]
    B_qkv [3D, r]  = lora_B of q | k | v      (peft lora_B.weight is [out, r])
    B_o   [D,  r]
    B_gu  [2F, r]  = gate | up
    B_d   [D,  r]
The stacked A block of a group is exactly the packed ``Acat`` operand (rows
j < nmods*r), so dA lands in place; dB is scattered block-diagonally
(``ospo_gemm_f32acc`` diag mode).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

GROUPS = (
    # name, modules, Kin key, Nmod key
    ("qkv", ("q_proj", "k_proj", "v_proj"), "D", "D"),
    ("o", ("o_proj",), "D", "D"),
    ("gu", ("gate_proj", "up_proj"), "D", "F"),
    ("down", ("down_proj",), "F", "D"),
)


def roundup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class Group:
    name: str
    modules: Tuple[str, ...]
    nmods: int
    Kin: int
    Nmod: int
    Rp: int
    a_off: int  # offset (elements) of the A block inside the layer slice
    b_off: int


class LoraLayout:
    def __init__(self, n_layers: int, D: int, F: int, r: int):
        self.L, self.D, self.F, self.r = n_layers, D, F, r
        dims = {"D": D, "F": F}
        off = 0
        groups: List[Group] = []
        for name, mods, kin, nmod in GROUPS:
            groups.append(Group(name, mods, len(mods), dims[kin], dims[nmod], roundup(len(mods) * r, 64), off, 0))
            off += len(mods) * r * dims[kin]
        for g in groups:
            g.b_off = off
            off += g.nmods * g.Nmod * r
        self.groups = {g.name: g for g in groups}
        self.per_layer = off
        self.numel = off * n_layers

    def layer_off(self, i: int) -> int:
        return i * self.per_layer

    def slices(self) -> List[Tuple[str, int, Tuple[int, int]]]:
        """(peft-style name, flat offset, shape) for every adapter tensor."""
        out = []
        r = self.r
        for i in range(self.L):
            base = self.layer_off(i)
            for g in self.groups.values():
                for j, m in enumerate(g.modules):
                    out.append((f"layers.{i}.{m}.lora_A", base + g.a_off + j * r * g.Kin, (r, g.Kin)))
                    out.append((f"layers.{i}.{m}.lora_B", base + g.b_off + j * g.Nmod * r, (g.Nmod, r)))
        return out

    def to_flat(self, tensors: Dict[str, "torch.Tensor"], flat: "torch.Tensor") -> "torch.Tensor":
        for name, off, shape in self.slices():
            t = tensors[name]
            if tuple(t.shape) != shape:
                raise ValueError(f"{name}: expected {shape}, got {tuple(t.shape)}")
            flat[off:off + shape[0] * shape[1]].copy_(t.reshape(-1))
        return flat

    def from_flat(self, flat: "torch.Tensor") -> Dict[str, "torch.Tensor"]:
        return {name: flat[off:off + s[0] * s[1]].view(*s) for name, off, s in self.slices()}


PEFT_MODULE_ORDER = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")


def peft_param_order(n_layers: int) -> List[str]:
    """The adapter tensors in ``model.parameters()`` order of the peft-wrapped Llama (layer by
    layer; self_attn q, k, v, o then mlp gate, up, down; lora_A before lora_B) -- the order of
    the trainable entries of the reference's ``AdamW(self.parameters())`` (train.py:108-115)."""
    return [f"layers.{i}.{m}.lora_{ab}" for i in range(n_layers) for m in PEFT_MODULE_ORDER for ab in "AB"]


def peft_key(name: str) -> str:
    """layers.{i}.{proj}.lora_{A,B} -> the key PL/peft write into the .ckpt state_dict
    (model.language_model.base_model.model.model.layers.{i}.{self_attn|mlp}.{proj}.lora_A.default.weight)."""
    _, i, proj, ab = name.split(".")
    grp = "self_attn" if proj in ("q_proj", "k_proj", "v_proj", "o_proj") else "mlp"
    return f"model.language_model.base_model.model.model.layers.{i}.{grp}.{proj}.{ab}.default.weight"
