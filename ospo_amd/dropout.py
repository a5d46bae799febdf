"""LoRA dropout masks of the HIP path (peft lora.Linear: y = W x + s B A dropout(x),
ospo/utils/model.py:50-57 with configs/peft/lora.yaml lora_dropout).

The mask is counter based, so the forward (skinny u kernel) and the backward (dX
GEMM epilogue, dA on the stored masked input) regenerate the same bits without
storing them: element idx = m * K + k of a [M, K] adapter input is kept iff the
16-bit half (idx & 1) of drop_hash(idx >> 1, seed) is >= p * 2^16 (one hash per two
adjacent elements; K is even), kept values become bf16(x / (1 - p)).
``drop_hash`` / ``keep_bits`` restate ``ospo_amd/csrc/common.h`` (drop_hash, drop_keep)
bit for bit (numpy uint32).

One mask per adapter INPUT per layer and step: q/k/v share the mask of the
attention-norm output and gate/up that of the MLP-norm output (their LoRA A's are
fused into one product).  peft draws an independent mask per module; the
per-module marginal distribution and the expectation are the same.
"""
from __future__ import annotations

import numpy as np

GROUP_IDS = {"qkv": 0, "o": 1, "gu": 2, "down": 3}
_M32 = np.uint32(0xFFFFFFFF)


def _mad24(x, c):
    """common.h drop_mad24: x + lo24(x) * c (c even), a bijection of uint32 (one v_mad_u32_u24)."""
    return (x & np.uint32(0xFFFFFF)) * np.uint32(c) + x


def drop_hash(idx, seed):
    """uint32 hash of element (pair) index idx (array) under seed (int), as on the device: four
    multiply-xorshift rounds on 24-bit multiplies, each a 32-bit bijection, the seed keyed in after the
    first (common.h drop_hash, round 5)."""
    with np.errstate(over="ignore"):
        x = _mad24(np.asarray(idx, dtype=np.uint32), 0xED5AD4)
        x ^= x >> np.uint32(16)
        x ^= np.uint32(seed & 0xFFFFFFFF)
        x = _mad24(x, 0xAC4C1A)
        x ^= x >> np.uint32(15)
        x = _mad24(x, 0x9E3778)
        x ^= x >> np.uint32(13)
        x = _mad24(x, 0xC2B2AE)
        x ^= x >> np.uint32(16)
    return x


def _seed_mix(idx, seed):
    """The host-side seed mixer of layer_seed (32-bit multiply-xorshift; never evaluated on the device)."""
    with np.errstate(over="ignore"):
        x = np.asarray(idx, dtype=np.uint32) * np.uint32(0x9E3779B1) + np.uint32(seed & 0xFFFFFFFF)
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x


def threshold(p: float) -> int:
    """16-bit keep threshold (common.h drop_threshold)."""
    return int(float(p) * 65536.0)


def keep_bits(idx, seed, p: float):
    """bool keep decision of flat element indices idx (array) -- common.h drop_keep."""
    idx = np.asarray(idx, dtype=np.uint32)
    h = drop_hash(idx >> np.uint32(1), seed)
    half = np.where((idx & np.uint32(1)) != 0, h >> np.uint32(16), h & np.uint32(0xFFFF))
    return half >= np.uint32(threshold(p))


def layer_seed(base: int, call: int, layer: int, group: str) -> int:
    """Seed of one adapter input's mask: distinct per (base seed, forward call, layer, group)."""
    h = _seed_mix(np.uint32((call * 131 + layer * 8 + GROUP_IDS[group]) & 0xFFFFFFFF), base & 0xFFFFFFFF)
    return int(_seed_mix(h, 0x5BD1E995))


def keep_mask(M: int, K: int, seed: int, p: float) -> np.ndarray:
    """bool [M, K] keep mask of an adapter input (test / oracle use)."""
    idx = np.arange(M * K, dtype=np.uint64).astype(np.uint32).reshape(M, K)
    return keep_bits(idx, seed, p)
