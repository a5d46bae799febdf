"""SimPO loss + one training step on the HIP path.

``simpo_loss`` mirrors ``ospo/wrapper/train.py:317-342`` (sigmoid / hinge,
label smoothing, gamma_beta_ratio) and ``losses.mean()`` (:419); the autograd
Functions let the reference-shaped wrapper call ``loss.backward()`` exactly as
PL does, while the hot loop (bench.py) calls ``train_step`` directly.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import ops


@dataclass
class SimPOConfig:
    """configs/step5.yaml ``algo`` block (+ optimizer / clip of the Trainer)."""
    beta: float = 10.0
    gamma_beta_ratio: float = 0.5
    label_smoothing: float = 0.0
    loss_type: str = "sigmoid"
    sft_weight: float = 0.0
    lr: float = 4e-5
    betas: tuple = (0.9, 0.95)
    eps: float = 1e-8
    weight_decay: float = 0.0
    max_norm: float = 1.0

    def __post_init__(self):
        ops.loss_type_id(self.loss_type)  # ValueError on unknown type, like train.py:335-337
        if self.sft_weight < 0:
            raise ValueError("sft_weight must be >= 0")


class SimPOLossBuffers:
    def __init__(self, max_pairs: int, device):
        f = lambda n: torch.zeros(n, dtype=torch.float32, device=device)  # noqa: E731
        self.losses, self.mean, self.rewards = f(max_pairs), f(1), f(2 * max_pairs)
        self.glogps, self.one = f(2 * max_pairs), torch.ones(1, dtype=torch.float32, device=device)


def simpo_forward(logps: torch.Tensor, B: int, cfg: SimPOConfig, buf: SimPOLossBuffers):
    ops.simpo_fwd(logps, B, cfg.beta, cfg.gamma_beta_ratio, cfg.label_smoothing, cfg.loss_type,
                  buf.losses, buf.mean, buf.rewards)
    return buf.losses[:B], buf.mean, buf.rewards[: 2 * B]


def simpo_backward(logps: torch.Tensor, B: int, cfg: SimPOConfig, buf: SimPOLossBuffers,
                   g_loss: Optional[torch.Tensor] = None) -> torch.Tensor:
    ops.simpo_bwd(logps, B, cfg.beta, cfg.gamma_beta_ratio, cfg.label_smoothing, cfg.loss_type,
                  buf.one if g_loss is None else g_loss, buf.glogps)
    return buf.glogps[: 2 * B]


def train_step(engine, text_ids, chosen_ids, rejected_ids, cfg: SimPOConfig, buf: SimPOLossBuffers,
               allreduce=None, optimizer: bool = True) -> Dict[str, torch.Tensor]:
    """fwd (2B sequences) -> SimPO loss -> bwd to LoRA -> [DP all-reduce] -> clip + AdamW.
    Everything stays on device; returns device tensors (no host sync)."""
    B = chosen_ids.shape[0]
    logps = engine.forward(text_ids, chosen_ids, rejected_ids)
    losses, mean, rewards = simpo_forward(logps, B, cfg, buf)
    glogps = simpo_backward(logps, B, cfg, buf)
    sft = None
    if cfg.sft_weight > 0.0:
        # train.py:421-428: CE over the chosen logits' valid (image-token) positions; every chosen row
        # has exactly N of them, so CE = -mean(chosen per-token-mean logps) and d/d logps = -1/B
        sft = -logps[:B].mean()
        mean = mean + cfg.sft_weight * sft
        glogps[:B] -= cfg.sft_weight / B
    engine.zero_grad()
    if allreduce is not None and hasattr(allreduce, "begin"):
        allreduce.begin(engine.grads)  # layer buckets all-reduced while the backward runs on
        engine.backward(glogps, on_layer_grads=allreduce.push)
        allreduce.finish()
    else:
        engine.backward(glogps)
        if allreduce is not None:
            allreduce(engine.grads)
    if optimizer:
        engine.optimizer_step(cfg.lr, cfg.betas, cfg.eps, cfg.weight_decay, cfg.max_norm)
    out = {"loss": mean, "losses": losses, "logps": logps, "rewards": rewards}
    if sft is not None:
        out["sft_loss"] = sft
    return out


# --------------------------------------------------------------------------- autograd
class PolicyLogps(torch.autograd.Function):
    """logps = policy(batch); backward drives the explicit HIP backward and leaves
    the LoRA gradient in ``engine.grads`` (flat fp32).  ``anchor`` is the flat
    LoRA tensor so autograd has a leaf to reach; its returned grad is None
    (the optimizer reads engine.grads, as PL's AdamW reads p.grad)."""

    @staticmethod
    def forward(ctx, anchor, engine, text_ids, chosen_ids, rejected_ids):
        ctx.engine = engine
        return engine.forward(text_ids, chosen_ids, rejected_ids).clone()

    @staticmethod
    def backward(ctx, g):
        # engine.layer_grads_hook (Trainer.fit sets it to GradAllReduce.push on the step's last micro-batch): the
        # DP all-reduce of each layer's grads starts while the backward runs on, as in train_step
        ctx.engine.backward(g.contiguous().float(), on_layer_grads=getattr(ctx.engine, "layer_grads_hook", None))
        return None, None, None, None, None


class SimPOLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logps, B, cfg, buf):
        ctx.save_for_backward(logps)
        ctx.B, ctx.cfg, ctx.buf = B, cfg, buf
        losses, _, _ = simpo_forward(logps.contiguous(), B, cfg, buf)
        return losses.clone()

    @staticmethod
    def backward(ctx, g_losses):
        (logps,) = ctx.saved_tensors
        # d/dlogps of sum_i g_i * loss_i: loss_i depends on (c_i, r_i) only and the kernel gives
        # d(mean)/dlogps = (1/B) dloss_i/d(c_i, r_i) for a unit upstream grad, so scale by B * g_i
        # (no host sync; losses.mean() gives g_i = 1/B)
        g = g_losses.contiguous().float()
        glogps = simpo_backward(logps.contiguous(), ctx.B, ctx.cfg, ctx.buf)
        return glogps * (ctx.B * torch.cat([g, g])), None, None, None
