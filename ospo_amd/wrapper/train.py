"""JanusProTrainWrapper -- the reference's SimPO plugin (ospo/wrapper/train.py:18-473)
re-homed on the MI355X engine.  Same constructor, same hyper-parameter keys and
defaults (:30-43), same method names and return shapes, same errors:

  training_step(batch, batch_idx) -> loss                         (:87-95)
  preprocess_batch(batch) -> dict                                 (:219-279)
  concatenated_inputs(batch) -> dict                              (:282-314)
  concatenated_forward(batch) -> (c_logps, r_logps, c_logits, r_logits, c_labels)  (:345-372)
  get_batch_logps(logits, labels, average_log_prob) -> [S]        (:375-396)
  simpo_loss(c, r) -> (losses, chosen_rewards, rejected_rewards)  (:317-342)
  get_batch_loss_metrics(batch, train_eval) -> loss               (:399-445)
  compute_loss(inputs) -> loss                                    (:448-456)
  configure_optimizers() -> ([opt], [{"scheduler", "interval"}])  (:108-132)
  compute_total_grad_norm() -> float                              (:459-469)

Differences by construction (documented in DESIGN.md):
  * images arrive as VQ token ids (int [1, N]); VQ encode is the step before the
    hot path.  Float pixel tensors raise NotImplementedError.
  * the embeddings are assembled inside the fused engine, so preprocess_batch
    returns ids/labels instead of [B, T, D] inputs_embeds.
  * logits are materialised for the N image-token positions only (the positions
    whose log-probs the loss uses); ``logits/*`` logging averages over those.
"""
from __future__ import annotations

from typing import Any, Dict, List, Literal, Optional, Tuple

import torch

from .. import dist as odist
from .. import ops
from ..config import save_config
from ..simpo import PolicyLogps, SimPOConfig, SimPOLossBuffers, SimPOLossFn


class FusedLoraAdamW:
    """torch.optim.AdamW over the LoRA adapters as one fused HIP kernel (clip folded in).

    ``param_groups[0]['lr']`` is read at every step, so LR schedulers work as with torch."""

    def __init__(self, engine, lr, betas, eps, weight_decay, max_norm):
        self.engine = engine
        self.param_groups = [{"lr": float(lr), "initial_lr": float(lr), "betas": tuple(betas), "eps": float(eps),
                              "weight_decay": float(weight_decay)}]
        self.max_norm = float(max_norm or 0.0)

    def step(self):
        g = self.param_groups[0]
        self.engine.optimizer_step(g["lr"], g["betas"], g["eps"], g["weight_decay"], self.max_norm)

    def zero_grad(self, set_to_none: bool = True):
        self.engine.zero_grad()

    def state_dict(self):
        e = self.engine
        return {"step": e.opt_step, "exp_avg": e.exp_avg.cpu(), "exp_avg_sq": e.exp_avg_sq.cpu(),
                "param_groups": [dict(g) for g in self.param_groups]}

    def load_state_dict(self, sd):
        e = self.engine
        e.opt_step = int(sd["step"])
        e.exp_avg.copy_(sd["exp_avg"])
        e.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.param_groups = [dict(g) for g in sd["param_groups"]]


class ConstantLR:
    """torch ConstantLR(factor=1.0) as used at train.py:117-118."""

    def __init__(self, optimizer, factor=1.0, total_iters=None):
        self.optimizer, self.last_epoch = optimizer, 0

    def step(self):
        self.last_epoch += 1

    def state_dict(self):
        return {"last_epoch": self.last_epoch}

    def load_state_dict(self, sd):
        self.last_epoch = sd["last_epoch"]


class CosineDecayWarmUpRestarts:
    """ospo/utils/train.py:119-148 (linear warm-up, cosine decay to eta_min)."""

    def __init__(self, optimizer, warmup_iter, max_iter, eta_min=0.0, eta_max=1.5e-4):
        self.optimizer, self.warmup_iter, self.max_iter = optimizer, warmup_iter, max_iter
        self.eta_min, self.eta_max, self.iteration = eta_min, eta_max, 0
        self._apply()

    def get_lr(self):
        import math
        if self.iteration < self.warmup_iter:
            return self.eta_max * self.iteration / self.warmup_iter
        if self.iteration > self.max_iter:
            return self.eta_min
        ratio = (self.iteration - self.warmup_iter) / (self.max_iter - self.warmup_iter)
        assert 0 <= ratio <= 1
        return self.eta_min + (self.eta_max - self.eta_min) * 0.5 * (1.0 + math.cos(math.pi * ratio))

    def _apply(self):
        lr = self.get_lr()
        for g in self.optimizer.param_groups:
            g["lr"] = g["lr_scale"] * lr if "lr_scale" in g else lr

    def step(self):
        self.iteration += 1
        self._apply()

    def state_dict(self):
        return {"iteration": self.iteration}

    def load_state_dict(self, sd):
        self.iteration = sd["iteration"]
        self._apply()


class JanusProTrainWrapper:
    def __init__(self, config, model, chat_processor=None, image_processor=None, tokenizer=None):
        self.config = config
        self.model = model
        self.chat_processor, self.image_processor, self.tokenizer = chat_processor, image_processor, tokenizer
        simpo_config = config["algo"]
        tokenizer_config = config["tokenizer"]
        self.loss_type = simpo_config.get("loss_type", "sigmoid")
        self.beta = simpo_config.get("beta", 1.0)
        self.gamma_beta_ratio = simpo_config.get("gamma_beta_ratio", 0.0)
        self.label_smoothing = simpo_config.get("label_smoothing", 0.0)
        self.sft_weight = simpo_config.get("sft_weight", 0.0)
        self.label_pad_token_id = tokenizer_config.get("label_pad_token_id", -100)
        self.padding_value = getattr(tokenizer, "pad_token_id", None)
        self.max_length = tokenizer_config.get("max_length", 512)
        self.max_prompt_length = tokenizer_config.get("max_prompt_length", 128)
        self.simpo_cfg = SimPOConfig(beta=float(self.beta), gamma_beta_ratio=float(self.gamma_beta_ratio),
                                     label_smoothing=float(self.label_smoothing), loss_type=self.loss_type,
                                     sft_weight=float(self.sft_weight))
        self.engine = model.engine
        self.device = self.engine.device
        self._buf = SimPOLossBuffers(max(1, self.engine.cap_pairs), self.device)
        self.global_step = 0
        self.logged: Dict[str, float] = {}
        self.trainer = None
        self.log_dir = None

    # ------------------------------------------------------------ lifecycle
    def setup(self, stage: str = "fit", log_dir: Optional[str] = None):
        self.log_dir = log_dir
        if log_dir is not None and odist.env_world()[1] == 0:
            save_config(log_dir, self.config)
        self.freeze_param()

    def freeze_param(self):
        """train.py:148-216: with use_peft only the LoRA adapters train.  Any request to
        un-freeze a non-LLM module (gen_head, gen_aligner, ...) is out of the built path."""
        freeze = self.config.get("experiment", {}).get("freeze", {}) or {}
        for mod in ("vision_model", "aligner", "gen_vision_model", "gen_aligner", "gen_head", "gen_embed"):
            if freeze.get(mod, True) is False:
                raise NotImplementedError(f"training {mod} is not on the built path (LoRA-only SimPO)")

    def print_trainable_parameters(self):
        for name, t in self.model.named_lora_parameters().items():
            print(f"{name}: {tuple(t.shape)}, dtype={t.dtype}")

    # ------------------------------------------------------------ logging (PL log / log_dict)
    def log(self, name, value, sync_dist: bool = True, **kw):
        t = value.detach().float().reshape(1).to(self.device) if torch.is_tensor(value) else \
            torch.tensor([float(value)], device=self.device)
        if sync_dist:
            odist.all_reduce_mean_(t)
        self.logged[name] = float(t.item())

    def log_dict(self, d: Dict[str, Any], sync_dist: bool = True, **kw):
        names = list(d)
        vals = torch.stack([(v.detach().float().reshape(()) if torch.is_tensor(v) else torch.tensor(float(v)))
                            .to(self.device) for v in d.values()])
        if sync_dist:
            odist.all_reduce_mean_(vals)  # one fused all-reduce for all scalars
        for n, v in zip(names, vals.tolist()):
            self.logged[n] = v

    # ------------------------------------------------------------ the step
    def training_step(self, batch, batch_idx):
        preprocessed = self.preprocess_batch(batch)
        loss = self.compute_loss(inputs=preprocessed)
        lr = self.trainer.optimizers[0].param_groups[0]["lr"] if self.trainer is not None else float("nan")
        self.log_dict({"train/loss": loss, "train/lr": lr, "train/global_step": self.global_step})
        return loss

    def on_before_optimizer_step(self, *args, **kwargs):
        self.log("train/grad_norm", self.compute_total_grad_norm(), sync_dist=False)

    def configure_optimizers(self):
        c = self.config
        opt = FusedLoraAdamW(self.engine, c["optimizer"]["init_lr"], c["optimizer"]["betas"], c["optimizer"]["eps"],
                             c["optimizer"]["weight_decay"], c["experiment"].get("gradient_clip_val") or 0.0)
        max_steps = c["experiment"].get("max_training_steps")
        if c["optimizer"]["scheduler_type"] == "constant":
            sched = ConstantLR(opt, factor=1.0, total_iters=max_steps)
        elif c["optimizer"]["scheduler_type"] == "cosine":
            warm = max_steps * c["experiment"]["warmup_ratio"]
            sched = CosineDecayWarmUpRestarts(opt, warmup_iter=warm, max_iter=max_steps,
                                              eta_min=c["optimizer"]["min_lr"], eta_max=c["optimizer"]["init_lr"])
        else:
            raise ValueError(f"unknown scheduler_type {c['optimizer']['scheduler_type']}")
        return [opt], [{"scheduler": sched, "interval": "step"}]

    # ------------------------------------------------------------ data -> ids
    def preprocess_batch(self, batch: Tuple) -> Dict[str, Any]:
        item_ids, text_tokens, chosen_t, rejected_t = batch
        B = len(item_ids)
        Lt = max(int(t.shape[-1]) for t in text_tokens)
        text_ids = torch.full((B, Lt), -1, dtype=torch.int32)
        for i, t in enumerate(text_tokens):
            text_ids[i, : t.shape[-1]] = t.reshape(-1).to(torch.int32)
        ch = torch.stack([self._image_ids(x) for x in chosen_t])
        rj = torch.stack([self._image_ids(x) for x in rejected_t])
        d = self.engine.dims
        if int(text_ids.max()) >= d.vocab:
            raise ValueError(f"text token id >= vocab ({d.vocab})")
        if int(torch.cat([ch, rj]).max()) >= d.img_vocab or int(torch.cat([ch, rj]).min()) < 0:
            raise ValueError(f"VQ token id outside [0, {d.img_vocab})")
        lab_txt = torch.full((B, Lt), self.label_pad_token_id, dtype=torch.long)
        return {
            "item_ids": list(item_ids),
            "text_ids": text_ids.to(self.device, non_blocking=True),
            "chosen_ids": ch.to(self.device, torch.int32), "rejected_ids": rj.to(self.device, torch.int32),
            "chosen_labels": torch.cat([lab_txt, ch.long()], 1), "rejected_labels": torch.cat([lab_txt, rj.long()], 1),
        }

    @staticmethod
    def _image_ids(x: torch.Tensor) -> torch.Tensor:
        if x.is_floating_point():
            raise NotImplementedError("pixel tensors need VQ encode, which is not on the built path "
                                      "(SURVEY §8f rank 3): feed VQ token ids (dataset token_cache)")
        return x.reshape(-1).long()

    def concatenated_inputs(self, batch: Dict[str, Any]) -> Dict[str, torch.Tensor]:
        """cat chosen | rejected along dim 0 (train.py:282-314; pad_to_length is a no-op here)."""
        return {
            "concatenated_labels": torch.cat([batch["chosen_labels"], batch["rejected_labels"]], 0),
            "concatenated_image_ids": torch.cat([batch["chosen_ids"], batch["rejected_ids"]], 0),
            "concatenated_text_ids": torch.cat([batch["text_ids"], batch["text_ids"]], 0),
        }

    def concatenated_forward(self, batch):
        len_chosen = batch["chosen_labels"].shape[0]
        all_logps = PolicyLogps.apply(self.model.lora_anchor, self.engine, batch["text_ids"], batch["chosen_ids"],
                                      batch["rejected_ids"])
        e = self.engine
        logits = e.logits[: e.S * e.N].view(e.S, e.N, -1)
        return (all_logps[:len_chosen], all_logps[len_chosen:], logits[:len_chosen], logits[len_chosen:],
                batch["chosen_labels"])

    def get_batch_logps(self, logits: torch.Tensor, labels: torch.LongTensor, average_log_prob: bool = True):
        """Standalone form over materialised logits [S, T, V] (HIP log-softmax + gather)."""
        if logits.shape[:-1] != labels.shape:
            raise ValueError("Logits (batch and sequence length dim) and labels must have the same shape.")
        labels = labels[:, 1:].clone()
        logits = logits[:, :-1, :]
        loss_mask = labels != self.label_pad_token_id
        labels[labels == self.label_pad_token_id] = 0
        S, T, V = logits.shape
        flat = logits.reshape(S * T, V).to(torch.bfloat16).contiguous()
        lab = labels.reshape(-1).to(torch.int32).to(flat.device)
        lse = torch.empty(S * T, device=flat.device)
        tok = torch.empty(S * T, device=flat.device)
        seq = torch.empty(S, device=flat.device)
        ops.logprob_fwd(flat, lab, T, lse, tok, seq)
        per_token = tok.view(S, T) * loss_mask.to(tok.device)
        if average_log_prob:
            return per_token.sum(-1) / loss_mask.to(tok.device).sum(-1)
        return per_token.sum(-1)

    def simpo_loss(self, policy_chosen_logps, policy_rejected_logps):
        B = policy_chosen_logps.shape[0]
        logps = torch.cat([policy_chosen_logps, policy_rejected_logps]).float()
        losses = SimPOLossFn.apply(logps, B, self.simpo_cfg, self._buf)
        chosen_rewards = self.beta * policy_chosen_logps.detach()
        rejected_rewards = self.beta * policy_rejected_logps.detach()
        return losses, chosen_rewards, rejected_rewards

    def get_batch_loss_metrics(self, batch, train_eval: Literal["train", "val"] = "train"):
        prefix = "val" if train_eval == "val" else "train"
        c, r, cl, rl, _ = self.concatenated_forward(batch)
        losses, cr, rr = self.simpo_loss(c, r)
        loss = losses.mean()
        if self.sft_weight > 0.0:
            raise NotImplementedError("sft_weight > 0 is not on the built path")
        self.log_dict({f"{prefix}/rewards/chosen": cr.mean(), f"{prefix}/rewards/rejected": rr.mean(),
                       f"{prefix}/rewards/accuracies": (cr > rr).float().mean(),
                       f"{prefix}/rewards/margins": (cr - rr).mean(),
                       f"{prefix}/logps/rejected": r.detach().mean(), f"{prefix}/logps/chosen": c.detach().mean(),
                       f"{prefix}/logits/rejected": rl.float().mean(), f"{prefix}/logits/chosen": cl.float().mean()})
        return loss

    def compute_loss(self, inputs):
        return self.get_batch_loss_metrics(inputs, train_eval="train")

    def compute_total_grad_norm(self):
        return float(self.engine.grad_norm_sq().sqrt().item())
