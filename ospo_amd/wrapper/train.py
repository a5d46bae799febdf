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

Batches come in the reference's collate format (train_dataset.py:53-55): images as f32
pixel tensors [1, 3, 384, 384], VQ-encoded on the GPU inside ``preprocess_batch`` (all 2B
images of the step in one encode, train.py:246-261), or as VQ token ids [1, N] (a token cache).

Differences by construction (documented in DESIGN.md):
  * the VQ encode runs in fp32: the ids of the reference's fp32 vq_model.py; its bf16-precision run
    encodes in bf16 and ~10 % of its ids differ (a documented deviation).
  * the embeddings are assembled inside the fused engine, so preprocess_batch
    returns ids/labels instead of [B, T, D] inputs_embeds.
  * concatenated_forward returns the logits of the N image-token positions (a copy,
    [B, N, V]; the other positions carry label -100); ``logits/*`` logging still averages
    over all [B, T, V] logits as the reference does (engine.logit_sums).
  * logged scalars stay on the device until read (``logged``), so a step has no host sync.
"""
from __future__ import annotations

from typing import Any, Dict, List, Literal, Optional, Tuple

import torch

from .. import dist as odist
from .. import ops
from ..config import save_config
from ..lora import peft_param_order
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
        """torch.optim.AdamW's format: ``state`` {i: {step, exp_avg, exp_avg_sq}} and ``param_groups``
        [{..., params: [0..n-1]}] over the adapter tensors in peft ``parameters()`` order
        (``ospo_param_names`` names them)."""
        e = self.engine
        names = peft_param_order(e.dims.n_layers)
        m, v = e.layout.from_flat(e.exp_avg), e.layout.from_flat(e.exp_avg_sq)
        step = torch.tensor(float(e.opt_step))
        state = {i: {"step": step.clone(), "exp_avg": m[n].detach().cpu().clone(),
                     "exp_avg_sq": v[n].detach().cpu().clone()} for i, n in enumerate(names)} if e.opt_step else {}
        g = dict(self.param_groups[0], amsgrad=False, maximize=False, foreach=None, capturable=False,
                 differentiable=False, fused=None, params=list(range(len(names))))
        g["betas"] = tuple(g["betas"])
        return {"state": state, "param_groups": [g], "ospo_param_names": names}

    def load_state_dict(self, sd):
        """Our state_dict, or a torch AdamW state_dict over the whole reference module tree
        (``AdamW(self.parameters())``): only the adapters train, so its entries WITH state are the
        adapter tensors in peft order, which is how they are mapped."""
        e = self.engine
        names = peft_param_order(e.dims.n_layers)
        if "state" not in sd or "param_groups" not in sd:
            raise ValueError("optimizer state: expected a torch.optim.AdamW state_dict (state, param_groups)")
        keys = sorted(sd["state"])
        if keys and len(keys) != len(names):
            raise ValueError(f"optimizer state holds {len(keys)} tensors with state, the adapters are {len(names)}")
        shapes = {n: s for n, _, s in e.layout.slices()}
        m, v = {}, {}
        steps = set()
        for k, n in zip(keys, names):
            st = sd["state"][k]
            if tuple(st["exp_avg"].shape) != shapes[n]:
                raise ValueError(f"optimizer state {k}: shape {tuple(st['exp_avg'].shape)} != {n} {shapes[n]}")
            m[n], v[n] = st["exp_avg"], st["exp_avg_sq"]
            steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"optimizer state: adapters at different step counts {sorted(steps)}")
        if keys:
            e.layout.to_flat({n: t.to(e.exp_avg.dtype) for n, t in m.items()}, fm := torch.zeros_like(e.exp_avg, device="cpu"))
            e.layout.to_flat({n: t.to(e.exp_avg_sq.dtype) for n, t in v.items()}, fv := torch.zeros_like(e.exp_avg_sq, device="cpu"))
            e.exp_avg.copy_(fm)
            e.exp_avg_sq.copy_(fv)
        else:
            e.exp_avg.zero_()
            e.exp_avg_sq.zero_()
        e.opt_step = steps.pop() if steps else 0
        g = sd["param_groups"][0]
        self.param_groups = [{k: g[k] for k in ("lr", "initial_lr", "betas", "eps", "weight_decay") if k in g}]
        self.param_groups[0].setdefault("initial_lr", self.param_groups[0]["lr"])


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
    """ospo/utils/train.py:119-148 (linear warm-up, cosine decay to eta_min).  As there, construction
    takes the first step: torch's _LRScheduler.__init__ calls the overridden step() once, so the first
    optimizer step already runs at iteration 1 (lr = eta_max / warmup_iter, not 0) -- pinned by
    tests/golden/sched_golden.json (make_golden_sched.py runs the reference's class)."""

    def __init__(self, optimizer, warmup_iter, max_iter, eta_min=0.0, eta_max=1.5e-4):
        self.optimizer, self.warmup_iter, self.max_iter = optimizer, warmup_iter, max_iter
        self.eta_min, self.eta_max, self.iteration = eta_min, eta_max, 0
        for g in optimizer.param_groups:
            g.setdefault("initial_lr", g["lr"])
        self.step()

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
        self._logged: Dict[str, float] = {}
        # name -> (device tensor of one log_dict call, index): only the latest value per name is kept, so a
        # run that never reads .logged holds one small tensor per log_dict call site, not one per step
        self._pending: Dict[str, Tuple[torch.Tensor, int]] = {}
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
    @property
    def logged(self) -> Dict[str, float]:
        """The logged scalars as floats (reading them is the only host sync of the logging)."""
        if self._pending:
            host = {}
            for n, (vals, i) in self._pending.items():
                if id(vals) not in host:
                    host[id(vals)] = vals.tolist()
                self._logged[n] = host[id(vals)][i]
            self._pending = {}
        return self._logged

    def log(self, name, value, sync_dist: bool = True, **kw):
        self.log_dict({name: value}, sync_dist=sync_dist)

    def log_dict(self, d: Dict[str, Any], sync_dist: bool = True, **kw):
        # host numbers (lr, global_step) are the same on every rank: they are logged as they are, without a
        # device round trip (a pageable host->device copy would stall the host until the stream drains)
        dev = {n: v for n, v in d.items() if torch.is_tensor(v)}
        for n, v in d.items():
            if not torch.is_tensor(v):
                self._logged[n] = float(v)
                self._pending.pop(n, None)
        if not dev:
            return
        names = list(dev)
        vals = torch.stack([v.detach().float().reshape(()).to(self.device) for v in dev.values()])
        if sync_dist:
            odist.all_reduce_mean_(vals)  # one fused all-reduce for all scalars
        for i, n in enumerate(names):
            self._pending[n] = (vals, i)

    # ------------------------------------------------------------ the step
    def training_step(self, batch, batch_idx):
        preprocessed = self.preprocess_batch(batch)
        loss = self.compute_loss(inputs=preprocessed)
        lr = self.trainer.optimizers[0].param_groups[0]["lr"] if self.trainer is not None else float("nan")
        self.log_dict({"train/loss": loss, "train/lr": lr, "train/global_step": self.global_step})
        return loss

    def on_before_optimizer_step(self, *args, **kwargs):
        self.log("train/grad_norm", self.engine.grad_norm_sq().sqrt(), sync_dist=False)  # stays on device

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
        """train.py:219-279: text ids right-padded to the batch max (the engine zero-embeds the
        padding), image ids from the VQ encoder (pixels) or as given (token ids), labels
        [-100 x Lt | image ids]."""
        item_ids, text_tokens, chosen_t, rejected_t = batch
        B = len(item_ids)
        Lt = max(int(t.shape[-1]) for t in text_tokens)
        text_ids = torch.full((B, Lt), -1, dtype=torch.int32)
        for i, t in enumerate(text_tokens):
            text_ids[i, : t.shape[-1]] = t.reshape(-1).to(torch.int32)
        d = self.engine.dims
        if int(text_ids.max()) >= d.vocab:
            raise ValueError(f"text token id >= vocab ({d.vocab})")
        images = list(chosen_t) + list(rejected_t)
        pixels = [x.is_floating_point() for x in images]
        if all(pixels):
            # gen_vision_model.encode of all 2B images at once (the reference loops per sample)
            ids = self.model.vq_encode(torch.cat([x.reshape(-1, *x.shape[-3:]) for x in images]))
            if ids.shape != (2 * B, self.engine.N):
                raise ValueError(f"{ids.shape[1]} VQ tokens per image, the engine expects {self.engine.N}")
            text_dev = self._upload(text_ids.reshape(-1)).view(B, Lt)
            ch, rj = ids[:B], ids[B:]
        elif not any(pixels):
            ids = torch.stack([x.reshape(-1).to(torch.int32) for x in images])
            if int(ids.max()) >= d.img_vocab or int(ids.min()) < 0:
                raise ValueError(f"VQ token id outside [0, {d.img_vocab})")
            # text and image ids in ONE asynchronous copy from pinned memory (a pageable copy would hold
            # the host until the previous step's kernels drain)
            flat = self._upload(torch.cat([text_ids.reshape(-1), ids.reshape(-1)]))
            text_dev = flat[: B * Lt].view(B, Lt)
            ids_dev = flat[B * Lt:].view(2 * B, -1)
            ch, rj = ids_dev[:B], ids_dev[B:]
        else:
            raise ValueError("a batch mixes pixel tensors and VQ token ids")
        lab_txt = torch.full((B, Lt), self.label_pad_token_id, dtype=torch.long, device=ch.device)
        return {
            "item_ids": list(item_ids),
            "text_ids": text_dev,
            "chosen_ids": ch, "rejected_ids": rj,
            "chosen_labels": torch.cat([lab_txt, ch.long()], 1), "rejected_labels": torch.cat([lab_txt, rj.long()], 1),
        }

    def _upload(self, host: torch.Tensor) -> torch.Tensor:
        """int32 host ids -> a fresh device tensor by a non-blocking copy from one of two pinned staging
        buffers (each reused only after its previous copy has completed: an event wait, normally already
        satisfied one step later)."""
        if self.device.type != "cuda":
            return host.to(self.device)
        n = host.numel()
        st = getattr(self, "_pin", None)
        if st is None or st[0][0].numel() < n:
            cap = max(n, 1 << 16)
            st = self._pin = [[torch.empty(cap, dtype=torch.int32).pin_memory(), None] for _ in range(2)]
            self._pin_i = 0
        slot = st[self._pin_i]
        self._pin_i ^= 1
        if slot[1] is not None:
            slot[1].synchronize()
        slot[0][:n].copy_(host)
        out = torch.empty(n, dtype=torch.int32, device=self.device)
        out.copy_(slot[0][:n], non_blocking=True)
        slot[1] = torch.cuda.Event()
        slot[1].record()
        return out

    def concatenated_inputs(self, batch: Dict[str, Any]) -> Dict[str, torch.Tensor]:
        """cat chosen | rejected along dim 0 (train.py:282-314; pad_to_length is a no-op here)."""
        return {
            "concatenated_labels": torch.cat([batch["chosen_labels"], batch["rejected_labels"]], 0),
            "concatenated_image_ids": torch.cat([batch["chosen_ids"], batch["rejected_ids"]], 0),
            "concatenated_text_ids": torch.cat([batch["text_ids"], batch["text_ids"]], 0),
        }

    def concatenated_forward(self, batch, return_logits: bool = True):
        """train.py:345-372: (chosen_logps, rejected_logps, chosen_logits, rejected_logits, chosen_labels), the
        logits gen_head's [B, T, V] bf16 over every position as the reference returns them (evaluated on
        request: the loss needs only the N predicting positions, which the engine keeps internally).
        return_logits=False (get_batch_loss_metrics): the two logits entries are None."""
        len_chosen = batch["chosen_labels"].shape[0]
        all_logps = PolicyLogps.apply(self.model.lora_anchor, self.engine, batch["text_ids"], batch["chosen_ids"],
                                      batch["rejected_ids"])
        if not return_logits:
            return all_logps[:len_chosen], all_logps[len_chosen:], None, None, batch["chosen_labels"]
        logits = self.engine.full_logits()  # a new tensor: backward() rewrites only the engine's own buffers
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
        c, r, _, _, _ = self.concatenated_forward(batch, return_logits=False)
        losses, cr, rr = self.simpo_loss(c, r)
        loss = losses.mean()
        e = self.engine
        sft = self.sft_weight > 0.0
        if sft:
            # train.py:421-428: CrossEntropyLoss(ignore -100) over logits[:, :-1] vs labels[:, 1:] of the chosen
            # rows.  Each chosen row has exactly N valid labels, so CE = -mean(chosen per-token-mean logps):
            # the same value and gradient without the [B, T-1, V] tensor
            sft_loss = -c.mean()
            loss = self.sft_weight * sft_loss + loss
            self.log(f"{prefix}/sft_loss", sft_loss.detach(), sync_dist=True)
        # logits/*: mean over all [B, T, V] (over [B, T-1, V] for chosen with sft, train.py:422, 441-442)
        B, T, V = e.B, e.T, e.dims.img_vocab
        sums = e.logit_sums()
        lc = (e.logit_sums(skip_last=True)[:B].sum() / (B * (T - 1) * V)) if sft else sums[:B].sum() / (B * T * V)
        self.log_dict({f"{prefix}/rewards/chosen": cr.mean(), f"{prefix}/rewards/rejected": rr.mean(),
                       f"{prefix}/rewards/accuracies": (cr > rr).float().mean(),
                       f"{prefix}/rewards/margins": (cr - rr).mean(),
                       f"{prefix}/logps/rejected": r.detach().mean(), f"{prefix}/logps/chosen": c.detach().mean(),
                       f"{prefix}/logits/rejected": sums[B:].sum() / (B * T * V), f"{prefix}/logits/chosen": lc})
        return loss

    def compute_loss(self, inputs):
        return self.get_batch_loss_metrics(inputs, train_eval="train")

    def compute_total_grad_norm(self):
        return float(self.engine.grad_norm_sq().sqrt().item())
