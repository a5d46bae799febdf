"""A Lightning-shaped fit loop for the SimPO wrapper (what PL 1.9.4's Trainer does
for step 5: ospo/utils/train.py:10-59 + ospo/step5.py:43-50), one process per
GPU, RCCL data parallel.

Per optimizer step: ``accumulate_grad_batches`` x (training_step -> loss.backward)
-> RCCL all-reduce of the flat LoRA grads -> on_before_optimizer_step (grad-norm
log) -> clip + AdamW (fused) -> scheduler.step -> metrics JSONL (TensorBoard is
absent) -> ModelCheckpoint every ``save_steps``.

The all-reduce overlaps the last micro-batch's backward exactly as the timed path
(simpo.train_step) does: GradAllReduce.begin, each layer's range pushed from the
engine's backward hook as soon as its grads are final, finish before the optimizer
(DDP's bucketed all-reduce during backward, ospo/utils/train.py:26-28).
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional

from . import dist as odist
from .ckpt import load_checkpoint, next_version_dir, save_checkpoint, step_ckpt_name
from .config import get


class Trainer:
    def __init__(self, config, world: int = 1, rank: int = 0):
        self.config, self.world, self.rank = config, world, rank
        save_path = get(config, "base.save_path") or "./outputs"
        exp = get(config, "base.exp_name") or "ospo_simpo"
        self.log_dir = next_version_dir(save_path, exp) if rank == 0 else None
        self.max_steps = int(get(config, "experiment.max_training_steps") or 10)
        self.accum = int(get(config, "experiment.gradient_accumulation_steps") or 1)
        self.save_steps = get(config, "experiment.save_steps")
        # PL's log_every_n_steps (the reference passes experiment.log_steps, empty in its step5.yaml -> PL's 50)
        self.log_steps = int(get(config, "experiment.log_steps") or 50)
        self.enable_ckpt = bool(get(config, "experiment.enable_checkpointing", True))
        self.global_step = 0
        self.allreduce = odist.GradAllReduce(world)

    def backward(self, wrapper, loss, last: bool):
        """loss.backward(); on the optimizer step's last micro-batch the grads' all-reduce is begun and fed layer by
        layer from the engine's backward (GradAllReduce.push via engine.layer_grads_hook); the caller finishes it."""
        eng = wrapper.engine
        if last:
            self.allreduce.begin(eng.grads)
            eng.layer_grads_hook = self.allreduce.push
        try:
            (loss / self.accum).backward() if self.accum > 1 else loss.backward()
        finally:
            eng.layer_grads_hook = None

    def fit(self, wrapper, train_dataloaders, ckpt_path: Optional[str] = None):
        wrapper.trainer = self
        wrapper.setup("fit", self.log_dir)
        opts, scheds = wrapper.configure_optimizers()
        self.optimizers = opts
        opt, sched = opts[0], scheds[0]["scheduler"]
        epoch = 0
        if ckpt_path:
            ck = load_checkpoint(ckpt_path, wrapper.engine, opt, sched)
            self.global_step, epoch = int(ck["global_step"]), int(ck["epoch"])
        wrapper.global_step = self.global_step
        opt.zero_grad()
        metrics_f = open(os.path.join(self.log_dir, "metrics.jsonl"), "a") if self.log_dir else None
        micro = 0
        t0 = time.time()
        while self.global_step < self.max_steps:
            sampler = getattr(train_dataloaders, "sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            for idx, batch in enumerate(train_dataloaders):
                loss = wrapper.training_step(batch, idx)
                self.backward(wrapper, loss, last=(micro + 1) % self.accum == 0)
                micro += 1
                if micro % self.accum:
                    continue
                self.allreduce.finish()
                wrapper.on_before_optimizer_step()
                opt.step()
                sched.step()
                opt.zero_grad()
                self.global_step += 1
                wrapper.global_step = self.global_step
                if metrics_f and self.global_step % self.log_steps == 0:
                    rec = {"step": self.global_step, "time": round(time.time() - t0, 3), **wrapper.logged}
                    metrics_f.write(json.dumps(rec) + "\n")
                    metrics_f.flush()
                if (self.enable_ckpt and self.save_steps and self.global_step % int(self.save_steps) == 0
                        and self.rank == 0):
                    save_checkpoint(os.path.join(self.log_dir, step_ckpt_name(self.global_step)), wrapper.engine,
                                    opt, sched, epoch, self.global_step)
                if self.global_step >= self.max_steps:
                    break
            epoch += 1
        if metrics_f:
            metrics_f.close()
        odist.barrier()
        return self
