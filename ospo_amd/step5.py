"""Step-5 entry point (mirrors ospo/step5.py:17-59).

    python -m ospo_amd.step5 --cfg_path configs/step5.yaml key=val ...
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m ospo_amd.step5 --cfg_path ...

Same YAML schema as configs/step5.yaml (use_peft / use_lora both accepted),
same seed, resume via ``base.resume``; one process per GPU over RCCL.
"""
from __future__ import annotations

import argparse
import os
import random

import numpy as np
import torch

from . import dist as odist
from .config import build_config, get
from .data import train_dataloader
from .model import get_model
from .trainer import Trainer
from .wrapper.train import JanusProTrainWrapper


def seed_everything(seed: int):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def main(config):
    world, rank, local = odist.init()
    if get(config, "base.save_path") is not None:
        os.makedirs(config["base"]["save_path"], exist_ok=True)
    seed_everything(int(get(config, "experiment.seed", 42)))
    prec = get(config, "experiment.precision", "bf16")
    # fp8 / mx8: bf16 activations, MXFP8 frozen Linears (get_model reads the same key)
    dtype = torch.bfloat16 if prec in ("bf16", None, "auto", "fp8", "mx8") else torch.float32
    model, chat_processor, image_processor, tokenizer = get_model(mode="train", dtype=dtype, config=config,
                                                                  seed=int(get(config, "experiment.seed", 42)))
    dl = train_dataloader(config, tokenizer, rank=rank, world=world, img_vocab=model.engine.dims.img_vocab)
    wrapper = JanusProTrainWrapper(config, model=model, chat_processor=chat_processor,
                                   image_processor=image_processor, tokenizer=tokenizer)
    trainer = Trainer(config, world=world, rank=rank)
    resume = get(config, "base.resume")
    if resume is not None and os.path.exists(resume):
        print("Training resume.")
        trainer.fit(wrapper, dl, ckpt_path=resume)
    else:
        trainer.fit(wrapper, train_dataloaders=dl)
    return trainer, wrapper


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("--cfg_path", type=str, default="configs/step5.yaml")
    args, unknown = parser.parse_known_args()
    main(build_config(cfg_path=args.cfg_path, argv=unknown))
