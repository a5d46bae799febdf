"""Preference data (mirrors ospo/dataclass/train_dataset.py:16-97 and
ospo/dataclass/datamodule.py:11-45).

``PreferenceDataset[i] -> (item_id, int32 [1, Lt_i] text tokens, chosen, rejected)``
with the reference's prompt: DeepSeek SFT template ``"User: {prompt}\\n\\nAssistant:"``
(janus/utils/conversation.py:80-91, system prompt empty, .strip() at
janus/models/processing_vlm.py:175) + ``<begin_of_image>`` (image_start_tag),
tokenised with BOS.

Images: the built path consumes VQ token ids (int [1, 576]) -- VQ encode is the
step BEFORE the hot path.  Sources, in order:
  * ``token_cache``: an .npz with ``{item_id}/chosen`` and ``{item_id}/rejected``
    int arrays (e.g. produced offline by the reference's VQ encoder);
  * ``synthetic_tokens``: deterministic random ids per (item_id, side) -- what
    this container can do, no VQ weights exist offline.
Text: a HF tokenizer when ``tokenizer_path`` loads; otherwise deterministic
synthetic ids (one per whitespace piece) -- no Janus tokenizer exists offline.
"""
from __future__ import annotations

import hashlib
import json
import random
from typing import Dict, List, Optional

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, DistributedSampler

IMAGE_START_TAG = "<begin_of_image>"
IMAGE_TOKEN_NUM_PER_IMAGE = 576  # ospo/constant.py:4


def sft_prompt(prompt: str) -> str:
    """get_image_generation_prompt (train_dataset.py:59-65)."""
    conv = f"User: {prompt.strip()}\n\nAssistant:"
    return conv.strip() + IMAGE_START_TAG


class SyntheticTokenizer:
    """Stand-in for the absent Janus/LLaMA tokenizer: BOS + one id per piece."""

    def __init__(self, vocab: int = 102400, bos_id: int = 100000, pad_token_id: int = 100002):
        self.vocab, self.bos_id, self.pad_token_id = vocab, bos_id, pad_token_id

    def encode(self, text: str) -> List[int]:
        body = text.replace(IMAGE_START_TAG, " " + IMAGE_START_TAG)
        ids = [self.bos_id]
        for piece in body.split():
            ids.append(int(hashlib.md5(piece.encode()).hexdigest(), 16) % (self.vocab - 8))
        return ids


def load_tokenizer(path: Optional[str], vocab: int = 102400):
    if path:
        try:
            from transformers import AutoTokenizer
            return AutoTokenizer.from_pretrained(path)
        except Exception:  # offline / absent: fall through to the synthetic stand-in
            pass
    return SyntheticTokenizer(vocab=vocab, bos_id=vocab - 2, pad_token_id=vocab - 1)


class PreferenceDataset(Dataset):
    def __init__(self, seed: int, data_path: str, tokenizer, num_samples: Optional[int] = None,
                 sampling_rate: float = 1.0, token_cache: Optional[str] = None, synthetic_tokens: bool = True,
                 img_vocab: int = 16384, n_img_tokens: int = IMAGE_TOKEN_NUM_PER_IMAGE):
        with open(data_path) as f:
            self.dataset = json.load(f)
        if num_samples is not None:
            assert num_samples > 0, "num_samples must be greater than 0"
            assert num_samples <= len(self.dataset), "num_samples cannot exceed dataset size"
            rng = random.Random(seed)
            idx = rng.sample(range(len(self.dataset)), num_samples)
            self.dataset = [self.dataset[i] for i in idx]
        elif sampling_rate != 1.0:
            n = int(len(self.dataset) * sampling_rate)
            assert n > 0, "Dataset size must be bigger than 1."
            self.dataset = self.dataset[:n]
        self.tokenizer = tokenizer
        self.cache = np.load(token_cache, allow_pickle=False) if token_cache else None
        if self.cache is None and not synthetic_tokens:
            raise ValueError("no VQ token source: give dataset.train.token_cache (VQ ids per item) "
                             "or set dataset.train.synthetic_tokens=true")
        self.img_vocab, self.n_img = img_vocab, n_img_tokens

    def __len__(self):
        return len(self.dataset)

    def __getitem__(self, idx):
        return self.decode(self.dataset[idx])

    def collate_fn(self, batch):
        item_ids, text_tokens, chosen, rejected = zip(*batch)
        return list(item_ids), list(text_tokens), list(chosen), list(rejected)

    def get_text_token(self, text: str) -> torch.Tensor:
        ids = self.tokenizer.encode(sft_prompt(text))
        return torch.tensor(ids, dtype=torch.int32).view(1, -1)

    def get_image_tokens(self, item_id: str, side: str) -> torch.Tensor:
        if self.cache is not None:
            return torch.from_numpy(self.cache[f"{item_id}/{side}"].astype(np.int64)).view(1, -1)
        seed = int(hashlib.md5(f"{item_id}/{side}".encode()).hexdigest(), 16) % (2 ** 31)
        g = torch.Generator().manual_seed(seed)
        return torch.randint(0, self.img_vocab, (1, self.n_img), generator=g)

    def decode(self, example: Dict):
        if "prompt" not in example or "chosen" not in example or "rejected" not in example:
            raise ValueError("Could not format example as dialogue for SimPO task!\n"
                             f"This example only has {example.keys()} keys.\n")
        item_id = example["item_id"]
        return (item_id, self.get_text_token(example["prompt"]), self.get_image_tokens(item_id, "chosen"),
                self.get_image_tokens(item_id, "rejected"))


def train_dataloader(config, tokenizer, rank: int = 0, world: int = 1, img_vocab: int = 16384) -> DataLoader:
    """TrainDataModule.train_dataloader (datamodule.py:35-43) + the DistributedSampler PL's DDP adds."""
    tr = config["dataset"]["train"]
    ds = PreferenceDataset(seed=config["experiment"]["seed"], data_path=tr["data_path"], tokenizer=tokenizer,
                           num_samples=tr.get("num_samples"), token_cache=tr.get("token_cache"),
                           synthetic_tokens=tr.get("synthetic_tokens", True), img_vocab=img_vocab)
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True,
                                 seed=config["experiment"]["seed"]) if world > 1 else None
    return DataLoader(ds, batch_size=tr["batch_size"], shuffle=sampler is None, sampler=sampler,
                      collate_fn=ds.collate_fn, num_workers=tr.get("num_workers") or 0, drop_last=False)
