"""Preference data (mirrors ospo/dataclass/train_dataset.py:16-97 and
ospo/dataclass/datamodule.py:11-45).

``PreferenceDataset[i] -> (item_id, int32 [1, Lt_i] text tokens, chosen, rejected)``
with the reference's prompt: DeepSeek SFT template ``"User: {prompt}\\n\\nAssistant:"``
(janus/utils/conversation.py:80-91, system prompt empty, .strip() at
janus/models/processing_vlm.py:175) + ``<begin_of_image>`` (image_start_tag),
tokenised with BOS.

Images, in the reference's collate format by default:
  * pixels (default, as the reference): ``VLMImageProcessor`` -> f32 [1, 3, 384, 384] in
    [-1, 1]; the wrapper VQ-encodes them on the GPU inside ``preprocess_batch``
    (train.py:246-261);
  * ``token_cache``: an .npz with ``{item_id}/chosen`` and ``{item_id}/rejected`` int
    arrays (``python -m ospo_amd.vq`` writes it) -- the encode is then skipped;
  * ``synthetic_tokens: true`` (explicit opt-in): deterministic random ids per
    (item_id, side), for throughput runs without images.
Text: a HF tokenizer from ``tokenizer_path`` (default: ``model_path``, where the reference
loads its processor); the md5 stand-in only when no path is given at all.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, DistributedSampler

IMAGE_START_TAG = "<begin_of_image>"
IMAGE_TOKEN_NUM_PER_IMAGE = 576  # ospo/constant.py:4
IMG_SIZE = 384                   # ospo/constant.py:2


def sft_prompt(prompt: str) -> str:
    """get_image_generation_prompt (train_dataset.py:59-65)."""
    conv = f"User: {prompt.strip()}\n\nAssistant:"
    return conv.strip() + IMAGE_START_TAG


class ChatProcessor:
    """The parts of janus VLChatProcessor the step-5 dataset uses (processing_vlm.py:84-177):
    ``image_start_tag``, ``sft_format`` and ``apply_sft_template_for_multi_turn_prompts`` with the
    DeepSeek separator style (conversation.py:76-91: sep "\\n\\n", sep2 end-of-sentence)."""

    SEP, SEP2 = "\n\n", "<｜end▁of▁sentence｜>"

    def __init__(self, tokenizer=None, image_start_tag: str = IMAGE_START_TAG, sft_format: str = "deepseek",
                 system_prompt: str = ""):
        self.tokenizer, self.image_start_tag, self.sft_format = tokenizer, image_start_tag, sft_format
        self.system_prompt = system_prompt
        self.image_processor = VLMImageProcessor()

    def apply_sft_template_for_multi_turn_prompts(self, conversations: List[Dict[str, str]],
                                                  sft_format: str = "deepseek", system_prompt: str = "") -> str:
        if sft_format != "deepseek":
            raise NotImplementedError(f"sft_format {sft_format!r}: only the deepseek template is on the path")
        ret = system_prompt + self.SEP if system_prompt else ""
        for i, m in enumerate(conversations):
            msg = m["content"].strip()
            ret += (m["role"] + ": " + msg + (self.SEP, self.SEP2)[i % 2]) if msg else (m["role"] + ":")
        return ret.strip()


def expand2square(img, background_color):
    """image_processing_vlm.py:41-52 (pad the short side, image centred)."""
    from PIL import Image
    w, h = img.size
    if w == h:
        return img
    s = max(w, h)
    out = Image.new(img.mode, (s, s), background_color)
    out.paste(img, (0, (s - h) // 2) if w > h else ((s - w) // 2, 0))
    return out


class VLMImageProcessor:
    """janus VLMImageProcessor (image_processing_vlm.py:92-192) with the Janus-Pro gen settings
    (image_size 384, mean = std = 0.5): bicubic resize of the long side to image_size (PIL, which
    antialiases, as torchvision's PIL path), pad to square with the mean colour, x/255 (f64, then
    f32 as HF ``rescale``), (x - mean) / std in f32 (HF ``normalize``).
    ``processor([pil, ...])["pixel_values"]`` -> f32 [n, 3, image_size, image_size]."""

    def __init__(self, image_size: int = IMG_SIZE, min_size: int = 14, image_mean=(0.5, 0.5, 0.5),
                 image_std=(0.5, 0.5, 0.5), rescale_factor: float = 1.0 / 255.0, do_normalize: bool = True):
        self.image_size, self.min_size = image_size, min_size
        self.image_mean, self.image_std = tuple(image_mean), tuple(image_std)
        self.rescale_factor, self.do_normalize = rescale_factor, do_normalize
        self.background_color = (127, 127, 127) if image_mean is None else tuple(int(x * 255) for x in image_mean)

    def resize(self, pil_img) -> np.ndarray:
        from PIL import Image
        w, h = pil_img.size
        m = max(w, h)
        size = (max(int(h / m * self.image_size), self.min_size), max(int(w / m * self.image_size), self.min_size))
        if w <= 0 or h <= 0:
            raise ValueError("Invalid size!")
        if (h, w) != size:
            pil_img = pil_img.resize((size[1], size[0]), Image.BICUBIC)
        pil_img = expand2square(pil_img, self.background_color)
        return np.asarray(pil_img).transpose(2, 0, 1)  # [3, H, W] uint8

    def preprocess(self, images: Sequence) -> Dict[str, torch.Tensor]:
        out = []
        for im in images:
            x = (self.resize(im).astype(np.float64) * self.rescale_factor).astype(np.float32)
            if self.do_normalize:
                mean = np.asarray(self.image_mean, dtype=np.float32)[:, None, None]
                std = np.asarray(self.image_std, dtype=np.float32)[:, None, None]
                x = (x - mean) / std
            out.append(torch.from_numpy(np.ascontiguousarray(x)))
        return {"pixel_values": torch.stack(out)}

    __call__ = preprocess


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
    """HF tokenizer from ``path`` (the reference loads it with the processor from model_path,
    ospo/utils/model.py:26).  A given path that does not load is an error; the synthetic stand-in
    is used only when no path is given (offline synthetic runs)."""
    if path:
        from transformers import AutoTokenizer
        return AutoTokenizer.from_pretrained(path)
    return SyntheticTokenizer(vocab=vocab, bos_id=vocab - 2, pad_token_id=vocab - 1)


def _path_mapper(path_map) -> "callable":
    """``{old_prefix: new_prefix}`` or ``["OLD=NEW", ...]`` -> a path rewriter (the example
    train.json holds absolute paths of the authors' machine)."""
    if not path_map:
        pairs: List[Tuple[str, str]] = []
    elif isinstance(path_map, dict):
        pairs = [(str(k), str(v)) for k, v in path_map.items()]
    else:
        pairs = [tuple(str(m).split("=", 1)) for m in path_map]

    def remap(p: str) -> str:
        for old, new in pairs:
            if p.startswith(old):
                return new + p[len(old):]
        return p
    return remap


class PreferenceDataset(Dataset):
    """Same constructor as the reference (seed, data_path, chat_processor, image_processor,
    tokenizer, sampling_rate, num_samples) plus the image-source keywords above."""

    def __init__(self, seed: int, data_path: str, chat_processor=None, image_processor=None, tokenizer=None,
                 sampling_rate: float = 1.0, num_samples: Optional[int] = None, token_cache: Optional[str] = None,
                 synthetic_tokens: bool = False, img_vocab: int = 16384,
                 n_img_tokens: int = IMAGE_TOKEN_NUM_PER_IMAGE, path_map=None):
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
        if tokenizer is None:
            raise ValueError("PreferenceDataset needs a tokenizer")
        self.tokenizer = tokenizer
        self.chat_processor = chat_processor or ChatProcessor(tokenizer)
        self.image_processor = image_processor or VLMImageProcessor()
        self.cache = np.load(token_cache, allow_pickle=False) if token_cache else None
        self.synthetic = bool(synthetic_tokens) and self.cache is None
        self.img_vocab, self.n_img = img_vocab, n_img_tokens
        self.remap = _path_mapper(path_map)

    def __len__(self):
        return len(self.dataset)

    def __getitem__(self, idx):
        return self.decode(self.dataset[idx])

    def collate_fn(self, batch):
        item_ids, text_tokens, chosen, rejected = zip(*batch)
        return list(item_ids), list(text_tokens), list(chosen), list(rejected)

    def get_image_generation_prompt(self, prompt: str) -> str:
        conv = [{"role": "User", "content": prompt}, {"role": "Assistant", "content": ""}]
        sft = self.chat_processor.apply_sft_template_for_multi_turn_prompts(conversations=conv, sft_format="deepseek",
                                                                            system_prompt="")
        return sft + self.chat_processor.image_start_tag

    def get_text_token(self, text: str) -> torch.Tensor:
        ids = self.tokenizer.encode(self.get_image_generation_prompt(text))
        return torch.tensor(ids, dtype=torch.int32).view(1, -1)

    def get_image_tensor(self, img_path: str) -> torch.Tensor:
        """train_dataset.py:79-84: f32 [1, 3, 384, 384] pixel_values."""
        from PIL import Image
        with Image.open(self.remap(img_path)) as im:
            return self.image_processor([im.convert("RGB")])["pixel_values"]

    def get_image(self, example: Dict, side: str) -> torch.Tensor:
        item_id = example["item_id"]
        if self.cache is not None:
            return torch.from_numpy(self.cache[f"{item_id}/{side}"].astype(np.int64)).view(1, -1)
        if self.synthetic:
            seed = int(hashlib.md5(f"{item_id}/{side}".encode()).hexdigest(), 16) % (2 ** 31)
            g = torch.Generator().manual_seed(seed)
            return torch.randint(0, self.img_vocab, (1, self.n_img), generator=g)
        return self.get_image_tensor(example[side])

    def decode(self, example: Dict):
        if "prompt" not in example or "chosen" not in example or "rejected" not in example:
            raise ValueError("Could not format example as dialogue for SimPO task!\n"
                             f"This example only has {example.keys()} keys.\n")
        return (example["item_id"], self.get_text_token(example["prompt"]), self.get_image(example, "chosen"),
                self.get_image(example, "rejected"))


def train_dataloader(config, tokenizer, rank: int = 0, world: int = 1, img_vocab: int = 16384,
                     chat_processor=None, image_processor=None) -> DataLoader:
    """TrainDataModule.train_dataloader (datamodule.py:35-43) + the DistributedSampler PL's DDP adds."""
    tr = config["dataset"]["train"]
    ds = PreferenceDataset(seed=config["experiment"]["seed"], data_path=tr["data_path"], chat_processor=chat_processor,
                           image_processor=image_processor, tokenizer=tokenizer, num_samples=tr.get("num_samples"),
                           token_cache=tr.get("token_cache"), synthetic_tokens=tr.get("synthetic_tokens", False),
                           img_vocab=img_vocab, path_map=tr.get("path_map"))
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True,
                                 seed=config["experiment"]["seed"]) if world > 1 else None
    return DataLoader(ds, batch_size=tr["batch_size"], shuffle=sampler is None, sampler=sampler,
                      collate_fn=ds.collate_fn, num_workers=tr.get("num_workers") or 0, drop_last=False)
