"""Golden batch of the REFERENCE's step-5 dataset (this container only).

Run:  python tests/golden/make_golden_dataset.py          (needs /root/reference)

Runs the reference's own ``ospo/dataclass/train_dataset.py`` ``PreferenceDataset`` +
``collate_fn`` -- the loader ``ospo/step5.py:17-23`` builds -- on the example pairs of
``tests/golden/train_pixels.json`` with the processor objects ``ospo_amd.model.get_model``
returns (``ChatProcessor``, ``VLMImageProcessor``) and the synthetic tokenizer, i.e. what
INTEGRATION.md §2's import swap hands to the reference's unchanged dataloader.  Absent
third-party modules (pyrootutils, janus processing / torchvision) are stubbed; they hold no
arithmetic on this path.

Output ``tests/golden/dataset_batch.npz`` (data only): item ids, the int text tokens and the
sha256 + a strided sample of every f32 pixel tensor of the collated batch.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def install_stubs():
    pr = types.ModuleType("pyrootutils")
    pr.setup_root = lambda *a, **k: None
    sys.modules["pyrootutils"] = pr
    # ospo.utils.processor imports these two names only to type the generation helpers
    pv = types.ModuleType("janus.models.processing_vlm")
    pv.VLChatProcessorOutput = pv.BatchedVLChatProcessorOutput = object
    for name in ("janus", "janus.models"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["janus.models.processing_vlm"] = pv


def load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    install_stubs()
    sys.path.insert(0, REF)
    common = types.ModuleType("ospo.utils.common")  # its read_json is json.load; the module pulls in omegaconf
    common.read_json = lambda p: json.load(open(p))
    for name in ("ospo", "ospo.utils"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["ospo.utils.common"] = common
    load("ospo.utils.processor", "ospo/utils/processor.py")
    ds_mod = load("ospo_ref_train_dataset", "ospo/dataclass/train_dataset.py")
    from ospo_amd.data import ChatProcessor, SyntheticTokenizer, VLMImageProcessor
    items = json.load(open(os.path.join(HERE, "train_pixels.json")))
    for ex in items:  # the reference has no path map: point the pairs at the example tree
        for k in ("chosen", "rejected"):
            ex[k] = ex[k].replace("/home/elicer/OSPO/example", os.path.join(REF, "examples"))
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(items, f)
    tok = SyntheticTokenizer()
    ds = ds_mod.PreferenceDataset(seed=42, data_path=f.name, chat_processor=ChatProcessor(tok),
                                  image_processor=VLMImageProcessor(), tokenizer=tok)
    ids, text, ch, rj = ds.collate_fn([ds[i] for i in range(len(ds))])
    out = {"item_ids": np.array(ids)}
    for i, t in enumerate(text):
        out[f"text{i}"] = t.numpy().astype(np.int32)
    for side, ts in (("chosen", ch), ("rejected", rj)):
        for i, t in enumerate(ts):
            a = t.numpy()
            assert a.dtype == np.float32 and a.shape == (1, 3, 384, 384)
            out[f"{side}{i}_sha256"] = np.array(hashlib.sha256(a.tobytes()).hexdigest())
            out[f"{side}{i}_sample"] = a.reshape(-1)[::997].copy()
    np.savez_compressed(os.path.join(HERE, "dataset_batch.npz"), **out)
    os.unlink(f.name)
    print("wrote dataset_batch.npz:", list(ids), [tuple(t.shape) for t in text])


if __name__ == "__main__":
    main()
