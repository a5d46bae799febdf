"""Golden vectors of the VQ image tokenizer from the REFERENCE's own code (this container only).

Run:  python tests/golden/make_golden_vq.py          (needs /root/reference)

Loads ``janus/models/vq_model.py`` from the reference tree (importlib; it depends on torch only),
builds ``VQModel(ModelArgs())`` (the VQ-16 gen_vision_model of Janus-Pro), loads the seeded weights of
``oracle.vq_ref.init_vq_weights`` into it (no checkpoint exists offline; the decoder keeps its own
init and is not used) and runs ``encode`` in fp32, eval mode, on example PNGs of the reference
(``examples/step3/...``): two at 128 px (bicubic) and one at 384 px.

Output ``tests/golden/vq_golden.npz`` (data only): the uint8 pixels actually fed (after resize), the
weight seed, the reference's indices (``encode(x)[2][2]``, what train.py:257-258 keeps), its
quant_conv output z and the top-2 distance margin per token.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import vq_ref as V  # noqa: E402

IMAGES = [("examples/step3/negative/layout/1000003/01.png", 128),
          ("examples/step3/negative/layout/1000005/00.png", 128),
          ("examples/step3/negative/layout/1000001/02.png", 384)]
SEED = 7


def main():
    spec = importlib.util.spec_from_file_location("ref_vq_model", os.path.join(REF, "janus/models/vq_model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(0)
    model = mod.VQModel(mod.ModelArgs()).eval()
    w = V.init_vq_weights(SEED)
    missing, unexpected = model.load_state_dict(w, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith(("decoder.", "post_quant_conv.", "quantize.codebook_used")) for k in missing), missing
    out = {"seed": np.int64(SEED)}
    torch.set_num_threads(8)
    for i, (rel, size) in enumerate(IMAGES):
        from PIL import Image
        im = Image.open(os.path.join(REF, rel)).convert("RGB")
        if im.size != (size, size):
            im = im.resize((size, size), Image.BICUBIC)
        u8 = np.asarray(im, dtype=np.uint8).copy()
        x = (torch.from_numpy(u8).permute(2, 0, 1).float()[None] / 255.0 - 0.5) / 0.5
        with torch.no_grad():
            h = model.quant_conv(model.encoder(x))
            _, _, info = model.quantize(h)
        ids = info[2].reshape(-1)
        _, _, margin = None, None, V.quantize_ref(h, w["quantize.embedding.weight"])[1]
        out[f"img{i}_u8"] = u8
        out[f"img{i}_ids"] = ids.numpy().astype(np.int64)
        out[f"img{i}_z"] = h[0].numpy().astype(np.float32)
        out[f"img{i}_margin"] = margin.reshape(-1).numpy().astype(np.float32)
        print(rel, size, "tokens", ids.numel(), "min margin", float(margin.min()))
    np.savez_compressed(os.path.join(HERE, "vq_golden.npz"), **out)


if __name__ == "__main__":
    main()
