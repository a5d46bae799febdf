"""Golden vectors of the VQ image tokenizer from the REFERENCE's own code (this container only).

Run:  python tests/golden/make_golden_vq.py          (needs /root/reference)

Loads ``janus/models/vq_model.py`` from the reference tree (importlib; it depends on torch only),
builds ``VQModel(ModelArgs())`` (the VQ-16 gen_vision_model of Janus-Pro), loads the seeded weights of
``oracle.vq_ref.init_vq_weights`` into it (no checkpoint exists offline; the decoder keeps its own
init and is not used) and runs ``encode`` in fp32, eval mode, on example PNGs of the reference
(``examples/step3/...``): two at 128 px and one at 384 px.  The pixels are the reference's own
``VLMImageProcessor`` output (``image_processing_vlm.py:127-192`` at image_size 128 / 384, mean = std
= 0.5; loaded as ``make_golden_image.py`` loads it): bicubic resize, then x/255 in f64 -> f32,
then (x - 0.5) / 0.5 in f32.

Output ``tests/golden/vq_golden.npz`` (data only): the uint8 pixels after the processor's resize,
the sha256 of the f32 pixel tensor the processor made of them, the weight seed, the reference's indices (``encode(x)[2][2]``, what train.py:257-258 keeps), its
quant_conv output z and the top-2 distance margin per token.

Decoder (step 3, ``image_generation.py:174-181``): with ``oracle.vq_ref.init_vq_decoder_weights(DEC_SEED)``
loaded as well, the reference's ``decode_code`` of image 0's ids (128 px, decoded in full, fp32) and of
image 2's ids (384 px: the uint8 image of image_generation.py:175-181 plus a strided fp32 sample),
into ``tests/golden/vq_decode_golden.npz``.
"""
from __future__ import annotations

import hashlib
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

sys.path.insert(0, HERE)
from make_golden_image import load_reference_processor  # noqa: E402

IMAGES = [("examples/step3/negative/layout/1000003/01.png", 128),
          ("examples/step3/negative/layout/1000005/00.png", 128),
          ("examples/step3/negative/layout/1000001/02.png", 384)]
SEED = 7
DEC_SEED = 11


def main():
    spec = importlib.util.spec_from_file_location("ref_vq_model", os.path.join(REF, "janus/models/vq_model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(0)
    model = mod.VQModel(mod.ModelArgs()).eval()
    w = V.init_vq_weights(SEED)
    w.update(V.init_vq_decoder_weights(DEC_SEED))
    missing, unexpected = model.load_state_dict(w, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith("quantize.codebook_used") for k in missing), missing
    out = {"seed": np.int64(SEED)}
    torch.set_num_threads(8)
    ip = load_reference_processor()
    for i, (rel, size) in enumerate(IMAGES):
        from PIL import Image
        im = Image.open(os.path.join(REF, rel)).convert("RGB")
        # the reference's own VLMImageProcessor at image_size = size (Janus-Pro mean = std = 0.5)
        proc = ip.VLMImageProcessor(image_size=size, image_mean=ip.IMAGENET_INCEPTION_MEAN,
                                    image_std=ip.IMAGENET_INCEPTION_STD, do_normalize=True)
        u8 = np.ascontiguousarray(proc.resize(im).transpose(1, 2, 0)).astype(np.uint8)
        x = torch.as_tensor(proc([im])["pixel_values"])
        assert x.dtype == torch.float32 and tuple(x.shape) == (1, 3, size, size)
        out[f"img{i}_px_sha256"] = np.array(hashlib.sha256(x.numpy().tobytes()).hexdigest())
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
    dec = {"seed": np.int64(SEED), "dec_seed": np.int64(DEC_SEED)}
    with torch.no_grad():
        d0 = model.decode_code(torch.from_numpy(out["img0_ids"]).view(1, -1).int(), shape=[1, 8, 8, 8])
        d2 = model.decode_code(torch.from_numpy(out["img2_ids"]).view(1, -1).int(), shape=[1, 8, 24, 24])
    dec["img0_dec"] = d0.numpy().astype(np.float32)
    a2 = d2.numpy().astype(np.float32)
    dec["img2_dec_sample"] = a2.reshape(-1)[::101].copy()
    # image_generation.py:175-181
    img = np.clip((a2.transpose(0, 2, 3, 1) + 1) / 2 * 255, 0, 255)
    u8 = np.zeros(img.shape, dtype=np.uint8)
    u8[:] = img
    dec["img2_u8"] = u8
    np.savez_compressed(os.path.join(HERE, "vq_decode_golden.npz"), **dec)
    print("decode: 128 px", d0.shape, "384 px", d2.shape)


if __name__ == "__main__":
    main()
