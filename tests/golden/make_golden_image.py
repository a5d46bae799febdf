"""Golden pixel tensors of the REFERENCE's image processor (this container only).

Run:  python tests/golden/make_golden_image.py          (needs /root/reference)

Runs the reference's own ``janus/models/image_processing_vlm.py`` ``VLMImageProcessor`` --
``resize`` (:127-162: long side to image_size, bicubic + antialias, ``expand2square`` with the
mean colour) and ``preprocess`` (:164-192: HF ``rescale`` 1/255, HF ``normalize``) -- the call
``ospo/dataclass/train_dataset.py:79-84`` makes for every chosen / rejected PNG, with the Janus-Pro
generation settings (image_size 384, mean = std = 0.5: IMAGENET_INCEPTION_MEAN / _STD, :37-38).

``rescale`` / ``normalize`` are the container's transformers (5.15; the reference pins 4.38.2,
whose two functions are the same f64-scale-then-f32 and f32 ``(x - mean) / std``).  The module
is executed from its source without its ``AutoImageProcessor.register`` statement (:199),
because transformers 5 gates that registry on torchvision.
torchvision is absent: ``torchvision.transforms.functional.resize`` is stubbed by what its PIL
path does (torchvision 0.15, the version torch 2.0.1 pins): return the image unchanged when the
size already matches, else ``img.resize((w, h), PIL.Image.BICUBIC)`` (PIL's filter always
antialiases, so ``antialias=True`` is what it does anyway).

Images: the five example PNGs under ``tests/golden/step3`` (384 x 384: the resize is the
identity) and three derived from the first of them, so the resize and the padding run:
a 500 x 320 landscape crop (downsampled to 384 x 245, padded top/bottom), the image upscaled to
512 x 512 (downsampled to 384 x 384) and a 200 x 300 portrait crop (upsampled to 256 x 384, padded
left/right).  The derived inputs are stored as uint8 arrays, so the test needs no reference.

Output ``tests/golden/image_golden.npz`` (data only): per case the sha256 of the reference's f32
[1, 3, 384, 384] ``pixel_values`` bytes and a strided sample of them, plus the uint8 HWC input of
each derived case.
"""
from __future__ import annotations

import glob
import hashlib
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def install_torchvision_stub():
    from PIL import Image

    class InterpolationMode:
        BICUBIC = "bicubic"

    def resize(img, size, interpolation=None, antialias=None):
        assert interpolation == InterpolationMode.BICUBIC
        h, w = int(size[0]), int(size[1])
        if (img.size[1], img.size[0]) == (h, w):
            return img
        return img.resize((w, h), Image.BICUBIC)

    tv = types.ModuleType("torchvision")
    tr = types.ModuleType("torchvision.transforms")
    fn = types.ModuleType("torchvision.transforms.functional")
    fn.resize, fn.InterpolationMode = resize, InterpolationMode
    tv.transforms, tr.functional = tr, fn
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tr, "torchvision.transforms.functional": fn})


def load_reference_processor():
    """The reference module, executed from its source minus the module-level
    ``AutoImageProcessor.register(...)`` statement (:199): transformers 5 gates that registry on
    torchvision, and the registration does no arithmetic."""
    import ast
    import transformers  # noqa: F401  (before the stub: transformers probes for torchvision with find_spec)
    install_torchvision_stub()
    path = os.path.join(REF, "janus/models/image_processing_vlm.py")
    tree = ast.parse(open(path).read(), path)
    tree.body = [n for n in tree.body
                 if not (isinstance(n, ast.Expr) and isinstance(n.value, ast.Call)
                         and ast.unparse(n.value.func) == "AutoImageProcessor.register")]
    mod = types.ModuleType("ref_image_processing_vlm")
    mod.__file__ = path
    sys.modules[mod.__name__] = mod  # the config class is made a dataclass, which looks its module up
    exec(compile(tree, path, "exec"), mod.__dict__)
    return mod


def cases():
    from PIL import Image
    pngs = sorted(glob.glob(os.path.join(HERE, "step3", "**", "*.png"), recursive=True))
    out = []
    for p in pngs:
        with Image.open(p) as im:
            out.append((os.path.relpath(p, HERE), np.asarray(im.convert("RGB")).copy()))
    base = Image.fromarray(out[0][1])
    out.append(("landscape_500x320", np.asarray(base.resize((500, 500), Image.BICUBIC).crop((0, 90, 500, 410)))))
    out.append(("square_512", np.asarray(base.resize((512, 512), Image.BICUBIC))))
    out.append(("portrait_200x300", np.asarray(base.crop((50, 20, 250, 320)))))
    return out


def main():
    from PIL import Image
    mod = load_reference_processor()
    proc = mod.VLMImageProcessor(image_size=384, image_mean=mod.IMAGENET_INCEPTION_MEAN,
                                 image_std=mod.IMAGENET_INCEPTION_STD, do_normalize=True)
    out = {}
    names = []
    for i, (name, arr) in enumerate(cases()):
        px = proc([Image.fromarray(arr)])["pixel_values"]
        a = px.numpy() if hasattr(px, "numpy") else np.asarray(px)
        assert a.dtype == np.float32 and a.shape == (1, 3, 384, 384), (a.dtype, a.shape)
        if not name.endswith(".png"):  # derived inputs: stored (the example PNGs are in tests/golden/step3)
            out[f"in{i}"] = arr.astype(np.uint8)
        out[f"px{i}_sha256"] = np.array(hashlib.sha256(a.tobytes()).hexdigest())
        out[f"px{i}_sample"] = a.reshape(-1)[::331].copy()
        names.append(name)
    out["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "image_golden.npz"), **out)
    print("wrote image_golden.npz:", names)


if __name__ == "__main__":
    main()
