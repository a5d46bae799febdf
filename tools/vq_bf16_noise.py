"""How reproducible are the reference's bf16 VQ ids?  (this container only: needs /root/reference)

Runs the reference's own ``janus/models/vq_model.py`` in bf16 on the 384-px golden image (the seeded
weights of ``tests/golden/make_golden_vq.py``), then three restatements on the same bf16 pixels:
  fp32      -- ``oracle.vq_ref.encode_ref`` (what ``ospo_amd.vq.VQEncoder`` computes);
  bf16-f32  -- every rounding point of the bf16 module tree restated (conv = bf16(fp32 acc + bias),
               GroupNorm bf16, swish = bf16(y * bf16(sigmoid y)), residual adds, bmm, the attention
               scale, softmax, the bf16 quantizer: normalise, |z|^2, |e|^2, z.e, d), fp32 accumulation;
  bf16-f64  -- the same rounding points with fp64-accumulated convolutions.
Output: one JSON line, the number of ids each restatement disagrees on with the reference's bf16 run.
"""
import importlib.util
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from oracle import vq_ref as V  # noqa: E402
from make_golden_image import load_reference_processor  # noqa: E402

REF = "/root/reference"


def rb(t):
    return t.bfloat16().float()


def bf16_restated(x, w, acc):
    def gn(x, p, swish):
        y = rb(F.group_norm(x, 32, w[p + ".weight"], w[p + ".bias"], eps=1e-6))
        return rb(y * rb(torch.sigmoid(y))) if swish else y

    def conv(x, p, stride=1, padding=1):
        return rb(F.conv2d(x.to(acc), w[p + ".weight"].to(acc), w[p + ".bias"].to(acc), stride=stride,
                           padding=padding))

    for kind, p, cin, cout, k in V.encoder_plan():
        if kind == "conv":
            x = conv(x, p, padding=k // 2)
        elif kind == "down":
            x = conv(F.pad(x, (0, 1, 0, 1)), p, stride=2, padding=0)
        elif kind == "res":
            h = conv(gn(x, p + ".norm1", True), p + ".conv1")
            h = conv(gn(h, p + ".norm2", True), p + ".conv2")
            if cin != cout:
                x = conv(x, p + ".nin_shortcut", padding=0)
            x = rb(x + h)
        elif kind == "attn":
            h = gn(x, p + ".norm", False)
            q, kk, v = (conv(h, p + "." + n, padding=0) for n in ("q", "k", "v"))
            b, c, hh, ww = q.shape
            a = rb(torch.bmm(q.reshape(b, c, hh * ww).permute(0, 2, 1), kk.reshape(b, c, hh * ww)))
            a = rb(F.softmax(rb(a * (int(c) ** (-0.5))), dim=2))
            o = rb(torch.bmm(v.reshape(b, c, hh * ww), a.permute(0, 2, 1))).reshape(b, c, hh, ww)
            x = rb(x + conv(o, p + ".proj_out", padding=0))
        elif kind == "norm_out":
            x = gn(x, p, True)
    b, e, h, ww = x.shape
    zf = x.permute(0, 2, 3, 1).reshape(-1, e)

    def nrm(t):
        return rb(t / rb(t.norm(dim=-1, keepdim=True)).clamp_min(1e-12))

    zf, emb = nrm(zf), nrm(w["quantize.embedding.weight"])
    d = rb(rb(rb(rb(zf * zf).sum(1, keepdim=True)) + rb(rb(emb * emb).sum(1))) - 2 * rb(zf @ emb.t()))
    return torch.argmin(d, dim=1)


def main():
    torch.set_num_threads(8)
    spec = importlib.util.spec_from_file_location("ref_vq_model", os.path.join(REF, "janus/models/vq_model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    W = V.init_vq_weights(7)
    model = mod.VQModel(mod.ModelArgs()).eval()
    model.load_state_dict(W, strict=False)
    model = model.bfloat16()
    from PIL import Image
    ip = load_reference_processor()
    im = Image.open(os.path.join(REF, "examples/step3/negative/layout/1000001/02.png")).convert("RGB")
    proc = ip.VLMImageProcessor(image_size=384, image_mean=ip.IMAGENET_INCEPTION_MEAN,
                                image_std=ip.IMAGENET_INCEPTION_STD, do_normalize=True)
    x = torch.as_tensor(proc([im])["pixel_values"])
    with torch.no_grad():
        ref = model.quantize(model.quant_conv(model.encoder(x.bfloat16())))[2][2].reshape(-1)
        wb = {k: rb(v) for k, v in W.items()}
        out = {"tokens": int(ref.numel())}
        out["fp32_differ"] = int((V.encode_ref(x, W)[0].reshape(-1) != ref).sum())
        out["bf16_f32acc_differ"] = int((bf16_restated(rb(x), wb, torch.float32) != ref).sum())
        out["bf16_f64acc_differ"] = int((bf16_restated(rb(x), wb, torch.float64) != ref).sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
