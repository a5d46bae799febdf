"""VQ image tokenizer on the MI355X, through the C ABI: the f32-MFMA convolution,
GroupNorm and quantizer against fp32 torch / the oracle, and the whole encoder against the ids the
reference's own janus/models/vq_model.py produced (tests/golden/vq_golden.npz) -- exact ids."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests import fixtures as FX

from oracle import vq_ref as V

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vq_golden.npz")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from ospo_amd import _lib
    _lib.lib()
    torch.manual_seed(0)


def call(*a):
    from ospo_amd._lib import call as c
    return c(*a)


def s():
    return torch.cuda.current_stream().cuda_stream


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,stride,pad,res", [
    (2, 32, 32, 3, 128, 3, 1, 1, False), (1, 24, 24, 64, 96, 3, 1, 1, True), (2, 16, 16, 64, 64, 1, 1, 0, False),
    (1, 48, 48, 128, 128, 3, 2, 0, False), (3, 8, 8, 256, 8, 1, 1, 0, False), (1, 20, 12, 40, 70, 3, 1, 1, True)])
def test_conv2d_f32(B, H, W, Cin, Cout, k, stride, pad, res):
    x = torch.randn(B, Cin, H, W)
    w = torch.randn(Cout, Cin, k, k) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout)
    if stride == 2:  # Downsample: pad (0, 1, 0, 1), then a stride-2 3x3 conv without padding
        ref = F.conv2d(F.pad(x, (0, 1, 0, 1)), w, b, stride=2)
    else:
        ref = F.conv2d(x, w, b, stride=stride, padding=pad)
    Ho, Wo = ref.shape[2], ref.shape[3]
    r = torch.randn(B, Ho, Wo, Cout) if res else None
    if res:
        ref = ref + r.permute(0, 3, 1, 2)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    wd = w.permute(0, 2, 3, 1).contiguous().to(DEV)
    out = torch.empty(B, Ho, Wo, Cout, device=DEV)
    bd = b.to(DEV)
    rd = r.to(DEV) if res else None  # device copies held for the call (a temporary's pointer would dangle)
    call("ospo_vq_conv2d", xd.data_ptr(), B, H, W, Cin, wd.data_ptr(), Cout, k, k, stride, pad, pad, Ho, Wo,
         bd.data_ptr(), rd.data_ptr() if res else None, out.data_ptr(), s())
    assert relerr(out.cpu().permute(0, 3, 1, 2), ref) < 2e-6


def test_groupnorm_swish_and_attention_products():
    B, H, W, C = 2, 24, 24, 512
    x = torch.randn(B, C, H, W) * 3 + 1
    g, b = 1 + torch.randn(C) * 0.1, torch.randn(C) * 0.1
    ref = F.group_norm(x, 32, g, b, eps=1e-6)
    ref = ref * torch.sigmoid(ref)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    out = torch.empty_like(xd)
    from ospo_amd._lib import query
    ws = torch.empty(query("ospo_vq_groupnorm_ws_bytes", B, 32) // 4 + 4, device=DEV)
    gd, bd = g.to(DEV), b.to(DEV)
    call("ospo_vq_groupnorm", xd.data_ptr(), B, H * W, C, 32, gd.data_ptr(), bd.data_ptr(), 1e-6, 1,
         out.data_ptr(), ws.data_ptr(), ws.numel() * 4, s())
    assert relerr(out.cpu().permute(0, 3, 1, 2), ref) < 1e-6
    n = H * W
    q, k = torch.randn(B, n, C), torch.randn(B, n, C)
    sc = torch.empty(B, n, n, device=DEV)
    qd, kd = q.to(DEV), k.to(DEV)
    call("ospo_vq_bmm_nt", qd.data_ptr(), kd.data_ptr(), B, n, n, C, sc.data_ptr(), s())
    ref = torch.bmm(q, k.transpose(1, 2))
    assert relerr(sc.cpu(), ref) < 2e-6
    call("ospo_vq_softmax_rows", sc.data_ptr(), B * n, n, float(C ** -0.5), s())
    assert relerr(sc.cpu(), torch.softmax(ref * C ** -0.5, -1)) < 1e-5
    vt = torch.empty(B, C, n, device=DEV)
    v = torch.randn(B, n, C).to(DEV)
    call("ospo_vq_transpose", v.data_ptr(), B, n, C, vt.data_ptr(), s())
    assert torch.equal(vt, v.transpose(1, 2).contiguous())


def test_quantize_matches_oracle_given_z():
    torch.manual_seed(1)
    cb = V.init_vq_weights(3)["quantize.embedding.weight"]
    z = torch.randn(4, 8, 24, 24)
    ids_ref, margin = V.quantize_ref(z, cb)
    cbn = torch.empty(16384, 8, device=DEV)
    cbd = cb.to(DEV)
    call("ospo_vq_l2norm_rows", cbd.data_ptr(), 16384, 8, cbn.data_ptr(), s())
    zd = z.permute(0, 2, 3, 1).contiguous().to(DEV)
    ids = torch.empty(4 * 576, dtype=torch.int32, device=DEV)
    call("ospo_vq_quantize", zd.data_ptr(), 4 * 576, 8, cbn.data_ptr(), 16384, ids.data_ptr(), None, s())
    ids = ids.cpu().long().view(4, 576)
    diff = ids != ids_ref
    # only exact near-ties may differ (fp32 summation order of |z|^2 + |e|^2 - 2 z.e)
    assert bool((margin[diff] < 1e-6).all()), margin[diff]
    assert int(diff.sum()) <= 2


def test_encoder_matches_reference_golden_ids():
    from ospo_amd.vq import VQEncoder
    z = np.load(GOLD)
    enc = VQEncoder(V.init_vq_weights(int(z["seed"])), device=DEV)
    for i in range(3):
        x = FX.golden_vq_pixels(z, i)  # the reference processor's pixels (sha256-checked)
        ids, zq, _ = enc.encode(x, return_z=True)
        ref_ids = torch.from_numpy(z[f"img{i}_ids"])
        ref_z = torch.from_numpy(z[f"img{i}_z"])  # [8, h, w]
        zz = zq[0].permute(2, 0, 1).cpu()
        print(f"\nimg{i}: {ref_ids.numel()} tokens, z rel err {relerr(zz, ref_z):.2e}, "
              f"id mismatches {int((ids.cpu().long().view(-1) != ref_ids).sum())}")
        assert relerr(zz, ref_z) < 1e-5
        assert torch.equal(ids.cpu().long().view(-1), ref_ids)


def test_token_cache_cli_reads_step5_json(tmp_path):
    """python -m ospo_amd.vq over a step-5 train.json: PNG -> VLMImageProcessor pixels -> ids, keyed
    "{item_id}/chosen|rejected" as the SimPO dataloader reads them (ospo_amd/data.py)."""
    import json
    from PIL import Image
    from ospo_amd import vq
    z = np.load(GOLD)
    png = tmp_path / "img.png"
    Image.fromarray(z["img2_u8"]).save(png)
    data = [{"item_id": "0000042", "prompt": "a cat", "chosen": "/old/root/img.png", "rejected": str(png)}]
    jp = tmp_path / "train.json"
    jp.write_text(json.dumps(data))
    out = tmp_path / "cache.npz"
    vq.main(["--data-path", str(jp), "--out", str(out), "--seed", str(int(z["seed"])),
             "--path-map", f"/old/root={tmp_path}"])
    cache = np.load(out)
    assert sorted(cache.files) == ["0000042/chosen", "0000042/rejected"]
    for k in cache.files:
        assert np.array_equal(cache[k].astype(np.int64), z["img2_ids"])


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 12, 12, 128, 128), (1, 24, 24, 512, 512), (1, 7, 5, 40, 70)])
def test_conv2d_up2_equals_upsample_then_conv(B, H, W, Cin, Cout):
    """The Upsample (nearest 2x, vq_model.py:411-427) read on the fly by the convolution: bit-identical to
    the convolution of the explicitly upsampled tensor (same gathers, same order)."""
    x = torch.randn(B, H, W, Cin, device=DEV)
    w = (torch.randn(Cout, 3, 3, Cin) / (9 * Cin) ** 0.5).to(DEV)
    b = torch.randn(Cout, device=DEV)
    up = x.repeat_interleave(2, 1).repeat_interleave(2, 2).contiguous()
    a = torch.empty(B, 2 * H, 2 * W, Cout, device=DEV)
    c = torch.empty_like(a)
    call("ospo_vq_conv2d", up.data_ptr(), B, 2 * H, 2 * W, Cin, w.data_ptr(), Cout, 3, 3, 1, 1, 1, 2 * H, 2 * W,
         b.data_ptr(), None, a.data_ptr(), s())
    call("ospo_vq_conv2d_up2", x.data_ptr(), B, H, W, Cin, w.data_ptr(), Cout, 3, 3, 1, b.data_ptr(), None,
         c.data_ptr(), s())
    torch.cuda.synchronize()
    assert torch.equal(a, c)


def test_decoder_matches_reference_golden():
    """decode_code (image_generation.py:174) on the GPU against the reference's own vq_model.py decode of
    the golden ids (tests/golden/vq_decode_golden.npz): fp32 decode to fp32 noise; the uint8 images of
    image_generation.py:175-181 equal but for values within fp32 noise of an integer (+-1)."""
    from ospo_amd.vq import VQDecoder
    z = np.load(GOLD)
    d = np.load(GOLD.replace("vq_golden", "vq_decode_golden"))
    w = V.init_vq_weights(int(d["seed"]))
    w.update(V.init_vq_decoder_weights(int(d["dec_seed"])))
    dec = VQDecoder(w, device=DEV)
    o0 = dec.decode_code(torch.from_numpy(z["img0_ids"]).view(1, -1), 8, 8)
    ref0 = torch.from_numpy(d["img0_dec"]).permute(0, 2, 3, 1)
    e0 = float((o0.cpu() - ref0).abs().max() / ref0.abs().max())
    o2 = dec.decode_code(torch.from_numpy(z["img2_ids"]).view(1, -1), 24, 24)
    smp = o2.permute(0, 3, 1, 2).reshape(-1)[::101].cpu().numpy()
    e2 = float(np.abs(smp - d["img2_dec_sample"]).max() / np.abs(d["img2_dec_sample"]).max())
    u8 = dec.to_images(o2).cpu().numpy()
    diff = np.abs(u8.astype(np.int16) - d["img2_u8"].astype(np.int16))
    print(f"\nVQ decode: 128 px max rel err {e0:.2e}, 384 px sample {e2:.2e}, uint8 pixels off by 1: "
          f"{int((diff > 0).sum())} of {diff.size}")
    assert e0 < 1e-4 and e2 < 1e-4
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3


def test_generate_images_decodes_the_sampled_tokens():
    """T2IGenerator.generate_images = generate + decode_code + uint8 (image_generation.py:109-181) at
    small LLM width: the images are the decoder's images of the tokens generate() returns."""
    from ospo_amd.engine import ModelDims
    from ospo_amd.generate import T2IGenerator
    from ospo_amd.vq import VQDecoder
    from oracle import simpo_ref as O
    dims = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=16384, gen_head_dim=256)
    w = O.init_weights(dims, seed=23, dtype=torch.bfloat16, lora_b_std=1e-2)
    vw = V.init_vq_weights(1)
    vw.update(V.init_vq_decoder_weights(2))
    gen = T2IGenerator(ModelDims.from_any(dims), w, device=DEV, max_batch=2, max_prompt_len=16, n_img_tokens=64,
                       vq_weights=vw)
    prompts = [[5, 9, 200, 31], [7, 8, 9]]
    imgs = gen.generate_images(prompts, seed=4, img_size=128)
    tok = gen.generate(prompts, seed=4)
    dec = VQDecoder(vw, device=DEV)
    ref = dec.to_images(dec.decode_code(tok, 8, 8))
    assert imgs.shape == (2, 128, 128, 3) and imgs.dtype == torch.uint8
    assert torch.equal(imgs, ref)


def test_decoder_reproduces_reference_generate_image_pngs():
    """The HIP decoder on the tokens the reference's generate_image sampled (tests/golden/
    generate_golden.npz, make_golden_generate.py) writes the PNG pixels the reference saved (+-1 where
    a value sits within fp32 noise of an integer)."""
    from ospo_amd.vq import VQDecoder
    z = np.load(GOLD.replace("vq_golden", "generate_golden"))
    _, vq_seed, vq_dec_seed, _ = z["seeds"].tolist()
    w = V.init_vq_weights(int(vq_seed))
    w.update(V.init_vq_decoder_weights(int(vq_dec_seed)))
    dec = VQDecoder(w, device=DEV)
    u8 = dec.to_images(dec.decode_code(torch.from_numpy(z["tokens"]), 8, 8)).cpu().numpy()
    diff = np.abs(u8.astype(np.int16) - z["images_u8"].astype(np.int16))
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3
