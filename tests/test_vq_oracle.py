"""CPU: the VQ tokenizer oracle (oracle/vq_ref.py) against the vectors the reference's own
janus/models/vq_model.py produced (tests/golden/make_golden_vq.py): identical ids, z to fp32 noise."""
import os

import numpy as np
import torch

from tests import fixtures as FX

from oracle import vq_ref as V

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vq_golden.npz")


def test_vq_oracle_matches_reference_golden():
    z = np.load(GOLD)
    w = V.init_vq_weights(int(z["seed"]))
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    for i in range(3):
        x = FX.golden_vq_pixels(z, i)  # the reference processor's pixels (sha256-checked)
        ids, zq, margin = V.encode_ref(x, w)
        assert torch.equal(ids.reshape(-1), torch.from_numpy(z[f"img{i}_ids"]))
        ref = torch.from_numpy(z[f"img{i}_z"])
        assert float((zq[0] - ref).abs().max() / ref.abs().max()) < 1e-4


def test_vq_weight_names_and_plan():
    w = V.init_vq_weights(0)
    assert w["encoder.conv_in.weight"].shape == (128, 3, 3, 3)
    assert w["encoder.conv_blocks.2.res.0.nin_shortcut.weight"].shape == (256, 128, 1, 1)
    assert w["encoder.conv_blocks.4.attn.1.proj_out.weight"].shape == (512, 512, 1, 1)
    assert w["quant_conv.weight"].shape == (8, 256, 1, 1)
    cb = w["quantize.embedding.weight"]
    assert cb.shape == (16384, 8) and torch.allclose(cb.norm(dim=1), torch.ones(16384), atol=1e-6)
    kinds = [k for k, *_ in V.encoder_plan()]
    assert kinds.count("down") == 4 and kinds.count("attn") == 3 and kinds.count("res") == 12


def test_vq_decoder_oracle_matches_reference_golden():
    """decode_code (image_generation.py:174) restated: the reference's own vq_model.py decode of the
    golden ids (tests/golden/make_golden_vq.py, seeded decoder weights), fp32; the uint8 image of
    image_generation.py:175-181 equal except where a value sits within fp32 noise of an integer."""
    z = np.load(GOLD)
    d = np.load(GOLD.replace("vq_golden", "vq_decode_golden"))
    w = V.init_vq_weights(int(d["seed"]))
    w.update(V.init_vq_decoder_weights(int(d["dec_seed"])))
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    d0 = V.decode_code_ref(torch.from_numpy(z["img0_ids"]).view(1, -1), w, 8, 8)
    ref0 = torch.from_numpy(d["img0_dec"])
    assert float((d0 - ref0).abs().max() / ref0.abs().max()) < 1e-5
    d2 = V.decode_code_ref(torch.from_numpy(z["img2_ids"]).view(1, -1), w, 24, 24)
    s = d2.reshape(-1)[::101].numpy()
    assert float(np.abs(s - d["img2_dec_sample"]).max() / np.abs(d["img2_dec_sample"]).max()) < 1e-5
    u8 = V.to_uint8_images(d2)
    diff = np.abs(u8.astype(np.int16) - d["img2_u8"].astype(np.int16))
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3


def test_vq_decoder_plan():
    w = V.init_vq_decoder_weights(0)
    assert w["post_quant_conv.weight"].shape == (256, 8, 1, 1)
    assert w["decoder.conv_in.weight"].shape == (512, 256, 3, 3)
    assert w["decoder.conv_blocks.1.res.0.nin_shortcut.weight"].shape == (256, 512, 1, 1)
    assert w["decoder.conv_blocks.3.upsample.conv.weight"].shape == (128, 128, 3, 3)
    assert w["decoder.conv_out.weight"].shape == (3, 128, 3, 3)
    kinds = [k for k, *_ in V.decoder_plan()]
    assert kinds.count("up") == 4 and kinds.count("attn") == 4 and kinds.count("res") == 17
