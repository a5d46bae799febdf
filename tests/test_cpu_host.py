"""CPU-side tests (no GPU): the C ABI library loads and exports every symbol
include/ospo_hip.h declares, its pre-launch validation returns the documented
status codes, and the host logic (LoRA layout, config, data, checkpoint layout,
FLOP model) behaves like the reference's."""
import ctypes
import json
import os
import types
import re
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ospo_hip.h")
LIB = os.path.join(ROOT, "ospo_amd", "libospo_hip.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "ospo_amd", "csrc"), "-j8"], check=True)
    from ospo_amd import _lib
    return _lib.lib()


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|unsigned|size_t|const char\*)\s+(ospo_[a-z0-9_]+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol(lib):
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/ospo_hip.h but not exported"
    from ospo_amd import _lib
    assert sorted(set(_lib.exported_symbols())) == syms, "ctypes signature table out of sync with the header"


def test_abi_version_and_strerror(lib):
    from ospo_amd import _lib
    assert lib.ospo_abi_version() == _lib.ABI_VERSION == 3
    assert lib.ospo_strerror(1) == b"shape / leading-dimension violation"


def test_workspace_counter_heads_from_the_library(lib):
    """The counter heads Python zeroes are the library's own sizes (no hard-coded 1024 / 2052)."""
    from ospo_amd import ops
    assert [ops.ws_counter_bytes(k) for k in (ops.WS_GEMM_TAIL, ops.WS_SKINNY, ops.WS_LORA_GDB,
                                               ops.WS_DECODE_LINEAR)] == [4096, 4096, 8208, 4096]
    assert lib.ospo_ws_counter_bytes(99) == 0
    ws = torch.full((4000,), 7.0)
    ops.zero_ws_counters(ws, ops.WS_LORA_GDB)
    assert int((ws == 0).sum()) == 8208 // 4 and float(ws[8208 // 4]) == 7.0


def test_clock_probe_validation_before_launch(lib):
    """ospo_gemm_clock_probe_bf16 (bench.py's box probe) refuses bad shapes, a short stamp buffer, null and
    misaligned pointers with a status before any HIP call."""
    P = ctypes.c_void_p
    buf = (ctypes.c_char * 4096)()
    a = ctypes.addressof(buf)
    st = 4 * 8 * 8  # (512 / 256)^2 tiles x 8 stamps x 8 B
    assert lib.ospo_gemm_clock_probe_bf16(P(a), P(a), P(a), 500, 512, 512, P(a), st, None) == 1  # M % 256
    assert lib.ospo_gemm_clock_probe_bf16(P(a), P(a), P(a), 512, 512, 96, P(a), st, None) == 1  # K % 64, K < 256
    assert lib.ospo_gemm_clock_probe_bf16(P(a), P(a), P(a), 512, 512, 512, P(a), st - 8, None) == 1  # stamps
    assert lib.ospo_gemm_clock_probe_bf16(P(a), P(a), None, 512, 512, 512, P(a), st, None) == 5  # null C
    assert lib.ospo_gemm_clock_probe_bf16(P(a + 2), P(a), P(a), 512, 512, 512, P(a), st, None) == 2  # align


def test_abi_version_mismatch_is_refused(monkeypatch):
    """A library of another ABI revision is refused at load, not silently mis-driven."""
    from ospo_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "ABI_VERSION", 999)
    with pytest.raises(_lib.OspoError, match="ABI version"):
        _lib.lib()
    monkeypatch.setattr(_lib, "ABI_VERSION", 3)
    monkeypatch.setattr(_lib, "_lib", None)
    _lib.lib()


def test_validation_before_launch(lib):
    """Shape/alignment/argument violations return a status BEFORE any HIP call (no GPU here)."""
    from ospo_amd import _lib
    P = ctypes.c_void_p
    buf = (ctypes.c_char * 4096)()
    a = ctypes.addressof(buf)
    # K % 64 != 0
    rc = lib.ospo_gemm_nt_bf16(P(a), 96, P(a), 96, 64, 64, 96, None, 0, None, 0, 0, ctypes.c_float(1.0),
                               None, None, 0, P(a), 64, 0, None, 0, None)
    assert rc == 1
    # misaligned A
    rc = lib.ospo_gemm_nt_bf16(P(a + 2), 64, P(a), 64, 64, 64, 64, None, 0, None, 0, 0, ctypes.c_float(1.0),
                               None, None, 0, P(a), 64, 0, None, 0, None)
    assert rc == 2
    # null output
    rc = lib.ospo_gemm_nt_bf16(P(a), 64, P(a), 64, 64, 64, 64, None, 0, None, 0, 0, ctypes.c_float(1.0),
                               None, None, 0, None, 64, 0, None, 0, None)
    assert rc == 5
    # split-K workspace: misaligned, or a tail split outside 0..8
    rc = lib.ospo_gemm_nt_bf16(P(a), 64, P(a), 64, 64, 256, 64, None, 0, None, 0, 0, ctypes.c_float(1.0),
                               None, None, 0, P(a), 256, 0, P(a + 4), 4096, None)
    assert rc == 5
    rc = lib.ospo_gemm_nt_bf16(P(a), 64, P(a), 64, 64, 256, 64, None, 0, None, 0, 0, ctypes.c_float(1.0),
                               None, None, 0, P(a), 256, 9, None, 0, None)
    assert rc == 5
    # workspace query: M = 4800 x N = 4096 is 304 tiles, a 48-tile tail round that the cost model splits 4
    # ways on 256 CUs (48 x 4 partial tiles of 256 KiB); a pinned split of 1 needs none
    assert lib.ospo_gemm_nt_ws_bytes(4800, 4096, 4096, 64, 0, 0) == 48 * 4 * 65536 * 4
    assert lib.ospo_gemm_nt_ws_bytes(4800, 4096, 4096, 64, 0, 1) == 0
    assert lib.ospo_gemm_nt_ws_bytes(4096, 4096, 4096, 0, 0, 0) == 0  # exactly one round
    # unknown SimPO loss type -> OSPO_ERR_ARG, like train.py:335-337 raising ValueError
    rc = lib.ospo_simpo_fwd(P(a), 2, ctypes.c_float(10), ctypes.c_float(0.5), ctypes.c_float(0), 7, P(a), P(a),
                            P(a), None)
    assert rc == 5
    with pytest.raises(ValueError):
        _lib.call("ospo_simpo_fwd", P(a), 2, ctypes.c_float(10), ctypes.c_float(0.5), ctypes.c_float(0), 7,
                  P(a), P(a), P(a), None)
    # attention head_dim other than 128 unsupported
    rc = lib.ospo_flash_attn_fwd(P(a), 384, 0, 128, 256, P(a), 128, P(a), 1, 8, 1, 64, ctypes.c_float(0.1), None)
    assert rc == 4
    # logprob rows not a multiple of N
    rc = lib.ospo_logprob_fwd(P(a), 64, P(a), 10, 3, P(a), P(a), P(a), None)
    assert rc == 1
    # nt tile: 256 x 256 8-phase whenever N % 256 == 0 (split-K tail absorbs quantisation), else 64
    assert lib.ospo_gemm_nt_tile(4800, 4096) == 256
    assert lib.ospo_gemm_nt_tile(4608, 16384) == 256
    assert lib.ospo_gemm_nt_tile(100, 192) == 64


def test_lora_layout_7b():
    from ospo_amd.lora import LoraLayout, peft_key
    lay = LoraLayout(30, 4096, 11008, 16)
    assert lay.numel == 37_478_400  # 37.48 M LoRA params at r=16
    sl = lay.slices()
    assert len(sl) == 30 * 7 * 2
    offs = sorted((o, s[0] * s[1]) for _, o, s in sl)
    pos = 0
    for o, n in offs:  # contiguous, non-overlapping
        assert o == pos
        pos += n
    assert pos == lay.numel
    g = lay.groups["qkv"]
    assert g.Rp == 64 and g.a_off == 0
    assert peft_key("layers.3.q_proj.lora_A") == \
        "model.language_model.base_model.model.model.layers.3.self_attn.q_proj.lora_A.default.weight"
    assert peft_key("layers.0.down_proj.lora_B").endswith("layers.0.mlp.down_proj.lora_B.default.weight")
    lay32 = LoraLayout(30, 4096, 11008, 32)
    assert lay32.groups["qkv"].Rp == 128 and lay32.numel == 2 * lay.numel


def test_lora_flat_roundtrip_matches_oracle_names():
    from oracle import simpo_ref as O
    from ospo_amd.lora import LoraLayout
    dims = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, vocab=64, img_vocab=256, gen_head_dim=256)
    w = O.init_lora(dims, seed=4, dtype=torch.bfloat16)
    lay = LoraLayout(2, 256, 512, 16)
    flat = torch.zeros(lay.numel, dtype=torch.bfloat16)
    lay.to_flat(w, flat)
    back = lay.from_flat(flat)
    assert set(back) == set(w)
    for k in w:
        assert torch.equal(back[k], w[k])
    # stacked A of a group == packed Acat rows (dA lands in place)
    g = lay.groups["qkv"]
    blk = flat[g.a_off:g.a_off + 3 * 16 * 256].view(48, 256)
    assert torch.equal(blk, torch.cat([w[f"layers.0.{p}.lora_A"] for p in ("q_proj", "k_proj", "v_proj")]))


def test_build_config_dotlist_and_aliases(tmp_path):
    from ospo_amd.config import build_config, save_config
    cfg = build_config(os.path.join(ROOT, "configs", "step5.yaml"),
                       argv=["experiment.max_training_steps=3", "lora.lora_rank=16", "base.exp_name=x",
                             "optimizer.betas=[0.9,0.99]", "base.resume=null"])
    assert cfg.experiment.max_training_steps == 3 and cfg.lora.lora_rank == 16
    assert cfg.use_lora is True and cfg.use_peft is True  # alias (SURVEY §5 defect i)
    assert cfg.optimizer.betas == [0.9, 0.99] and cfg.base.resume is None
    assert cfg["algo"]["beta"] == 10
    p = save_config(str(tmp_path), cfg)
    assert json.load(open(p))["lora"]["lora_rank"] == 16  # JSON text in config.yaml, like common.py:102-108


def test_preference_dataset_prompt_and_collate():
    from ospo_amd.data import PreferenceDataset, SyntheticTokenizer, sft_prompt
    assert sft_prompt("A black umbrella") == "User: A black umbrella\n\nAssistant:<begin_of_image>"
    ds = PreferenceDataset(seed=42, data_path=os.path.join(ROOT, "tests", "golden", "train_step4.json"),
                           tokenizer=SyntheticTokenizer(), num_samples=4, synthetic_tokens=True)
    assert len(ds) == 4
    items = [ds[i] for i in range(4)]
    ids, text, ch, rj = ds.collate_fn(items)
    assert all(t.dtype == torch.int32 and t.shape[0] == 1 for t in text)
    assert all(c.shape == (1, 576) and int(c.max()) < 16384 for c in ch)
    again = ds[0]
    assert torch.equal(again[2], items[0][2])  # deterministic tokens
    with pytest.raises(ValueError):
        ds.decode({"item_id": "x", "prompt": "p"})


def test_chat_processor_deepseek_template():
    """apply_sft_template_for_multi_turn_prompts (processing_vlm.py:137-177, conversation.py:80-91)."""
    from ospo_amd.data import ChatProcessor, sft_prompt
    cp = ChatProcessor()
    conv = [{"role": "User", "content": "  A red cube  "}, {"role": "Assistant", "content": ""}]
    assert cp.apply_sft_template_for_multi_turn_prompts(conv, "deepseek", "") + cp.image_start_tag == \
        sft_prompt("A red cube")
    assert cp.apply_sft_template_for_multi_turn_prompts(conv, "deepseek", "sys") == "sys\n\nUser: A red cube\n\nAssistant:"


def test_preference_dataset_pixels_reference_format():
    """Default image source = the reference's collate format: PIL -> VLMImageProcessor (384, mean = std
    = 0.5) -> f32 [1, 3, 384, 384]; the example train.json's absolute paths remapped to the fixtures.
    The 384-px example PNG gives exactly the pixels the VQ goldens were made from (make_golden_vq.py)."""
    import numpy as np
    from ospo_amd.data import PreferenceDataset, SyntheticTokenizer, VLMImageProcessor
    golden = os.path.join(ROOT, "tests", "golden")
    ds = PreferenceDataset(seed=42, data_path=os.path.join(golden, "train_pixels.json"), tokenizer=SyntheticTokenizer(),
                           path_map={"/home/elicer/OSPO/example": golden})
    item_id, text, ch, rj = ds[0]
    assert ch.dtype == torch.float32 and ch.shape == (1, 3, 384, 384) and rj.shape == (1, 3, 384, 384)
    assert float(ch.min()) >= -1.0 and float(ch.max()) <= 1.0
    u8 = np.load(os.path.join(golden, "vq_golden.npz"))["img2_u8"]
    px = ds.get_image_tensor("/home/elicer/OSPO/example/step3/negative/layout/1000001/02.png")
    want = ((u8.astype(np.float64) / 255.0).astype(np.float32) - 0.5) / 0.5
    assert np.array_equal(px[0].numpy(), want.transpose(2, 0, 1))
    # non-square input: long side resized to 384 (bicubic), padded with the mean colour
    from PIL import Image
    im = Image.fromarray(u8[:, :192])
    x = VLMImageProcessor()([im])["pixel_values"]
    assert x.shape == (1, 3, 384, 384)
    assert float(x[0, :, :, :96].abs().max()) == pytest.approx(abs(127 / 255 - 0.5) / 0.5)


def test_dataset_batch_equals_reference_dataset_with_our_processors():
    """The reference's own PreferenceDataset + collate_fn fed the processor objects get_model returns
    (tests/golden/make_golden_dataset.py) gives the batch our PreferenceDataset gives: same text ids,
    bit-identical pixel tensors.  So the reference's unchanged dataloader (ospo/step5.py:17-23) feeds
    the wrapper exactly what the GPU pixel-path tests feed it."""
    import hashlib
    import numpy as np
    from ospo_amd.data import PreferenceDataset, SyntheticTokenizer
    golden = os.path.join(ROOT, "tests", "golden")
    z = np.load(os.path.join(golden, "dataset_batch.npz"))
    ds = PreferenceDataset(seed=42, data_path=os.path.join(golden, "train_pixels.json"), tokenizer=SyntheticTokenizer(),
                           path_map={"/home/elicer/OSPO/example": golden})
    ids, text, ch, rj = ds.collate_fn([ds[i] for i in range(len(ds))])
    assert list(ids) == list(z["item_ids"])
    for i, t in enumerate(text):
        assert np.array_equal(t.numpy(), z[f"text{i}"])
    for side, ts in (("chosen", ch), ("rejected", rj)):
        for i, t in enumerate(ts):
            a = t.numpy()
            assert hashlib.sha256(a.tobytes()).hexdigest() == str(z[f"{side}{i}_sha256"]), (side, i)


def test_algorithmic_flops_match_survey():
    sys.path.insert(0, ROOT)
    import bench
    assert abs(bench.algorithmic_flops_per_pair() / 1e12 - 30.37) < 0.01


def test_checkpoint_roundtrip_cpu(tmp_path):
    """Lightning .ckpt layout with peft keys; resume restores adapters and AdamW moments."""
    from ospo_amd.ckpt import load_checkpoint, save_checkpoint, step_ckpt_name
    from ospo_amd.lora import LoraLayout, peft_key
    from ospo_amd.wrapper.train import ConstantLR, FusedLoraAdamW

    class StubEngine:
        def __init__(self):
            self.dims = types.SimpleNamespace(n_layers=2)
            self.layout = LoraLayout(2, 256, 512, 16)
            self.lora = torch.randn(self.layout.numel).to(torch.bfloat16)
            self.exp_avg = torch.randn(self.layout.numel).to(torch.bfloat16)
            self.exp_avg_sq = torch.rand(self.layout.numel).to(torch.bfloat16)
            self.opt_step = 7

        def lora_tensors(self):
            return self.layout.from_flat(self.lora)

        def pack_lora(self):
            pass

    e = StubEngine()
    opt = FusedLoraAdamW(e, 4e-5, (0.9, 0.95), 1e-8, 0.0, 1.0)
    sched = ConstantLR(opt)
    p = save_checkpoint(str(tmp_path / step_ckpt_name(5)), e, opt, sched, epoch=1, global_step=5)
    assert os.path.basename(p) == "step=000005.ckpt"
    ck = torch.load(p, weights_only=True)
    for k in ("state_dict", "optimizer_states", "lr_schedulers", "epoch", "global_step", "pytorch-lightning_version"):
        assert k in ck
    assert peft_key("layers.1.up_proj.lora_B") in ck["state_dict"]
    e2 = StubEngine()
    opt2 = FusedLoraAdamW(e2, 4e-5, (0.9, 0.95), 1e-8, 0.0, 1.0)
    load_checkpoint(p, e2, opt2, ConstantLR(opt2))
    assert torch.equal(e2.lora, e.lora) and torch.equal(e2.exp_avg_sq, e.exp_avg_sq) and e2.opt_step == 7
    assert torch.equal(e2.exp_avg, e.exp_avg)
    sd = ck["optimizer_states"][0]
    assert set(sd) >= {"state", "param_groups"} and len(sd["state"]) == 2 * 7 * 2


def test_optimizer_state_from_torch_adamw_over_the_reference_tree():
    """A torch.optim.AdamW state_dict as the reference's PL run writes it (AdamW(self.parameters()):
    frozen tensors interleaved, state only for the adapters) loads into the fused optimizer."""
    from ospo_amd.lora import LoraLayout, peft_param_order
    from ospo_amd.wrapper.train import FusedLoraAdamW
    layout = LoraLayout(2, 256, 512, 16)
    shapes = {n: s for n, _, s in layout.slices()}
    params = []
    for n in peft_param_order(2):
        if n.endswith("lora_A"):
            params.append(torch.zeros(4, 4, requires_grad=False))  # a frozen base weight before each module
        params.append(torch.randn(*shapes[n], requires_grad=True))
    opt = torch.optim.AdamW(params, lr=4e-5, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.0)
    for _ in range(3):
        for q in params:
            if q.requires_grad:
                q.grad = torch.randn_like(q)
        opt.step()
    sd = opt.state_dict()

    class StubEngine:
        dims = types.SimpleNamespace(n_layers=2)

        def __init__(self):
            self.layout = layout
            self.exp_avg = torch.zeros(layout.numel, dtype=torch.bfloat16)
            self.exp_avg_sq = torch.zeros(layout.numel, dtype=torch.bfloat16)
            self.opt_step = 0
    e = StubEngine()
    f = FusedLoraAdamW(e, 1e-3, (0.9, 0.99), 1e-6, 0.0, 1.0)
    f.load_state_dict(sd)
    assert e.opt_step == 3 and f.param_groups[0]["lr"] == 4e-5
    m = layout.from_flat(e.exp_avg)
    trained = [q for q in params if q.requires_grad]
    for n, q in zip(peft_param_order(2), trained):
        assert torch.equal(m[n], opt.state[q]["exp_avg"].to(torch.bfloat16)), n
    with pytest.raises(ValueError):
        f.load_state_dict({"step": 1, "exp_avg": None})  # not a torch AdamW state_dict


def test_dropout_hash_host_c_and_numpy_agree(lib):
    """ospo_amd/dropout.py restates the device mask hash bit for bit; keep rate ~ 1 - p."""
    import numpy as np
    from ospo_amd import dropout as D
    rng = np.random.default_rng(0)
    idx = rng.integers(0, 2 ** 32, 2000, dtype=np.uint64).astype(np.uint32)
    seeds = rng.integers(0, 2 ** 32, 2000, dtype=np.uint64).astype(np.uint32)
    ref = np.array([lib.ospo_dropout_hash(int(i), int(s)) for i, s in zip(idx, seeds)], dtype=np.uint32)
    assert np.array_equal(ref, np.array([D.drop_hash(i, int(s)) for i, s in zip(idx, seeds)], dtype=np.uint32))
    m = D.keep_mask(512, 4096, D.layer_seed(42, 1, 0, "qkv"), 0.05)
    assert abs(m.mean() - 0.95) < 2e-3
    # one hash per two adjacent elements: the halves of one hash are independent decisions
    pairs = m.reshape(-1, 2)
    assert abs((pairs[:, 0] & pairs[:, 1]).mean() - 0.95 ** 2) < 3e-3
    s0 = D.layer_seed(42, 1, 0, "qkv")
    k = D.keep_bits(np.arange(10, dtype=np.uint32), s0, 0.05)
    h = [int(D.drop_hash(np.uint32(i), s0)) for i in range(5)]
    assert list(k) == [((h[i // 2] >> (16 * (i & 1))) & 0xFFFF) >= D.threshold(0.05) for i in range(10)]
    m2 = D.keep_mask(512, 4096, D.layer_seed(42, 1, 0, "o"), 0.05)
    assert 0.90 < (m == m2).mean() < 0.91  # independent masks agree where both keep or both drop
    assert D.layer_seed(42, 1, 3, "gu") != D.layer_seed(42, 2, 3, "gu")


def _unhash(h, seed):
    """Inverse of dropout.drop_hash: undo each xorshift and each x + lo24(x) * c round (the low 24 bits of the
    result are lo24(x) * (c + 1) mod 2^24, c + 1 odd, so lo24(x) comes back with its inverse mod 2^24, and then
    x = result - lo24(x) * c)."""
    import numpy as np

    def unxorshift(y, s):
        x = y.copy()
        for _ in range(32 // s + 1):
            x = y ^ (x >> np.uint32(s))
        return x

    def unmad(y, c):
        cinv = pow(c + 1, -1, 1 << 24)
        lo = ((y & np.uint32(0xFFFFFF)).astype(np.uint64) * np.uint64(cinv)) & np.uint64(0xFFFFFF)
        return ((y.astype(np.uint64) - lo * np.uint64(c)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)

    x = np.asarray(h, dtype=np.uint32)
    for c, s in ((0xC2B2AE, 16), (0x9E3778, 13), (0xAC4C1A, 15)):
        x = unmad(unxorshift(x, s), c)
    x = unxorshift(x ^ np.uint32(seed), 16)
    return unmad(x, 0xED5AD4)


def test_dropout_hash_is_a_permutation_no_shared_hashes():
    """the round-4 hash multiplied only the low 24 bits, so pairs p and p ^ 0x01000100
    shared a hash for every seed and the down adapter's [4800, 11008] mask (26.4 M pairs) repeated ~36 % of
    itself.  Round 5: every step is a 32-bit bijection, so the hash permutes the pair index for each seed --
    shown by an explicit inverse (random pairs and seeds) -- and no two pairs of the bench's largest mask
    share a hash."""
    import numpy as np
    from ospo_amd import dropout as D
    rng = np.random.default_rng(5)
    for seed in (0, 1, D.layer_seed(42, 1, 29, "down"), int(rng.integers(0, 2 ** 32))):
        x = rng.integers(0, 2 ** 32, 1 << 16, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(_unhash(D.drop_hash(x, seed), seed), x)
        p = np.arange(1 << 20, dtype=np.uint32)
        assert not np.any(D.drop_hash(p, seed) == D.drop_hash(p ^ np.uint32(0x01000100), seed))
    M, K = 4800, 11008  # the bench's down_proj adapter input
    h = D.drop_hash(np.arange(M * K // 2, dtype=np.uint32), D.layer_seed(42, 1, 0, "down"))
    assert np.unique(h).size == h.size
    # the masks of two seeds are not one table re-indexed by an XOR of the seeds (the round-4 relation)
    s1, s2 = D.layer_seed(42, 1, 0, "down"), D.layer_seed(42, 1, 1, "down")
    i = np.arange(1 << 20, dtype=np.uint32)
    assert (D.drop_hash(i, s1) == D.drop_hash(i ^ np.uint32(s1 ^ s2), s2)).mean() < 1e-4


def test_checkpoint_keys_resolve_in_the_reference_module_tree(tmp_path):
    """What ospo/inference.py:268-281 consumes: config.yaml read with yaml.safe_load as get_lora_config
    (ospo/utils/model.py:74-89) reads it, and every adapter key of the .ckpt naming a Linear of the
    transformers Llama tree under peft's prefixes (model. = the LightningModule's self.model,
    language_model.base_model.model. = PeftModel -> LoraModel -> LlamaForCausalLM), with lora_A [r, in]
    and lora_B [out, r] shapes of that Linear."""
    import yaml
    from transformers import LlamaConfig, LlamaForCausalLM
    from ospo_amd.ckpt import save_checkpoint
    from ospo_amd.config import build_config, save_config
    from ospo_amd.lora import LoraLayout
    from ospo_amd.wrapper.train import ConstantLR, FusedLoraAdamW
    L, D, Fd, r = 2, 256, 512, 16
    llama = LlamaForCausalLM(LlamaConfig(vocab_size=512, hidden_size=D, intermediate_size=Fd, num_hidden_layers=L,
                                         num_attention_heads=2, num_key_value_heads=2))
    mods = dict(llama.named_modules())

    class StubEngine:
        dims = types.SimpleNamespace(n_layers=L)

        def __init__(self):
            self.layout = LoraLayout(L, D, Fd, r)
            self.lora = torch.randn(self.layout.numel).to(torch.bfloat16)
            self.exp_avg = torch.zeros(self.layout.numel, dtype=torch.bfloat16)
            self.exp_avg_sq = torch.zeros(self.layout.numel, dtype=torch.bfloat16)
            self.opt_step = 0

        def lora_tensors(self):
            return self.layout.from_flat(self.lora)
    e = StubEngine()
    opt = FusedLoraAdamW(e, 4e-5, (0.9, 0.95), 1e-8, 0.0, 1.0)
    p = save_checkpoint(str(tmp_path / "step=000001.ckpt"), e, opt, ConstantLR(opt), 0, 1)
    cfg = build_config(os.path.join(ROOT, "configs", "step5.yaml"), argv=["lora.lora_rank=16", "lora.lora_alpha=32"])
    save_config(str(tmp_path), cfg)
    ck_cfg = yaml.safe_load(open(tmp_path / "config.yaml"))  # get_lora_config's reads
    lc = ck_cfg["lora"]
    assert lc.get("lora_rank") == r and lc["lora_alpha"] == 32 and lc["lora_dropout"] is not None
    assert sorted(lc["target_modules"]) == sorted(["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj",
                                                   "down_proj"])
    sd = torch.load(p, weights_only=True)["state_dict"]
    assert len(sd) == L * 7 * 2
    pre = "model.language_model.base_model.model."
    for k, t in sd.items():
        assert k.startswith(pre) and k.endswith((".lora_A.default.weight", ".lora_B.default.weight")), k
        name, ab = k[len(pre):].rsplit(".lora_", 1)
        m = mods[name]
        assert isinstance(m, torch.nn.Linear), name
        assert tuple(t.shape) == ((r, m.in_features) if ab.startswith("A") else (m.out_features, r)), k
        assert name.split(".")[-1] in lc["target_modules"]


def test_tile_decode_weight_layout():
    """ops.tile_decode_weight is the layout include/ospo_hip.h states for ospo_decode_gemv ldw = 0:
    element 8 (16 g + l16) + e of tile (nb, ks) = w[16 nb + l16, 32 ks + 8 g + e]."""
    import torch
    from ospo_amd import ops
    N, K = 48, 96
    w = torch.arange(N * K, dtype=torch.float32).reshape(N, K).bfloat16()  # exact up to 256: compare indices below
    idx = torch.arange(N * K, dtype=torch.int64).reshape(N, K)
    t = ops.tile_decode_weight(w)
    assert t.shape == (N // 16, K // 32, 512) and t.is_contiguous()
    ti = idx.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(N // 16, K // 32, 512)
    for nb in range(N // 16):
        for ks in range(K // 32):
            for g in range(4):
                for l16 in range(16):
                    for e in (0, 7):
                        assert int(ti[nb, ks, 8 * (16 * g + l16) + e]) == (16 * nb + l16) * K + 32 * ks + 8 * g + e
    assert torch.equal(t, w.flatten()[ti.flatten()].reshape(t.shape))


def test_image_processor_equals_reference_processor_bytes():
    """ospo_amd.data.VLMImageProcessor against the reference's own
    janus/models/image_processing_vlm.py VLMImageProcessor (resize :127-162, preprocess :164-192,
    Janus-Pro mean = std = 0.5), run by tests/golden/make_golden_image.py: the f32 pixel tensors
    are byte-identical on the example PNGs (identity resize) and on a landscape 500x320 image
    (bicubic downsample + top/bottom padding), a 512x512 image (downsample) and a portrait 200x300
    image (upsample + left/right padding)."""
    import hashlib
    import numpy as np
    from PIL import Image
    from ospo_amd.data import VLMImageProcessor
    from tests import fixtures as FX
    z = FX.load("image_golden.npz")
    proc = VLMImageProcessor()
    names = [str(n) for n in z["names"]]
    assert len(names) == 8 and sum(not n.endswith(".png") for n in names) == 3
    for i, name in enumerate(names):
        if name.endswith(".png"):
            with Image.open(os.path.join(FX.GOLDEN, name)) as im:
                img = im.convert("RGB")
        else:
            img = Image.fromarray(z[f"in{i}"])
        x = proc([img])["pixel_values"].numpy()
        assert x.dtype == np.float32 and x.shape == (1, 3, 384, 384), name
        np.testing.assert_array_equal(x.reshape(-1)[::331], z[f"px{i}_sample"], err_msg=name)
        assert hashlib.sha256(x.tobytes()).hexdigest() == str(z[f"px{i}_sha256"]), name


def _golden_sched():
    with open(os.path.join(ROOT, "tests", "golden", "sched_golden.json")) as f:
        return json.load(f)


class _Opt:
    """The optimizer surface the schedules touch (param_groups)."""

    def __init__(self, lr, lr_scale=None):
        g = {"lr": float(lr)}
        if lr_scale is not None:
            g["lr_scale"] = lr_scale
        self.param_groups = [g]


@pytest.mark.parametrize("case", range(4))
def test_cosine_schedule_equals_reference_golden(case):
    """CosineDecayWarmUpRestarts (ospo_amd/wrapper/train.py) against the reference's own class
    (ospo/utils/train.py:119-148, run by tests/golden/make_golden_sched.py): the lr of every optimizer step,
    including the construction step torch's _LRScheduler takes (the first step runs at iteration 1)."""
    from ospo_amd.wrapper.train import CosineDecayWarmUpRestarts
    c = _golden_sched()["cosine"][case]
    opt = _Opt(c["init_lr"], c["lr_scale"])
    s = CosineDecayWarmUpRestarts(opt, warmup_iter=c["max_training_steps"] * c["warmup_ratio"],
                                  max_iter=c["max_training_steps"], eta_min=c["min_lr"], eta_max=c["init_lr"])
    got = [opt.param_groups[0]["lr"]]
    for _ in range(len(c["lrs"]) - 1):
        s.step()
        got.append(opt.param_groups[0]["lr"])
    assert got == pytest.approx(c["lrs"], rel=1e-12, abs=1e-18)
    # a resumed schedule continues where the checkpoint left it
    s2 = CosineDecayWarmUpRestarts(_Opt(c["init_lr"], c["lr_scale"]), warmup_iter=c["max_training_steps"] * c["warmup_ratio"],
                                   max_iter=c["max_training_steps"], eta_min=c["min_lr"], eta_max=c["init_lr"])
    s2.load_state_dict(s.state_dict())
    assert s2.optimizer.param_groups[0]["lr"] == pytest.approx(got[-1], rel=1e-12, abs=1e-18)


def test_constant_schedule_equals_reference_golden():
    from ospo_amd.wrapper.train import ConstantLR
    c = _golden_sched()["constant"][0]
    opt = _Opt(c["init_lr"])
    s = ConstantLR(opt, factor=1.0, total_iters=c["total_iters"])
    got = [opt.param_groups[0]["lr"]]
    for _ in range(len(c["lrs"]) - 1):
        s.step()
        got.append(opt.param_groups[0]["lr"])
    assert got == pytest.approx(c["lrs"], rel=1e-12)


def test_configure_optimizers_builds_reference_schedules():
    """configure_optimizers (ospo/wrapper/train.py:107-130): 'cosine' -> warm-up max_steps * warmup_ratio,
    eta_min = optimizer.min_lr, eta_max = optimizer.init_lr, interval 'step'; 'constant' -> ConstantLR."""
    from ospo_amd.wrapper.train import ConstantLR, CosineDecayWarmUpRestarts, JanusProTrainWrapper
    import inspect
    src = inspect.getsource(JanusProTrainWrapper.configure_optimizers)
    assert "warmup_ratio" in src and "min_lr" in src and "init_lr" in src and '"interval": "step"' in src
    assert issubclass(ConstantLR, object) and issubclass(CosineDecayWarmUpRestarts, object)


class _AccumWrapper:
    """A wrapper with the SimPO wrapper's trainer-facing surface over one CPU parameter, so the fit loop's
    gradient accumulation can be checked against PL 1.9's (loss / accumulate_grad_batches, one optimizer step,
    clip and scheduler step per accumulate_grad_batches micro-batches; ospo/utils/train.py:32)."""

    def __init__(self):
        self.w = torch.zeros(3, requires_grad=True)
        self.engine = types.SimpleNamespace(grads=torch.zeros(3))
        self.steps = []  # (the .grad seen by each optimizer step)
        self.global_step = 0
        outer = self

        class Opt:
            param_groups = [{"lr": 1.0}]

            def step(self_):
                outer.steps.append(outer.w.grad.clone())
                with torch.no_grad():
                    outer.w -= outer.w.grad

            def zero_grad(self_):
                outer.w.grad = None
        self.opt = Opt()

    def setup(self, stage, log_dir=None):
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)  # (the real wrapper writes its config there)

    def configure_optimizers(self):
        sched = types.SimpleNamespace(n=0)
        sched.step = lambda: setattr(sched, "n", sched.n + 1)
        self.sched = sched
        return [self.opt], [{"scheduler": sched, "interval": "step"}]

    def training_step(self, batch, idx):
        return (self.w * batch).sum() ** 2 / 2

    def on_before_optimizer_step(self):
        pass

    @property
    def logged(self):
        return {}


@pytest.mark.parametrize("accum", [1, 2, 3])
def test_trainer_gradient_accumulation_matches_pl(accum, tmp_path):
    from ospo_amd.trainer import Trainer
    cfg = {"base": {"save_path": str(tmp_path), "exp_name": "acc"},
           "experiment": {"max_training_steps": 2, "gradient_accumulation_steps": accum, "log_steps": 1,
                          "enable_checkpointing": False}}
    batches = [torch.tensor([1.0, 2.0, 3.0]) * (i + 1) for i in range(2 * accum)]
    wr = _AccumWrapper()
    Trainer(cfg).fit(wr, batches)
    assert len(wr.steps) == 2 and wr.sched.n == 2
    # PL: each micro-batch's loss / accum, grads summed over the window, one step per window
    w = torch.zeros(3, requires_grad=True)
    for s in range(2):
        g = torch.zeros(3)
        for b in batches[s * accum:(s + 1) * accum]:
            w_ = w.detach().clone().requires_grad_(True)
            ((w_ * b).sum() ** 2 / 2 / accum).backward()
            g += w_.grad
        assert torch.allclose(wr.steps[s], g, rtol=1e-6), (s, wr.steps[s], g)
        w = (w.detach() - g).requires_grad_(True)


def test_w4_k_loop_include_regenerates_byte_identical(tmp_path):
    """The committed hand-placed K loop (ospo_amd/csrc/gemm_w4_asm.inc) is what gen_gemm_w4.py generates; the
    Makefile regenerates it only on `make regen-w4` (never by mtime order after a checkout)."""
    import subprocess
    import sys
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ospo_amd", "csrc")
    out = tmp_path / "w4.inc"
    subprocess.run([sys.executable, os.path.join(csrc, "gen_gemm_w4.py"), str(out)], check=True, cwd=csrc)
    assert out.read_bytes() == open(os.path.join(csrc, "gemm_w4_asm.inc"), "rb").read()
