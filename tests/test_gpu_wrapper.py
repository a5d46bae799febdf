"""The reference-shaped plugin on the MI355X: JanusProTrainWrapper.training_step ->
loss.backward() -> fused clip+AdamW, the step5 Trainer loop with Lightning-layout
checkpoints and resume, and the standalone get_batch_logps against the
reference-generated known-answer vectors."""
import os

import pytest
import torch

from tests import fixtures as FX

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TINY = ["model.synthetic=true", "dataset.train.synthetic_tokens=true",
        f"dataset.train.data_path={ROOT}/tests/golden/train_step4.json", "model.arch=janus-pro-1b",
        "model.override={'n_layers': 2, 'd_model': 256, 'd_ff': 512, 'n_heads': 2, 'vocab': 512, "
        "'img_vocab': 2048, 'gen_head_dim': 256}",
        "lora.lora_rank=16", "lora.lora_alpha=32", "dataset.train.batch_size=2", "experiment.max_training_steps=4",
        "experiment.save_steps=2", "lora.lora_dropout=0.0"]  # (these tests compare forwards; step5.yaml trains at 0.05)


# images as the reference feeds them: the 2 example pairs' PNGs (tests/golden/step3) -> f32 pixels;
# the VQ codebook is 16384 x 8, so img_vocab stays 16384 and every image is 576 tokens
PIXELS = ["model.synthetic=true", f"dataset.train.data_path={ROOT}/tests/golden/train_pixels.json",
          "dataset.train.path_map={'/home/elicer/OSPO/example': '" + ROOT + "/tests/golden'}",
          "model.arch=janus-pro-1b",
          "model.override={'n_layers': 2, 'd_model': 256, 'd_ff': 512, 'n_heads': 2, 'vocab': 512, "
          "'gen_head_dim': 256}",
          "lora.lora_rank=16", "lora.lora_alpha=32", "dataset.train.batch_size=2", "lora.lora_dropout=0.0"]


def make(tmp_path, extra=(), base=TINY):
    from ospo_amd.config import build_config
    from ospo_amd.data import train_dataloader
    from ospo_amd.model import get_model
    from ospo_amd.wrapper.train import JanusProTrainWrapper
    cfg = build_config(os.path.join(ROOT, "configs", "step5.yaml"),
                       argv=list(base) + [f"base.save_path={tmp_path}"] + list(extra))
    model, cp, ip, tok = get_model(mode="train", config=cfg, seed=0)
    dl = train_dataloader(cfg, tok, img_vocab=model.engine.dims.img_vocab, chat_processor=cp, image_processor=ip)
    w = JanusProTrainWrapper(cfg, model, cp, ip, tok)
    return cfg, model, dl, w


def test_wrapper_backward_equals_engine_step(tmp_path):
    from ospo_amd.simpo import SimPOConfig, SimPOLossBuffers, train_step
    cfg, model, dl, w = make(tmp_path)
    batch = next(iter(dl))
    eng = w.engine
    eng.zero_grad()
    loss = w.training_step(batch, 0)
    loss.backward()
    g_wrapper = eng.grads.clone()
    pre = w.preprocess_batch(batch)
    out = train_step(eng, pre["text_ids"], pre["chosen_ids"], pre["rejected_ids"], SimPOConfig(),
                     SimPOLossBuffers(2, eng.device), optimizer=False)
    torch.cuda.synchronize()
    assert abs(float(loss) - float(out["loss"])) < 1e-6
    assert float((g_wrapper - eng.grads).norm() / eng.grads.norm()) < 1e-5
    for k in ("train/loss", "train/rewards/chosen", "train/rewards/margins", "train/logps/chosen",
              "train/logits/chosen"):
        assert k in w.logged and w.logged[k] == w.logged[k]  # present and not NaN
    assert w.compute_total_grad_norm() > 0


def test_trainer_fit_checkpoint_and_resume(tmp_path):
    from ospo_amd.trainer import Trainer
    cfg, model, dl, w = make(tmp_path)
    tr = Trainer(cfg).fit(w, dl)
    assert tr.global_step == 4
    ck2 = os.path.join(tr.log_dir, "step=000002.ckpt")
    assert os.path.exists(ck2) and os.path.exists(os.path.join(tr.log_dir, "step=000004.ckpt"))
    assert os.path.exists(os.path.join(tr.log_dir, "config.yaml"))
    lines = open(os.path.join(tr.log_dir, "metrics.jsonl")).read().strip().splitlines()
    assert len(lines) == 4
    sd = torch.load(ck2, weights_only=True)
    assert sd["global_step"] == 2 and len(sd["state_dict"]) == 2 * 7 * 2
    # resume from step 2 in a fresh process-equivalent: adapters/optimizer restored, loop continues to 4
    cfg2, model2, dl2, w2 = make(tmp_path, extra=[f"base.resume={ck2}"])
    tr2 = Trainer(cfg2)
    tr2.fit(w2, dl2, ckpt_path=ck2)
    assert tr2.global_step == 4
    assert w2.engine.opt_step == 4  # AdamW step count restored (2) and advanced (+2)


def test_get_batch_logps_matches_reference_kat(tmp_path):
    cfg, model, dl, w = make(tmp_path)
    z = FX.load("logps_kat.npz")
    logits = FX.bits_to_bf16(z["logits_bf16"]).cuda()
    labels = torch.from_numpy(z["labels"]).cuda()
    avg = w.get_batch_logps(logits, labels, average_log_prob=True).cpu()
    tot = w.get_batch_logps(logits, labels, average_log_prob=False).cpu()
    torch.testing.assert_close(avg, torch.from_numpy(z["logps_avg"]), rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(tot, torch.from_numpy(z["logps_sum"]), rtol=2e-5, atol=2e-4)
    with pytest.raises(ValueError):
        w.get_batch_logps(logits[:, :-1], labels)


def _vq_golden_weights(model):
    """Give the policy's VQ encoder the seeded weights the VQ goldens were made with (make_golden_vq.py)."""
    from oracle import vq_ref as V
    z = FX.load("vq_golden.npz")
    model._vq, model._vq_weights = None, V.init_vq_weights(int(z["seed"]))


def test_pixel_batches_vq_encoded_in_preprocess_match_token_cache(tmp_path):
    """The reference's collate format (f32 pixels, train_dataset.py:79-84) goes through the GPU VQ encode
    inside preprocess_batch (train.py:246-261): ids equal a token cache built by the same encoder, and
    the step's logps / loss / grads are identical to the cache path's."""
    import numpy as np
    from ospo_amd.vq import build_token_cache
    cfg, model, dl, w = make(tmp_path, base=PIXELS)
    _vq_golden_weights(model)
    batch = next(iter(torch.utils.data.DataLoader(dl.dataset, batch_size=2, shuffle=False,
                                                  collate_fn=dl.dataset.collate_fn)))
    assert batch[2][0].dtype == torch.float32 and batch[2][0].shape == (1, 3, 384, 384)
    pre = w.preprocess_batch(batch)
    assert pre["chosen_ids"].shape == (2, 576) and pre["chosen_ids"].is_cuda
    # the same PNGs through the token-cache CLI path
    golden = os.path.join(ROOT, "tests", "golden")
    items = []
    for ex in dl.dataset.dataset:
        for side in ("chosen", "rejected"):
            items.append((f"{ex['item_id']}/{side}", dl.dataset.remap(ex[side])))
    cache = build_token_cache(model.gen_vision_model, items, str(tmp_path / "cache.npz"))
    for i, ex in enumerate(dl.dataset.dataset):
        assert np.array_equal(pre["chosen_ids"][i].cpu().numpy(), cache[f"{ex['item_id']}/chosen"])
        assert np.array_equal(pre["rejected_ids"][i].cpu().numpy(), cache[f"{ex['item_id']}/rejected"])
    eng = w.engine
    eng.zero_grad()
    loss = w.training_step(batch, 0)
    loss.backward()
    g_pix = eng.grads.clone()
    id_batch = (batch[0], batch[1], [torch.from_numpy(cache[f"{i}/chosen"]).view(1, -1) for i in batch[0]],
                [torch.from_numpy(cache[f"{i}/rejected"]).view(1, -1) for i in batch[0]])
    eng.zero_grad()
    loss2 = w.training_step(id_batch, 0)
    loss2.backward()
    torch.cuda.synchronize()
    assert float(loss) == float(loss2)
    # same ids -> same step; the LoRA weight gradients sum K-split partials with fp32 atomics, so
    # only their summation order may differ between the two runs
    assert float((g_pix - eng.grads).norm() / eng.grads.norm()) < 1e-5
    # the 384-px example PNG the VQ goldens hold: ids identical to the reference vq_model.py's
    z = FX.load("vq_golden.npz")
    px = dl.dataset.get_image_tensor("/home/elicer/OSPO/example/step3/negative/layout/1000001/02.png")
    ids = model.vq_encode(px)
    assert np.array_equal(ids[0].cpu().numpy(), z["img2_ids"])


def test_wrapper_sft_weight_and_logits_metrics_vs_oracle(tmp_path):
    """algo.sft_weight > 0 (train.py:421-430) and the reference's logits/* logging (mean over all
    [B, T, V] logits, [B, T-1, V] for chosen with sft) through the wrapper, against the oracle."""
    from oracle import simpo_ref as O
    cfg, model, dl, w = make(tmp_path, extra=["algo.sft_weight=0.5", "lora.lora_dropout=0.0"])
    batch = next(iter(dl))
    eng = w.engine
    eng.zero_grad()
    loss = w.training_step(batch, 0)
    loss.backward()
    torch.cuda.synchronize()
    pre = w.preprocess_batch(batch)
    d = eng.dims
    dims = O.JanusDims(n_layers=d.n_layers, d_model=d.d_model, d_ff=d.d_ff, n_heads=d.n_heads, head_dim=d.head_dim,
                       vocab=d.vocab, img_vocab=d.img_vocab, img_embed=d.img_embed, gen_head_dim=d.gen_head_dim,
                       lora_r=d.lora_r, lora_alpha=d.lora_alpha)
    from ospo_amd.engine import synthetic_weights
    wts = {k: v.cpu() for k, v in synthetic_weights(d, "cuda", seed=0, lora_seed=1).items()}  # get_model's seeds
    text = [t.to(torch.int32) for t in batch[1]]
    ref = O.simpo_step(text, pre["chosen_ids"].cpu().long(), pre["rejected_ids"].cpu().long(), wts, dims,
                       dtype=torch.float32, sft_weight=0.5)
    lg = w.logged
    assert abs(float(loss) - float(ref.loss)) / abs(float(ref.loss)) < 1e-3
    assert lg["train/sft_loss"] == pytest.approx(ref.metrics["sft_loss"], rel=1e-3)
    for k in ("logits/chosen", "logits/rejected"):
        assert lg["train/" + k] == pytest.approx(ref.metrics[k], rel=2e-2, abs=2e-4), k
    g = eng.grad_tensors()
    errs = [FX.rel_err(g[k].cpu(), v) for k, v in ref.lora_grads.items()]
    assert max(errs) < 5e-2


def test_concatenated_forward_returns_full_logits(tmp_path):
    """train.py:345-372: concatenated_forward returns gen_head's logits over EVERY position, [B, T, V]
    per side, as the reference does (get_batch_loss_metrics itself skips them).  Against the oracle's
    gen_head over the final hidden state (fp32), and get_batch_logps of those logits reproduces the
    engine's log-probs (1e-3, north star)."""
    from oracle import simpo_ref as O
    from ospo_amd.engine import synthetic_weights
    cfg, model, dl, w = make(tmp_path, extra=["lora.lora_dropout=0.0"])  # two forwards below: same masks
    batch = next(iter(dl))
    pre = w.preprocess_batch(batch)
    c, r, cl, rl, lab = w.concatenated_forward(pre)
    e = w.engine
    B, T, V = e.B, e.T, e.dims.img_vocab
    assert cl.shape == (B, T, V) and rl.shape == (B, T, V) and cl.dtype == torch.bfloat16
    assert lab.shape == (B, T)
    c2, r2, ncl, nrl, _ = w.concatenated_forward(pre, return_logits=False)
    assert ncl is None and nrl is None and torch.equal(c, c2) and torch.equal(r, r2)
    lp = w.get_batch_logps(torch.cat([cl, rl]), torch.cat([lab, pre["rejected_labels"]]))
    assert FX.rel_err(lp.cpu(), torch.cat([c, r]).detach().cpu()) < 1e-3
    d = e.dims
    dims = O.JanusDims(n_layers=d.n_layers, d_model=d.d_model, d_ff=d.d_ff, n_heads=d.n_heads, head_dim=d.head_dim,
                       vocab=d.vocab, img_vocab=d.img_vocab, img_embed=d.img_embed, gen_head_dim=d.gen_head_dim,
                       lora_r=d.lora_r, lora_alpha=d.lora_alpha)
    wts = {k: v.cpu().float() for k, v in synthetic_weights(d, "cuda", seed=0, lora_seed=1).items()}
    text = [t.to(torch.int32) for t in batch[1]]
    bt = O.preprocess_batch(text, pre["chosen_ids"].cpu().long(), pre["rejected_ids"].cpu().long(), wts,
                            torch.float32)
    cb = O.concatenated_inputs(bt)
    with torch.no_grad():
        ref = O.gen_head(O.llama_hidden(cb["concatenated_inputs_embeds"], wts, dims, training=False), wts)
    got = torch.cat([cl, rl]).float().cpu()
    assert FX.rel_err(got, ref) < 2e-2  # bf16 logits of a bf16 path vs fp32


def test_wrapper_shipped_config_16_pairs_r32_dropout_7b_widths_vs_oracle(tmp_path):
    """The reference's shipped training configuration (configs/step5.yaml: dataset.train.batch_size 16 pairs
    per process, LoRA r = 32 / alpha 64, lora_dropout 0.05; /root/reference/configs/step5.yaml:15,23) through
    the drop-in path -- JanusProTrainWrapper.training_step + loss.backward -- at Janus-Pro-7B widths with 2
    decoder layers: M = 32 x 600 = 19 200 rows (memory fit and the int32 offset guards at twice config 3's
    per-GPU batch).  Against the oracle with the HIP dropout masks replayed: log-probs 1e-3 relative (north
    star) vs the bf16 and the fp32 oracle, loss 1e-3 of the fp32 oracle, LoRA grads vs the fp32 oracle within
    the 7B-shape tolerance."""
    from oracle import simpo_ref as O
    from ospo_amd.engine import synthetic_weights
    from tests.test_gpu_step import _LazyMasks
    cfg, model, dl, w = make(tmp_path, extra=[
        "model.arch=janus-pro-7b", "model.override={'n_layers': 2}", "lora.lora_rank=32", "lora.lora_alpha=64",
        "lora.lora_dropout=0.05", "dataset.train.batch_size=16"])
    batch = next(iter(dl))
    eng = w.engine
    d = eng.dims
    assert (d.d_model, d.d_ff, d.n_layers, d.lora_r) == (4096, 11008, 2, 32)
    eng.zero_grad()
    loss = w.training_step(batch, 0)
    loss.backward()
    torch.cuda.synchronize()
    pre = w.preprocess_batch(batch)
    B = pre["chosen_ids"].shape[0]
    assert B == 16 and eng.M == 32 * eng.T and eng.M >= 19_000
    grads = {k: v.float().cpu() for k, v in eng.grad_tensors().items()}
    loss = float(loss)
    call, p, M, base = eng._drop_call, eng.lora_dropout, eng.M, eng._drop_base
    wts = {k: v.cpu() for k, v in synthetic_weights(d, "cuda", seed=0, lora_seed=1).items()}  # get_model's seeds
    # the engine's own log-probs of the same forward (training_step keeps no copy): re-run the forward with the
    # same dropout call so the masks are the ones replayed below
    eng._drop_call = call - 1
    lp = eng.forward(pre["text_ids"], pre["chosen_ids"], pre["rejected_ids"]).float().cpu()
    assert eng._drop_call == call
    del model, w, eng
    torch.cuda.empty_cache()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    dims = O.JanusDims(n_layers=d.n_layers, d_model=d.d_model, d_ff=d.d_ff, n_heads=d.n_heads, head_dim=d.head_dim,
                       vocab=d.vocab, img_vocab=d.img_vocab, img_embed=d.img_embed, gen_head_dim=d.gen_head_dim,
                       lora_r=d.lora_r, lora_alpha=d.lora_alpha, lora_dropout=p)
    masks = _LazyMasks(M, {"qkv": d.d_model, "o": d.d_model, "gu": d.d_model, "down": d.d_ff}, base, call, p)
    text = [t.to(torch.int32) for t in batch[1]]
    ch, rj = pre["chosen_ids"].cpu().long(), pre["rejected_ids"].cpu().long()
    o16 = O.simpo_step(text, ch, rj, wts, dims, dtype=torch.bfloat16, backward=False, dropout_masks=masks)
    o32 = O.simpo_step(text, ch, rj, wts, dims, dtype=torch.float32, dropout_masks=masks)
    rel = FX.rel_err
    e16 = max(rel(lp[:B], o16.chosen_logps), rel(lp[B:], o16.rejected_logps))
    e32 = max(rel(lp[:B], o32.chosen_logps), rel(lp[B:], o32.rejected_logps))
    l32 = float(o32.loss)
    el32, floor_l = abs(loss - l32) / l32, abs(float(o16.loss) - l32) / l32
    g32 = max(rel(grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    from tests.conftest import record_parity
    record_parity("wrapper_shipped_config_16_pairs_r32_7b_2l", logp=e16, logp_vs_fp32=e32, loss=loss,
                  loss_bf16_oracle=float(o16.loss), loss_fp32_oracle=l32, loss_vs_fp32=el32,
                  oracle_bf16_vs_fp32_loss=floor_l, grad_vs_fp32=g32, rows=M)
    print(f"\nshipped config (16 pairs, r=32, dropout 0.05, 7B widths, 2 layers, M={M}): logp {e16:.2e} "
          f"(fp32 {e32:.2e}), loss {loss:.6f} vs fp32 {l32:.6f} ({el32:.2e}), grads vs fp32 {g32:.2e}")
    assert e16 < 1e-3 and e32 < 1e-3
    assert el32 < max(1e-3, floor_l), (el32, floor_l)
    assert g32 < 6.5e-2, g32
