"""Whole-step parity on the MI355X: the HIP engine (through the C ABI) against the
CPU oracle on the same seeded inputs, and against the reference-generated golden
vectors.  Tolerances (north star): per-sequence log-probs within 1e-3 relative of
the oracle's bf16 path.  SimPO loss: beta = 10 amplifies log-prob noise ~10x and
two bf16 implementations differ by their rounding noise (HIP-vs-fp32 and
oracle_bf16-vs-fp32 log-prob errors are equal, tests/diag_7b_precision.py), so
the loss is held to 1e-3 relative of the fp32 oracle (the value both bf16 paths
approximate) and of the bf16 oracle up to 2 layers; through all 30 layers the bf16 noise
of the log-probs alone moves a loss near 5 by 2e-3 .. 1e-2, so there the gate is the
log-probs: 1e-3 of both oracles and no further from fp32 than 1.25x the bf16 oracle's own
distance (pooled over 3 seeds of the bench workload; LOGP_NOISE_RATIO).  The
loss kernel is held to 1e-5 given the log-probs.  LoRA gradients (bf16 autograd in the oracle vs the fp32-accumulated
HIP backward) within 5e-2 relative L2.  VQ/label indexing is integer and exact
by construction (ids are gathered, never cast)."""
import json

import numpy as np
import pytest
import torch

from oracle import simpo_ref as O
from tests import fixtures as FX
from tests.conftest import record_parity

pytestmark = pytest.mark.gpu


# LoRA-grad relative L2 error vs the fp32 oracle: ~2x what was measured on MI355X (the tests log the
# measured values to $OSPO_PARITY_LOG; profiles/r02/parity_*.jsonl): tiny 1.10e-2, 1B 2-layer 1.92e-2,
# 7B-shape 2-layer 3.14e-2, r = 32 1.01e-2, r = 8 1.13e-2.  Each test also holds the HIP error to 1.25x
# the oracle's own bf16-autograd error against fp32 (GRAD_FLOOR_RATIO; measured ratios 0.87-0.97): the
# fp32-accumulated HIP backward is at least as close to the fp32 gradients as a bf16 autograd is.
# At 30 layers there is no fixed cap: the bound is 1.25x the oracle's own spread (0.12 / 0.14 / 0.16 for layers
# 0 / 15 / 29; measured HIP 0.11 / 0.12 / 0.14, profiles/r03/parity_suite_v4_final.jsonl).
GRAD_FP32_TOL = {"step_tiny_bf16.npz": 2.5e-2, "step_1b2l_bf16.npz": 4e-2, "tiny_fp32_ref": 2.5e-2, "7b_2l": 6.5e-2,
                 "r32": 2.5e-2, "r8": 2.5e-2}
GRAD_FLOOR_RATIO = 1.25
# Fixed before the round-6 suite run: at depth the HIP per-sequence log-probs must be no
# further from the fp32 oracle than 1.25x the bf16 oracle's own distance from it.
LOGP_NOISE_RATIO = 1.25


def pad_text(text):
    Lt = max(t.shape[1] for t in text)
    out = torch.full((len(text), Lt), -1, dtype=torch.int32)
    for i, t in enumerate(text):
        out[i, : t.shape[1]] = t[0]
    return out


def build_engine(dims, w, B, Lt, N):
    from ospo_amd.engine import ModelDims, SimPOEngine
    return SimPOEngine(ModelDims.from_any(dims), w, device="cuda", max_pairs=B, max_text_len=Lt, n_img_tokens=N)


def run_hip_step(eng, text, chosen, rejected, algo):
    from ospo_amd.simpo import SimPOConfig, SimPOLossBuffers, simpo_backward, simpo_forward
    cfg = SimPOConfig(beta=algo["beta"], gamma_beta_ratio=algo["gamma_beta_ratio"],
                      label_smoothing=algo["label_smoothing"], loss_type=algo["loss_type"])
    B = chosen.shape[0]
    buf = SimPOLossBuffers(B, "cuda")
    logps = eng.forward(pad_text(text).cuda(), chosen.int().cuda(), rejected.int().cuda())
    losses, mean, _ = simpo_forward(logps, B, cfg, buf)
    g = simpo_backward(logps, B, cfg, buf)
    eng.zero_grad()
    eng.backward(g)
    torch.cuda.synchronize()
    grads = {k: v.float().cpu() for k, v in eng.grad_tensors().items()}
    return logps.cpu().clone(), float(mean.item()), grads


def rel(a, b):
    return FX.rel_err(a.float(), b.float())


@pytest.mark.parametrize("name", ["step_tiny_bf16.npz", "step_1b2l_bf16.npz"])
def test_step_matches_oracle_and_golden(name):
    z = FX.load(name)
    dims = FX.dims_of(z)
    algo = json.loads(str(z["algo"]))
    text, chosen, rejected = FX.step_inputs(z)
    w = FX.step_weights(z, name, dims)
    B, N = chosen.shape
    Lt = max(t.shape[1] for t in text)
    eng = build_engine(dims, w, B, Lt, N)
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    ora = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16, beta=algo["beta"],
                       gamma_beta_ratio=algo["gamma_beta_ratio"], label_smoothing=algo["label_smoothing"],
                       loss_type=algo["loss_type"])
    o32 = O.simpo_step(text, chosen, rejected, {k: v.float() for k, v in w.items()}, dims, dtype=torch.float32)
    ref = FX.step_outputs(z)
    e_c = rel(logps[:B], ora.chosen_logps)
    e_r = rel(logps[B:], ora.rejected_logps)
    e_l = abs(loss - float(ora.loss)) / abs(float(ora.loss))
    e_l32 = abs(loss - float(o32.loss)) / abs(float(o32.loss))
    ge = {k: rel(grads[k], ora.lora_grads[k]) for k in ora.lora_grads}
    print(f"\n{name}: logp rel err chosen {e_c:.2e} rejected {e_r:.2e}; loss {loss:.6f} vs {float(ora.loss):.6f} "
          f"({e_l:.2e}), fp32 oracle {float(o32.loss):.6f} ({e_l32:.2e}); "
          f"golden-ref logp err {rel(logps[:B], ref['chosen_logps']):.2e}; "
          f"max grad rel err {max(ge.values()):.2e}")
    assert e_c < 1e-3 and e_r < 1e-3
    assert e_l32 < 1e-3 and e_l < 1e-3
    assert abs(float(O.simpo_loss(logps[:B], logps[B:])[0].mean()) - loss) < 1e-5
    # against the reference's own (bf16-log_softmax) run: bounded by the reference's bf16 reduction error
    assert rel(logps[:B], ref["chosen_logps"]) < 4e-3
    g32 = max(rel(grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    floor = max(rel(ora.lora_grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    record_parity(f"step_{name}", logp=max(e_c, e_r), loss_bf16=e_l, loss_fp32=e_l32, grad_vs_bf16=max(ge.values()),
                  grad_vs_fp32=g32, oracle_bf16_vs_fp32_grad=floor)
    assert max(ge.values()) < 5e-2, sorted(ge.items(), key=lambda kv: -kv[1])[:3]
    assert g32 < GRAD_FP32_TOL[name], (g32, floor)
    assert g32 < GRAD_FLOOR_RATIO * floor, (g32, floor)


def test_step_tiny_matches_fp32_reference():
    """Same inputs, the reference run entirely in fp32: the bf16 HIP path sits within bf16 noise."""
    z = FX.load("step_tiny_fp32.npz")
    dims = FX.dims_of(z)
    algo = json.loads(str(z["algo"]))
    text, chosen, rejected = FX.step_inputs(z)
    w = FX.step_weights(z, "step_tiny_fp32.npz", dims)
    B, N = chosen.shape
    eng = build_engine(dims, w, B, max(t.shape[1] for t in text), N)
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    ref = FX.step_outputs(z)
    assert rel(logps[:B], ref["chosen_logps"]) < 1e-3
    assert rel(logps[B:], ref["rejected_logps"]) < 1e-3
    assert abs(loss - float(ref["loss"])) / float(ref["loss"]) < 1e-3
    g32 = max(rel(grads[k], g) for k, g in ref["grads"].items())  # the reference's own fp32 run
    record_parity("step_tiny_vs_fp32_reference", grad_vs_fp32=g32)
    assert g32 < GRAD_FP32_TOL["tiny_fp32_ref"]


def test_step_full_size_7b_shapes_two_layers():
    """BASELINE shapes (Janus-Pro-7B: D 4096, F 11008, 32 heads, 576 image tokens,
    T = 600) with 2 of the 30 layers and two ragged pairs.

    Logps: 1e-3 relative vs the bf16 oracle (north star; measured 7e-5).  The
    SimPO loss kernel is exact given the logps (1e-5).  End to end, beta = 10
    amplifies the logp rounding noise of two different bf16 paths ~10x
    (measured: HIP-vs-fp32 and oracle_bf16-vs-fp32 per-sequence logp errors are
    equal, 8.2e-4 abs; a change of reduction order in one LoRA product moves the
    loss by 3e-4 relative); measured 2.4e-4 / 2.9e-4, held to 1e-3 (north star)
    against both the fp32 and the bf16 oracle."""
    dims = O.JanusDims(n_layers=2, lora_r=16, lora_alpha=32)
    w = O.init_weights(dims, seed=3, dtype=torch.bfloat16, lora_b_std=1e-2)
    g = torch.Generator().manual_seed(9)
    B = 2
    text = [torch.randint(0, dims.vocab, (1, 24 - i), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, 576), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, 576), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    eng = build_engine(dims, w, B, 24, 576)
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ora = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16)
    o32 = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.float32)
    e = max(rel(logps[:B], ora.chosen_logps), rel(logps[B:], ora.rejected_logps))
    ge = max(rel(grads[k], ora.lora_grads[k]) for k in ora.lora_grads)
    g32 = max(rel(grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    floor = max(rel(ora.lora_grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    record_parity("step_7b_shapes_2_layers", logp=e, loss_fp32=abs(loss - float(o32.loss)) / float(o32.loss),
                  loss_bf16=abs(loss - float(ora.loss)) / float(ora.loss), grad_vs_bf16=ge, grad_vs_fp32=g32,
                  oracle_bf16_vs_fp32_grad=floor)
    print(f"\n7B-shape 2-layer: logp rel err {e:.2e}, loss {loss:.6f} vs bf16 {float(ora.loss):.6f} "
          f"fp32 {float(o32.loss):.6f}, max grad err {ge:.2e}")
    assert e < 1e-3
    # the loss kernel itself is exact given the logps
    l_from = O.simpo_loss(logps[:B], logps[B:])[0].mean()
    assert abs(float(l_from) - loss) < 1e-5
    assert abs(loss - float(o32.loss)) / float(o32.loss) < 1e-3
    assert abs(loss - float(ora.loss)) / float(ora.loss) < 1e-3
    assert ge < 5e-2
    assert g32 < GRAD_FP32_TOL["7b_2l"], (g32, floor)
    assert g32 < GRAD_FLOOR_RATIO * floor, (g32, floor)


def _oracle_dims(dims):
    return O.JanusDims(**{k: getattr(dims, k) for k in ("n_layers", "d_model", "d_ff", "n_heads", "head_dim", "vocab",
                                                      "img_vocab", "img_embed", "gen_head_dim", "lora_r",
                                                      "lora_alpha")})


def _unpad(text):
    """bench.synthetic_batch's [B, Lt] (-1 = right padding) -> the reference's list of [1, Lt_i]."""
    t = text.cpu()
    return [t[i:i + 1, : int((t[i] >= 0).sum())] for i in range(t.shape[0])]


class _LazyMasks:
    """{(layer, group): keep mask} of the HIP path's dropout in one forward call, generated when the
    oracle first asks for a layer (ospo_amd/dropout.py restates the device hash bit for bit)."""

    def __init__(self, M, kin, base_seed, call, p):
        self.M, self.kin, self.base, self.call, self.p, self.memo = M, kin, base_seed, call, p, {}

    def __bool__(self):
        return True

    def get(self, key):
        from ospo_amd import dropout as Dm
        if key not in self.memo:
            i, grp = key
            self.memo[key] = torch.from_numpy(
                Dm.keep_mask(self.M, self.kin[grp], Dm.layer_seed(self.base, self.call, i, grp), self.p))
        return self.memo[key]


def test_step_full_depth_7b_30_layers():
    """BASELINE config 2's model end to end: Janus-Pro-7B shapes, ALL 30 layers, two ragged pairs,
    forward + SimPO loss + backward to every LoRA adapter, against the bf16 and the fp32 oracle
    through the same 30 layers.

    Log-probs: 1e-3 relative of both oracles (north star), and no further from the fp32 oracle than
    LOGP_NOISE_RATIO = 1.25x the bf16 oracle's own distance from it (round 6, fixed before the suite run).
    Loss: beta = 10 turns the per-sequence log-prob rounding noise of a bf16 path (~1e-4 relative at 30
    layers) into ~1e-2 of a loss near 5 (dloss/dlogp = beta * sigmoid), so the loss is held only to the
    loss kernel's formula applied to the HIP log-probs (1e-5) and a fixed 1e-2 gross-error ceiling against
    the fp32 oracle; the north-star 1e-3 loss bound holds to 2 layers (README).  LoRA grads of every layer (reported for layers 0, 15 and 29): at most 1.25x the
    oracle's own bf16-autograd error against fp32."""
    from ospo_amd.engine import JANUS_PRO_7B, SimPOEngine, synthetic_weights
    dims = JANUS_PRO_7B
    w = synthetic_weights(dims, "cuda", seed=5, lora_seed=6, lora_b_std=1e-2)
    B, Lt, N = 2, 24, 576
    g = torch.Generator().manual_seed(17)
    text = [torch.randint(0, dims.vocab, (1, Lt - 3 * i), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    eng = SimPOEngine(dims, w, device="cuda", max_pairs=B, max_text_len=Lt, n_img_tokens=N)
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    wc = {k: v.cpu() for k, v in w.items()}
    del w, eng
    torch.cuda.empty_cache()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    odims = _oracle_dims(dims)
    ora = O.simpo_step(text, chosen, rejected, wc, odims, dtype=torch.bfloat16)
    o32 = O.simpo_step(text, chosen, rejected, wc, odims, dtype=torch.float32)
    e = max(rel(logps[:B], ora.chosen_logps), rel(logps[B:], ora.rejected_logps))
    e32 = max(rel(logps[:B], o32.chosen_logps), rel(logps[B:], o32.rejected_logps))
    l32 = float(o32.loss)
    el32 = abs(loss - l32) / l32
    el16 = abs(loss - float(ora.loss)) / float(ora.loss)
    floor_l = abs(float(ora.loss) - l32) / l32
    ge = {k: rel(grads[k], o32.lora_grads[k]) for k in o32.lora_grads}
    fl = {k: rel(ora.lora_grads[k], o32.lora_grads[k]) for k in o32.lora_grads}
    by_layer = {i: (max(v for k, v in ge.items() if k.startswith(f"layers.{i}.")),
                    max(v for k, v in fl.items() if k.startswith(f"layers.{i}."))) for i in (0, 15, 29)}
    record_parity("step_full_depth_7b_30_layers", logp=e, logp_vs_fp32=e32, loss=loss, loss_bf16_oracle=float(ora.loss),
                  loss_fp32_oracle=l32, loss_vs_fp32=el32, loss_vs_bf16=el16, oracle_bf16_vs_fp32_loss=floor_l,
                  grad_vs_fp32=max(ge.values()), oracle_bf16_vs_fp32_grad=max(fl.values()),
                  grads_layers_0_15_29={str(i): list(v) for i, v in by_layer.items()},
                  hip=logps.tolist(), oracle=[*ora.chosen_logps.tolist(), *ora.rejected_logps.tolist()])
    print(f"\n7B 30 layers: logp rel err {e:.2e} (vs fp32 {e32:.2e}); loss {loss:.6f} vs fp32 {l32:.6f} ({el32:.2e}), "
          f"bf16 {float(ora.loss):.6f} ({el16:.2e}), oracle bf16-vs-fp32 {floor_l:.2e}; grads (HIP, oracle-bf16) vs "
          f"fp32 by layer {by_layer}")
    assert e < 1e-3 and e32 < 1e-3
    assert abs(float(O.simpo_loss(logps[:B], logps[B:])[0].mean()) - loss) < 1e-5
    # the log-prob noise criterion (fixed before the round-6 suite run): no further from fp32 than 1.25x the bf16
    # oracle; the loss only against the fixed gross-error ceiling (beta = 10 amplifies bf16 log-prob noise)
    h32 = torch.cat([o32.chosen_logps, o32.rejected_logps]).float()
    d_ora = rel(torch.cat([ora.chosen_logps, ora.rejected_logps]).float(), h32)
    record_parity("step_full_depth_7b_30_layers_logp_noise", logp_hip_vs_fp32=rel(logps.float(), h32),
                  logp_oracle_bf16_vs_fp32=d_ora)
    assert rel(logps.float(), h32) <= LOGP_NOISE_RATIO * d_ora, (rel(logps.float(), h32), d_ora)
    assert el32 < 1e-2, (el32, floor_l)
    worst = max(ge, key=lambda k: ge[k] / fl[k])
    assert ge[worst] < GRAD_FLOOR_RATIO * fl[worst], (worst, ge[worst], fl[worst])
    # the oracle's own bf16 autograd sits 0.12-0.16 from fp32 at 30 layers, so the bound is that spread, per
    # tensor above and over all here; plus a fixed ceiling just above the measured HIP errors (0.107 / 0.124 /
    # 0.145 for layers 0 / 15 / 29, profiles/r04/parity_suite_r4v.jsonl), so a kernel change that
    # doubled the HIP error while staying under the spread would still fail
    assert max(ge.values()) < GRAD_FLOOR_RATIO * max(fl.values()), (max(ge.values()), max(fl.values()))
    assert max(ge.values()) < 0.16, max(ge.values())


BENCH_SEEDS_FIXTURE = "bench_config_seeds_oracle.npz"


def bench_seed_runs(n_seeds=3, **setup):
    """The HIP side of the bench-config checks: bench.simpo_setup(**setup)'s workload, the forward + SimPO loss of
    the bench's batches 0 .. n_seeds - 1.  Returns (runs, weights on the host, dims, dropout p, digest); a run is (text,
    chosen, rejected, HIP log-probs, HIP loss, the forward call index, M), digest the float64 sums and sums of
    squares of every weight and input (on the device), which pin the fixture to this exact workload."""
    import bench
    from ospo_amd.simpo import SimPOConfig, SimPOLossBuffers, simpo_forward
    dims, eng, batches, w = bench.simpo_setup(**setup)
    dig = []
    for k in sorted(w):
        x = w[k].double()
        dig += [float(x.sum()), float((x * x).sum())]
    runs = []
    for s in range(n_seeds):
        text, chosen, rejected = batches[s]
        dig += [float(t.double().sum()) for t in (text, chosen, rejected)]
        B = chosen.shape[0]
        logps = eng.forward(text, chosen, rejected)
        buf = SimPOLossBuffers(B, "cuda")
        _, mean, _ = simpo_forward(logps, B, SimPOConfig(), buf)
        runs.append((text.cpu(), chosen.cpu().long(), rejected.cpu().long(), logps.cpu().clone(),
                     float(mean.item()), eng._drop_call, eng.M))
    p = eng.lora_dropout
    wc = {k: v.cpu() for k, v in w.items()}
    del w, eng
    torch.cuda.empty_cache()
    return runs, wc, dims, p, np.array(dig, dtype=np.float64)


def bench_seed_oracle(runs, wc, dims, p, progress=print, mx8=False):
    """The bf16 and fp32 oracles (forward + loss) of each run, with the HIP path's dropout masks replayed:
    {"r16": [3, 2B], "r32": [3, 2B], "loss16": [3], "loss32": [3], "call": [3], "M": [3]} (six 30-layer CPU
    passes, ~1-2 min each: progress() after each)."""
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    odims = O.JanusDims(**{**_oracle_dims(dims).__dict__, "lora_dropout": p})
    kin = {"qkv": dims.d_model, "o": dims.d_model, "gu": dims.d_model, "down": dims.d_ff}
    out = {"r16": [], "r32": [], "loss16": [], "loss32": [], "call": [], "M": []}
    for s, (text, ch, rj, _logps, _loss, call, M) in enumerate(runs):
        masks = _LazyMasks(M, kin, 42, call, p)
        tl = _unpad(text)
        for dt, tag in ((torch.bfloat16, "16"), (torch.float32, "32")):
            o = O.simpo_step(tl, ch, rj, wc, odims, dtype=dt, backward=False, dropout_masks=masks, mx8=mx8)
            out["r" + tag].append(torch.cat([o.chosen_logps, o.rejected_logps]).float().numpy())
            out["loss" + tag].append(float(o.loss))
            progress(f"bench config seed {s}: {'bf16' if tag == '16' else 'fp32'} oracle done")
        out["call"].append(call)
        out["M"].append(M)
    return {k: np.array(v) for k, v in out.items()}


def test_bench_config_three_seeds_vs_oracle(capsys):
    """The workload bench.py times (BASELINE config 2): bench.simpo_setup's weights and engine, 4 ragged pairs,
    LoRA r = 16, dropout 0.05, all 30 layers -- the forward + SimPO loss of THREE batches (the bench's batches
    0, 1, 2: synthetic_batch seeds 0, 1, 2, each a fresh forward call with its own dropout masks) against the
    bf16 and fp32 oracles with the HIP path's masks replayed.  Seed 0's loss is the bench line's
    ``loss_first_step``.

    The oracle side (six 30-layer CPU passes, ~6 min) is the committed fixture tests/golden/
    bench_config_seeds_oracle.npz (tools/make_bench_seeds_fixture.py: bench_seed_oracle below, run on a GPU box)
    when its digest of every weight and input equals this workload's (the weights are drawn on the device, so the
    digest pins them); otherwise the oracles run here, with a progress line after each pass.

    Criterion (round 6, fixed before the suite run):
    - per seed, every per-sequence log-prob within 1e-3 relative of the bf16 AND the fp32 oracle (north star);
    - per seed, the loss kernel within 1e-5 of the SimPO formula applied to the HIP log-probs;
    - pooled over the 3 seeds (24 log-probs), the HIP log-probs no further from the fp32 oracle than
      LOGP_NOISE_RATIO = 1.25x the bf16 oracle's own distance from it (relative L2).  Pooled, because one
      seed's 8-value L2 norm is a noisy statistic; 1.25x, because the fp32 oracle is the value both bf16 paths
      approximate and the HIP path (fp32 accumulation, the same bf16 rounding points) must be at least about
      as close to it as the reference's own bf16 arithmetic.
    The SimPO loss itself is NOT held to 1e-3 here: beta = 10 turns the ~1.5e-4 relative log-prob noise of
    ANY bf16 path into 1e-3 .. 1e-2 of a loss near 5 (the bf16 oracle sits 2.3e-3 from the fp32 one on seed 0),
    so the north-star loss bound holds to 2 layers only (README); a fixed 1e-2 ceiling
    guards against gross errors."""
    runs, wc, dims, p, dig = bench_seed_runs()
    ref = None
    if FX.exists(BENCH_SEEDS_FIXTURE):
        z = FX.load(BENCH_SEEDS_FIXTURE)
        if z["digest"].shape == dig.shape and np.allclose(z["digest"], dig, rtol=1e-12, atol=0):
            ref = {k: z[k] for k in ("r16", "r32", "loss16", "loss32", "call", "M")}
    if ref is None:
        def progress(msg):
            with capsys.disabled():
                print(msg, flush=True)
        progress("bench config: fixture digest differs or fixture absent, running the oracles")
        ref = bench_seed_oracle(runs, wc, dims, p, progress)
    H, R16, R32 = [], [], []
    for s, (text, ch, rj, logps, loss, call, M) in enumerate(runs):
        B = ch.shape[0]
        assert int(ref["call"][s]) == call and int(ref["M"][s]) == M, (s, call, M)
        r16, r32 = torch.from_numpy(ref["r16"][s]).float(), torch.from_numpy(ref["r32"][s]).float()
        l16, l32 = float(ref["loss16"][s]), float(ref["loss32"][s])
        e, e32 = rel(logps, r16), rel(logps, r32)
        el32, floor_l = abs(loss - l32) / l32, abs(l16 - l32) / l32
        record_parity("bench_config_seed", seed=s, logp=e, logp_vs_fp32=e32, oracle_bf16_logp_vs_fp32=rel(r16, r32),
                      loss=loss, loss_bf16_oracle=l16, loss_fp32_oracle=l32, loss_vs_fp32=el32,
                      oracle_bf16_vs_fp32_loss=floor_l, hip=logps.tolist(), oracle_bf16=r16.tolist(),
                      oracle_fp32=r32.tolist())
        print(f"\nbench config seed {s}: loss {loss:.6f} fp32 oracle {l32:.6f} ({el32:.2e}; bf16 oracle "
              f"{l16:.6f}, {floor_l:.2e}); logp rel err vs bf16 {e:.2e} vs fp32 {e32:.2e} (bf16 oracle "
              f"vs fp32 {rel(r16, r32):.2e})", flush=True)
        assert e < 1e-3 and e32 < 1e-3, (s, e, e32)
        assert abs(float(O.simpo_loss(logps[:B], logps[B:])[0].mean()) - loss) < 1e-5
        assert el32 < 1e-2, (s, el32)
        H.append(logps.float()), R16.append(r16), R32.append(r32)
    h, r16, r32 = torch.cat(H), torch.cat(R16), torch.cat(R32)
    d_hip, d_ora = rel(h, r32), rel(r16, r32)
    record_parity("bench_config_three_seeds_pooled", logp_hip_vs_fp32=d_hip, logp_oracle_bf16_vs_fp32=d_ora,
                  ratio=d_hip / d_ora)
    assert d_hip <= LOGP_NOISE_RATIO * d_ora, (d_hip, d_ora)


BENCH_MX8_FIXTURE = "bench_mx8_r32_seed_oracle.npz"


def _bench_mx8_30_layers(capsys):
    """Config 5 at depth: the MXFP8 bench workload (``bench.py --linear-dtype mx8 --lora-r 32``: bench.simpo_setup
    with MXFP8 decoder Linears, LoRA r = 32, dropout 0.05, 4 ragged pairs, all 30 layers), batch 0's forward +
    SimPO loss, and the oracle's fp8 mode (oracle/mx8_ref.py quantizers) in bf16 and fp32 with the masks replayed:
    the committed fixture tests/golden/bench_mx8_r32_seed_oracle.npz (tools/make_bench_seeds_fixture.py --mx8,
    digest-pinned as the bf16 3-seed test's; recomputed live when the digest differs)."""
    runs, wc, dims, p, dig = bench_seed_runs(n_seeds=1, lora_r=32, linear_dtype="mx8")
    ref = None
    if FX.exists(BENCH_MX8_FIXTURE):
        z = FX.load(BENCH_MX8_FIXTURE)
        if z["digest"].shape == dig.shape and np.allclose(z["digest"], dig, rtol=1e-12, atol=0):
            ref = {k: z[k] for k in ("r16", "r32", "loss16", "loss32", "call", "M")}
    if ref is None:
        def progress(msg):
            with capsys.disabled():
                print(msg, flush=True)
        progress("bench mx8 config: fixture digest differs or fixture absent, running the fp8 oracles")
        ref = bench_seed_oracle(runs, wc, dims, p, progress, mx8=True)
    text, ch, rj, logps, loss, call, M = runs[0]
    assert int(ref["call"][0]) == call and int(ref["M"][0]) == M, (call, M)
    r16, r32 = torch.from_numpy(ref["r16"][0]).float(), torch.from_numpy(ref["r32"][0]).float()
    e16, e32, d_ora = rel(logps, r16), rel(logps, r32), rel(r16, r32)
    record_parity("bench_mx8_r32_30_layers", logp_vs_mx8_bf16_oracle=e16, logp_vs_mx8_fp32_oracle=e32,
                  mx8_oracle_bf16_vs_fp32=d_ora, ratio=e32 / d_ora, loss=loss, loss_mx8_bf16_oracle=float(ref["loss16"][0]),
                  loss_mx8_fp32_oracle=float(ref["loss32"][0]), hip=logps.tolist(), oracle_bf16=r16.tolist(),
                  oracle_fp32=r32.tolist())
    print(f"\nbench mx8 r32 30 layers: logp rel err vs the fp8 oracle bf16 {e16:.2e} fp32 {e32:.2e} (oracle bf16 vs "
          f"fp32 {d_ora:.2e}); loss {loss:.6f} vs {float(ref['loss16'][0]):.6f} / {float(ref['loss32'][0]):.6f}",
          flush=True)
    return logps, loss, ch.shape[0], r16, r32, e32, d_ora


def test_bench_mx8_r32_30_layers_gross_errors(capsys):
    """Config 5 at 30 layers (see _bench_mx8_30_layers): every log-prob within 1e-2 relative of both fp8 oracles
    and the loss kernel within 1e-5 of the formula (the gross-error part of the criterion fixed before the run)."""
    logps, loss, B, r16, r32, _, _ = _bench_mx8_30_layers(capsys)
    assert abs(float(O.simpo_loss(logps[:B], logps[B:])[0].mean()) - loss) < 1e-5
    assert (logps.float() - r16).abs().div(r16.abs()).max() < 1e-2
    assert (logps.float() - r32).abs().div(r32.abs()).max() < 1e-2


@pytest.mark.xfail(strict=True, reason="measured round 6 (DESIGN section 8): the HIP fp8 log-probs sit 2.06e-3 "
                                       "from the fp32 fp8 oracle against the bf16 fp8 oracle's 1.43e-3 (1.44x > "
                                       "1.25x); they sit 1.0e-3 from the bf16 fp8 oracle")
def test_bench_mx8_r32_30_layers_noise_criterion(capsys):
    """The bf16 gate's noise criterion applied to config 5, fixed before the run: the HIP log-probs no further from
    the fp32 fp8 oracle than 1.25x the bf16 fp8 oracle's own distance from it.  It FAILS (1.44x) and is kept as
    a strict xfail, not loosened: in the fp8 arithmetic the fp32 oracle quantizes unrounded activations, so its
    fp8 codes differ from those of both bf16 paths (HIP and the bf16 oracle quantize bf16 activations alike), and
    the fp32 oracle is not the common target it is in bf16."""
    _, _, _, _, _, e32, d_ora = _bench_mx8_30_layers(capsys)
    assert e32 <= LOGP_NOISE_RATIO * d_ora, (e32, d_ora)


def test_step_7b_shapes_8_pairs_two_layers():
    """BASELINE config 3's per-GPU batch: 8 pairs (16 sequences, M = 9 600 rows) at Janus-Pro-7B
    shapes, 2 layers, ragged prompts, forward + loss + backward against both oracles.  Log-probs
    1e-3; loss 1e-3 of the fp32 oracle (north star); grads as the other 7B-shape cases."""
    dims = O.JanusDims(n_layers=2, lora_r=16, lora_alpha=32)
    w = O.init_weights(dims, seed=13, dtype=torch.bfloat16, lora_b_std=1e-2)
    g = torch.Generator().manual_seed(14)
    B = 8
    text = [torch.randint(0, dims.vocab, (1, 24 - (i % 5)), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, 576), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, 576), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    eng = build_engine(dims, w, B, 24, 576)
    assert eng.Mcap >= 9600
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    del eng
    torch.cuda.empty_cache()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ora = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16)
    o32 = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.float32)
    e = max(rel(logps[:B], ora.chosen_logps), rel(logps[B:], ora.rejected_logps))
    l32 = float(o32.loss)
    el32, el16 = abs(loss - l32) / l32, abs(loss - float(ora.loss)) / float(ora.loss)
    g32 = max(rel(grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    floor = max(rel(ora.lora_grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    record_parity("step_7b_shapes_8_pairs", logp=e, loss_fp32=el32, loss_bf16=el16, grad_vs_fp32=g32,
                  oracle_bf16_vs_fp32_grad=floor)
    print(f"\n7B-shape 8 pairs: logp {e:.2e}, loss vs fp32 {el32:.2e}, vs bf16 {el16:.2e}, grads {g32:.2e} "
          f"(floor {floor:.2e})")
    assert e < 1e-3
    assert abs(float(O.simpo_loss(logps[:B], logps[B:])[0].mean()) - loss) < 1e-5
    assert el32 < 1e-3 and el16 < 1e-3
    assert g32 < GRAD_FP32_TOL["7b_2l"], (g32, floor)
    assert g32 < GRAD_FLOOR_RATIO * floor, (g32, floor)


def test_trajectory_five_steps_7b_shapes_two_layers_vs_oracle():
    """Training past step 1: five optimizer steps of the bench workload (bench.simpo_setup: 4 ragged pairs,
    T = 600, LoRA r = 16, dropout 0.05) at Janus-Pro-7B widths with 2 decoder layers -- HIP forward, SimPO
    loss, backward, clip 1.0 + AdamW each step (simpo.train_step, the bench's step) -- against the oracle's
    own trajectory (oracle.simpo_step + clip_and_adamw: PL clip -> torch AdamW on the bf16 LoRA tensors,
    ospo/utils/train.py:30, ospo/wrapper/train.py:107-115), the HIP dropout masks of every step replayed.
    Run in bf16 (the reference's path) and in fp32 (the value both approximate).
    Bounds (fixed; round 6 dropped round 5's raised 4e-3 loss bound against the bf16 oracle -- the fp32
    trajectory is the target, the bf16 one only gauges the noise): every step's loss within 2e-3 relative of
    the fp32 trajectory (measured <= 1.1e-3); the LoRA update after 5 steps (params - init, all tensors) at
    most 1.25x as far from the fp32 trajectory's update as the bf16 oracle's update is, and within 0.5x of
    that distance of the bf16 oracle's update (round 4's bound, restored: measured 0.37x).
    Round 5: each trajectory starts from its own copy of the weights.  Until round 4, ``v.to(torch.bfloat16)``
    of the already-bf16 LoRA tensors returned the same tensors, the bf16 trajectory's AdamW updated the
    weights in place, and the fp32 trajectory started from the bf16 trajectory's step-5 params: that, not
    bf16 arithmetic, was the 2-11 % "bf16-vs-fp32 gap" (tools/traj_diag.py: 5e-4 at step 1 from the same
    weights, profiles/r05/traj_diag_step1.log)."""
    import bench
    from ospo_amd.simpo import SimPOConfig, SimPOLossBuffers, train_step
    dims, eng, batches, w = bench.simpo_setup(layers=2)
    cfg = SimPOConfig()
    B = batches[0][1].shape[0]
    buf = SimPOLossBuffers(B, "cuda")
    steps = 5
    hip_loss, calls, rows = [], [], []
    for s in range(steps):
        text, ch, rj = batches[s % len(batches)]
        out = train_step(eng, text, ch, rj, cfg, buf)
        hip_loss.append(float(out["loss"].item()))
        calls.append(eng._drop_call)
        rows.append(eng.M)
    torch.cuda.synchronize()
    hip_p = {k: v.float().cpu() for k, v in eng.lora_tensors().items()}
    p = eng.lora_dropout
    wc = {k: v.cpu() for k, v in w.items()}
    del w, eng
    torch.cuda.empty_cache()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    odims = O.JanusDims(**{**_oracle_dims(dims).__dict__, "lora_dropout": p})
    kin = {"qkv": dims.d_model, "o": dims.d_model, "gu": dims.d_model, "down": dims.d_ff}
    init = {k: v.float() for k, v in wc.items() if ".lora_" in k}

    def trajectory(dt):
        ww = {k: (v.to(dt).clone() if v.is_floating_point() else v) for k, v in wc.items()}
        params = {k: ww[k] for k in ww if ".lora_" in k}
        state, losses = {}, []
        for s in range(steps):
            text, ch, rj = batches[s % len(batches)]
            masks = _LazyMasks(rows[s], kin, 42, calls[s], p)
            o = O.simpo_step(_unpad(text), ch.cpu().long(), rj.cpu().long(), ww, odims, dtype=dt, dropout_masks=masks)
            losses.append(float(o.loss))
            O.clip_and_adamw(params, o.lora_grads, state, lr=cfg.lr, betas=cfg.betas, eps=cfg.eps,
                             weight_decay=cfg.weight_decay, max_norm=cfg.max_norm)
        return losses, {k: v.float() for k, v in params.items()}

    l16, p16 = trajectory(torch.bfloat16)
    l32, p32 = trajectory(torch.float32)
    names = sorted(init)
    cat = lambda d: torch.cat([(d[k] - init[k]).flatten() for k in names])  # noqa: E731
    d_hip, d16, d32 = cat(hip_p), cat(p16), cat(p32)
    e_upd32, floor_upd, e_upd16 = rel(d_hip, d32), rel(d16, d32), rel(d_hip, d16)
    e_loss = [abs(a - b) / abs(b) for a, b in zip(hip_loss, l32)]
    gap = [abs(a - b) / abs(b) for a, b in zip(l16, l32)]
    record_parity("trajectory_5steps_7b_2l", hip_loss=hip_loss, oracle_bf16_loss=l16, oracle_fp32_loss=l32,
                  loss_rel_vs_fp32=e_loss, oracle_bf16_loss_gap=gap, update_rel_vs_fp32=e_upd32,
                  update_rel_vs_bf16=e_upd16, oracle_bf16_update_vs_fp32=floor_upd,
                  update_norm_rel=float(d_hip.norm() / d32.norm()))
    e16 = [abs(a - b) / abs(b) for a, b in zip(hip_loss, l16)]
    record_parity("trajectory_5steps_7b_2l_vs_bf16", loss_rel_vs_bf16=e16)
    for s in range(steps):
        assert e_loss[s] < 2e-3, (s, e_loss[s], gap[s])
    assert hip_loss[-1] != hip_loss[0]  # the adapters did train
    assert e_upd32 < GRAD_FLOOR_RATIO * floor_upd, (e_upd32, floor_upd)
    # both bf16 trajectories round the same AdamW updates onto the same bf16 parameter grid, so their updates sit
    # closer to each other than either does to fp32 (measured 0.092 vs 0.25, round 5)
    assert e_upd16 < 0.5 * floor_upd, (e_upd16, floor_upd)


def test_engine_optimizer_step_matches_torch_adamw():
    """clip(1.0) + AdamW on the flat LoRA buffer vs torch.optim.AdamW on the oracle's tensors."""
    z = FX.load("step_tiny_bf16.npz")
    dims = FX.dims_of(z)
    w = FX.step_weights(z, "step_tiny_bf16.npz", dims)
    text, chosen, rejected = FX.step_inputs(z)
    B, N = chosen.shape
    eng = build_engine(dims, w, B, max(t.shape[1] for t in text), N)
    algo = json.loads(str(z["algo"]))
    _, _, grads = run_hip_step(eng, text, chosen, rejected, algo)
    params = {k: v.float().cpu().to(torch.bfloat16).clone() for k, v in eng.lora_tensors().items()}
    O.clip_and_adamw(params, grads, {}, lr=4e-5, betas=(0.9, 0.95), eps=1e-8, max_norm=1.0)
    eng.optimizer_step(4e-5, (0.9, 0.95), 1e-8, 0.0, 1.0)
    torch.cuda.synchronize()
    new = {k: v.cpu() for k, v in eng.lora_tensors().items()}
    mism = sum(int((new[k] != params[k]).sum()) for k in params)
    total = sum(p.numel() for p in params.values())
    assert mism / total < 0.01, (mism, total)


@pytest.mark.parametrize("r", [32, 8])
def test_step_lora_rank_variants_vs_oracle(r):
    """configs/peft/lora.yaml trains at r = 32 (alpha 64): u with 6 n-tiles over Rp = 128,
    g block-diagonal with 2 n-tiles per module.  r = 8 exercises the non-multiple-of-16
    fallback.  Small dims, bf16, against the oracle."""
    dims = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=2048,
                       gen_head_dim=256, lora_r=r, lora_alpha=2 * r)
    w = O.init_weights(dims, seed=11, dtype=torch.bfloat16, lora_b_std=1e-2)
    g = torch.Generator().manual_seed(12)
    B, N = 3, 64
    text = [torch.randint(0, dims.vocab, (1, 10 - 2 * i), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    eng = build_engine(dims, w, B, 10, N)
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    ora = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16)
    o32 = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.float32)
    assert max(rel(logps[:B], ora.chosen_logps), rel(logps[B:], ora.rejected_logps)) < 1e-3
    assert abs(loss - float(ora.loss)) / float(ora.loss) < 1e-3
    ge = max(rel(grads[k], ora.lora_grads[k]) for k in ora.lora_grads)
    g32 = max(rel(grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    floor = max(rel(ora.lora_grads[k], o32.lora_grads[k]) for k in o32.lora_grads)
    record_parity(f"step_lora_r{r}", grad_vs_bf16=ge, grad_vs_fp32=g32, oracle_bf16_vs_fp32_grad=floor)
    assert ge < 5e-2
    assert g32 < GRAD_FP32_TOL[f"r{r}"]
    assert g32 < GRAD_FLOOR_RATIO * floor, (g32, floor)


@pytest.mark.parametrize("r", [16, 32, 24])
def test_step_lora_dropout_vs_oracle_with_replayed_masks(r):
    """configs/peft/lora.yaml: lora_dropout 0.05 (at its r = 32 and the bench's r = 16; r = 24 gives q|k|v a
    5-tile u product, which writes no keep bits, so its consumers re-hash the mask).  The HIP path's
    counter-based masks (ospo_amd/dropout.py) are replayed into the oracle, which then computes peft's
    dropout(x) exactly: forward log-probs, loss and every LoRA grad must match."""
    from ospo_amd import dropout as Dm
    p = 0.05
    dims = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=2048,
                       gen_head_dim=256, lora_r=r, lora_alpha=2 * r, lora_dropout=p)
    w = O.init_weights(dims, seed=21, dtype=torch.bfloat16, lora_b_std=1e-2)
    g = torch.Generator().manual_seed(22)
    B, N = 2, 64
    text = [torch.randint(0, dims.vocab, (1, 8 - 2 * i), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    from ospo_amd.engine import ModelDims, SimPOEngine
    eng = SimPOEngine(ModelDims.from_any(dims), w, device="cuda", max_pairs=B, max_text_len=8, n_img_tokens=N,
                      lora_dropout=p, dropout_seed=7)
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    call = eng._drop_call
    M = 2 * B * (8 + N)
    kin = {"qkv": dims.d_model, "o": dims.d_model, "gu": dims.d_model, "down": dims.d_ff}
    masks = {(i, grp): torch.from_numpy(Dm.keep_mask(M, kin[grp], Dm.layer_seed(7, call, i, grp), p))
             for i in range(dims.n_layers) for grp in kin}
    ora = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16, dropout_masks=masks)
    assert max(rel(logps[:B], ora.chosen_logps), rel(logps[B:], ora.rejected_logps)) < 1e-3
    assert abs(loss - float(ora.loss)) / float(ora.loss) < 1e-3
    ge = max(rel(grads[k], ora.lora_grads[k]) for k in ora.lora_grads)
    assert ge < 5e-2, ge
    # without replaying the masks the grads differ: the mask is really applied
    plain = O.simpo_step(text, chosen, rejected, w, O.JanusDims(**{**dims.__dict__, "lora_dropout": 0.0}),
                         dtype=torch.bfloat16)
    assert max(rel(grads[k], plain.lora_grads[k]) for k in plain.lora_grads) > 0.05


def test_step_side_after_norm_same_grads():
    """side_after_norm only moves where a layer's dA work joins the side stream (after the input-norm
    backward instead of after the q|k|v dX GEMM); with dropout and 4 layers (both operand copies in use)
    the log-probs are bit-equal and the grads equal up to the dA kernel's fp32-atomic summation order."""
    dims = O.JanusDims(n_layers=4, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=2048,
                       gen_head_dim=256, lora_r=16, lora_alpha=32, lora_dropout=0.05)
    w = O.init_weights(dims, seed=41, dtype=torch.bfloat16, lora_b_std=1e-2)
    g = torch.Generator().manual_seed(42)
    B, Lt, N = 2, 8, 64
    text = [torch.randint(0, dims.vocab, (1, Lt - i), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    from ospo_amd.engine import ModelDims, SimPOEngine
    out = []
    for late in (False, True):
        eng = SimPOEngine(ModelDims.from_any(dims), w, device="cuda", max_pairs=B, max_text_len=Lt,
                          n_img_tokens=N, lora_dropout=0.05, dropout_seed=7, side_after_norm=late)
        out.append(run_hip_step(eng, text, chosen, rejected, algo))
    (l0, s0, g0), (l1, s1, g1) = out
    assert torch.equal(l0, l1) and s0 == s1
    assert max(rel(g1[k], g0[k]) for k in g0) < 1e-5


def test_step_gdb_gu_only_same_step():
    """gdb_groups=("gu",) (round 5 A/B): the q|k|v, o and down groups take g from the skinny product on the main
    stream and dB from the f32-atomic product on the side stream, instead of the fused ospo_lora_gdb stream (the
    gate|up group stays fused with the SwiGLU backward).  The forward is untouched (log-probs and loss bit-equal);
    g sums the same products in another order, so the grads agree to bf16 rounding of g, well inside the
    oracle tolerances."""
    dims = O.JanusDims(n_layers=4, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=2048,
                       gen_head_dim=256, lora_r=16, lora_alpha=32, lora_dropout=0.05)
    w = O.init_weights(dims, seed=43, dtype=torch.bfloat16, lora_b_std=1e-2)
    g = torch.Generator().manual_seed(44)
    B, Lt, N = 2, 8, 64
    text = [torch.randint(0, dims.vocab, (1, Lt - i), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    from ospo_amd.engine import ModelDims, SimPOEngine
    out = []
    for groups in (("qkv", "o", "gu", "down"), ("gu",)):
        eng = SimPOEngine(ModelDims.from_any(dims), w, device="cuda", max_pairs=B, max_text_len=Lt,
                          n_img_tokens=N, lora_dropout=0.05, dropout_seed=9, gdb_groups=groups)
        out.append(run_hip_step(eng, text, chosen, rejected, algo))
    (l0, s0, g0), (l1, s1, g1) = out
    assert torch.equal(l0, l1) and s0 == s1
    err = max(rel(g1[k], g0[k]) for k in g0)
    record_parity("gdb_gu_only_vs_fused", grad_rel=err)
    assert err < 1e-2, err


def _mx8_case(dims, seed, B, Lt, N):
    w = O.init_weights(dims, seed=seed, dtype=torch.bfloat16, lora_b_std=1e-2)
    g = torch.Generator().manual_seed(seed + 1)
    text = [torch.randint(0, dims.vocab, (1, Lt - i), generator=g, dtype=torch.int32) for i in range(B)]
    chosen = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    rejected = torch.randint(0, dims.img_vocab, (B, N), generator=g)
    algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
    from ospo_amd.engine import ModelDims, SimPOEngine
    eng = SimPOEngine(ModelDims.from_any(dims), w, device="cuda", max_pairs=B, max_text_len=Lt, n_img_tokens=N,
                      linear_dtype="mx8")
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ora = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16, mx8=True)
    bf = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16, backward=False)
    e = max(rel(logps[:B], ora.chosen_logps), rel(logps[B:], ora.rejected_logps))
    e_bf = max(rel(logps[:B], bf.chosen_logps), rel(logps[B:], bf.rejected_logps))
    el = abs(loss - float(ora.loss)) / float(ora.loss)
    ge = {k: rel(grads[k], ora.lora_grads[k]) for k in ora.lora_grads}
    # the noise floor of fp8 gradients: the oracle's own bf16 and fp32 runs of the same fp8 step differ
    # because bf16-level differences in a quantizer's input flip ~1/16 of the fp8 roundings they touch
    o32 = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.float32, mx8=True)
    floor = {k: rel(o32.lora_grads[k], ora.lora_grads[k]) for k in ora.lora_grads}
    _mx8_case.loss_floor = abs(float(o32.loss) - float(ora.loss)) / float(ora.loss)
    _mx8_case.el32 = abs(loss - float(o32.loss)) / float(o32.loss)
    ratio = {k: ge[k] / max(floor[k], 5e-2) for k in ge}
    print(f"\nmx8 D{dims.d_model}: logp rel err vs mx8 oracle {e:.2e} (vs bf16 oracle {e_bf:.2e}); "
          f"loss {loss:.6f} vs {float(ora.loss):.6f} ({el:.2e}); max grad rel err {max(ge.values()):.2e}, "
          f"oracle bf16-vs-fp32 grad floor {max(floor.values()):.2e}, max err/max(floor, 5e-2) {max(ratio.values()):.2f}")
    return logps, loss, e, el, ratio, ora, B


def test_step_mx8_small_vs_oracle():
    """BASELINE config 5 arithmetic (MXFP8 frozen Linears, bf16 LoRA) against the oracle's
    fp8 mode (oracle/mx8_ref.py: same quantizer, fp32 products of the dequantized operands).
    The two paths quantize bf16 activations that differ by bf16 rounding noise, so an
    occasional block lands on a different fp8 code; log-probs are held to 1e-3 relative as in
    bf16, the loss to 3e-3, and each LoRA grad to 1.5x the larger of 5e-2 and the fp8 noise floor
    (the oracle's own bf16-vs-fp32 difference on the same fp8 step)."""
    dims = O.JanusDims(n_layers=2, d_model=256, d_ff=512, n_heads=2, vocab=512, img_vocab=2048,
                       gen_head_dim=256, lora_r=16, lora_alpha=32)
    logps, loss, e, el, ratio, ora, B = _mx8_case(dims, 31, 3, 10, 64)
    assert e < 1e-3
    assert abs(float(O.simpo_loss(logps[:B], logps[B:])[0].mean()) - loss) < 1e-5
    assert el < 3e-3
    assert max(ratio.values()) < 1.5, sorted(ratio.items(), key=lambda kv: -kv[1])[:3]


def test_step_mx8_full_size_7b_shapes_two_layers():
    """Config 5 at Janus-Pro-7B shapes (D 4096, F 11008, 32 heads, T = 600), 2 layers, 2 pairs."""
    dims = O.JanusDims(n_layers=2, lora_r=16, lora_alpha=32)
    logps, loss, e, el, ratio, ora, B = _mx8_case(dims, 41, 2, 24, 576)
    assert e < 1e-3
    assert el < 3e-3
    assert max(ratio.values()) < 1.5, sorted(ratio.items(), key=lambda kv: -kv[1])[:3]


def test_step_mx8_full_size_7b_shapes_lora_r32():
    """Config 5 exactly: MXFP8 frozen Linears with LoRA r = 32 (alpha 64, configs/peft/lora.yaml) at
    Janus-Pro-7B shapes, 2 layers, 2 pairs.  Log-probs within 1e-3 (north star; measured 4.0e-4).  The
    loss: beta = 10 turns a 4e-4 relative log-prob difference (4e-3 absolute at logp ~ -10) into ~4e-2
    of the margin; measured 8.4e-3 relative against the bf16 fp8 oracle, so held to 1.5e-2 and to
    the side of the fp32 fp8 oracle no further than twice the oracle's own bf16-vs-fp32 spread
    (or 1e-2)."""
    dims = O.JanusDims(n_layers=2, lora_r=32, lora_alpha=64)
    logps, loss, e, el, ratio, ora, B = _mx8_case(dims, 43, 2, 24, 576)
    record_parity("step_mx8_7b_r32", logp=e, loss=el, loss_vs_fp32=_mx8_case.el32, loss_floor=_mx8_case.loss_floor,
                  grad_ratio=max(ratio.values()))
    assert e < 1e-3
    assert abs(float(O.simpo_loss(logps[:B], logps[B:])[0].mean()) - loss) < 1e-5
    assert el < 1.5e-2
    assert _mx8_case.el32 < max(1e-2, 2 * _mx8_case.loss_floor)
    assert max(ratio.values()) < 1.5, sorted(ratio.items(), key=lambda kv: -kv[1])[:3]
