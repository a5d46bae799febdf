"""Pin the CPU oracle (oracle/simpo_ref.py) against golden vectors produced by
the reference's own train.py functions (tests/golden/make_golden.py)."""
import hashlib
import json

import numpy as np
import pytest
import torch

from oracle import simpo_ref as O
from tests import fixtures as FX


def test_get_batch_logps_kat():
    z = FX.load("logps_kat.npz")
    logits = FX.bits_to_bf16(z["logits_bf16"]).float()
    labels = torch.from_numpy(z["labels"])
    avg = O.get_batch_logps(logits, labels, average_log_prob=True)
    tot = O.get_batch_logps(logits, labels, average_log_prob=False)
    torch.testing.assert_close(avg, torch.from_numpy(z["logps_avg"]), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(tot, torch.from_numpy(z["logps_sum"]), rtol=1e-6, atol=1e-5)


def test_get_batch_logps_shape_error():
    with pytest.raises(ValueError):
        O.get_batch_logps(torch.zeros(2, 5, 7), torch.zeros(2, 4, dtype=torch.long))


@pytest.mark.parametrize("j", range(4))
def test_simpo_loss_kat(j):
    z = FX.load("logps_kat.npz")
    beta, gbr, ls, lt = json.loads(str(z[f"simpo{j}::params"]))
    c, r = torch.from_numpy(z["c"]), torch.from_numpy(z["r"])
    losses, cr, rr = O.simpo_loss(c, r, beta, gbr, ls, lt)
    torch.testing.assert_close(losses, torch.from_numpy(z[f"simpo{j}::losses"]), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(cr, torch.from_numpy(z[f"simpo{j}::chosen_rewards"]))
    torch.testing.assert_close(rr, torch.from_numpy(z[f"simpo{j}::rejected_rewards"]))


def test_simpo_loss_unknown_type():
    with pytest.raises(ValueError):
        O.simpo_loss(torch.zeros(1), torch.zeros(1), loss_type="ipo")


def _run(name, dtype):
    z = FX.load(name)
    dims = FX.dims_of(z)
    algo = json.loads(str(z["algo"]))
    text, chosen, rejected = FX.step_inputs(z)
    w = FX.step_weights(z, name, dims)
    out = O.simpo_step(text, chosen, rejected, w, dims, dtype=dtype, beta=algo["beta"],
                       gamma_beta_ratio=algo["gamma_beta_ratio"], label_smoothing=algo["label_smoothing"],
                       loss_type=algo["loss_type"], sft_weight=algo.get("sft_weight", 0.0))
    return out, FX.step_outputs(z)


def test_oracle_tiny_fp32_matches_reference():
    """fp32: the oracle must equal the reference to fp32 round-off."""
    out, ref = _run("step_tiny_fp32.npz", torch.float32)
    torch.testing.assert_close(out.chosen_logps, ref["chosen_logps"], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out.rejected_logps, ref["rejected_logps"], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out.loss, ref["loss"], rtol=1e-5, atol=1e-5)
    for k, g in ref["grads"].items():
        assert FX.rel_err(out.lora_grads[k].float(), g) < 1e-4, k
    for k, v in ref["logged"].items():
        key = k.split("/", 1)[1]
        if key in out.metrics:
            assert out.metrics[key] == pytest.approx(v, rel=1e-4, abs=1e-5), k


def test_oracle_tiny_sft_fp32_matches_reference():
    """algo.sft_weight = 0.5: loss = SimPO + 0.5 * CE(chosen logits) (train.py:421-430), the
    grads through both terms and the logged sft_loss / logits metrics."""
    out, ref = _run("step_tiny_sft_fp32.npz", torch.float32)
    torch.testing.assert_close(out.loss, ref["loss"], rtol=1e-5, atol=1e-5)
    for k, g in ref["grads"].items():
        assert FX.rel_err(out.lora_grads[k].float(), g) < 1e-4, k
    for k, v in ref["logged"].items():
        assert out.metrics[k.split("/", 1)[1]] == pytest.approx(v, rel=1e-4, abs=1e-6), k


def test_oracle_tiny_bf16_matches_reference():
    """bf16: the oracle keeps log_softmax in fp32 while the reference
    CPU bf16 path runs it in bf16, so logps agree to ~3e-3 relative."""
    out, ref = _run("step_tiny_bf16.npz", torch.bfloat16)
    assert FX.rel_err(out.chosen_logps, ref["chosen_logps"]) < 4e-3
    assert FX.rel_err(out.rejected_logps, ref["rejected_logps"]) < 4e-3
    for k, g in ref["grads"].items():
        assert FX.rel_err(out.lora_grads[k].float(), g) < 0.1, k


def test_oracle_bf16_vs_fp32_reference():
    """The bf16 oracle against the fp32 reference (same bf16-representable weights)."""
    out, _ = _run("step_tiny_weights.npz".replace("weights", "bf16"), torch.bfloat16)
    ref32 = FX.step_outputs(FX.load("step_tiny_fp32.npz"))
    assert FX.rel_err(out.chosen_logps, ref32["chosen_logps"]) < 2e-3
    assert FX.rel_err(out.rejected_logps, ref32["rejected_logps"]) < 2e-3


def test_oracle_1b_2layer_matches_reference():
    z = FX.load("step_1b2l_bf16.npz")
    dims = FX.dims_of(z)
    w = FX.step_weights(z, "step_1b2l_bf16.npz", dims)
    h = hashlib.sha256()
    for k in sorted(w):
        h.update(k.encode())
        h.update(w[k].float().numpy().tobytes())
    assert h.hexdigest() == str(z["weights_sha256"]), "init_weights drifted from the fixture"
    out, ref = _run("step_1b2l_bf16.npz", torch.bfloat16)
    assert FX.rel_err(out.chosen_logps, ref["chosen_logps"]) < 4e-3
    assert FX.rel_err(out.rejected_logps, ref["rejected_logps"]) < 4e-3
