"""One small SimPO step on cuda:0 through libospo_hip.so, checked against the CPU
oracle (used by __graft_entry__.smoke())."""
import json

import torch

from oracle import simpo_ref as O
from tests import fixtures as FX


def run_smoke():
    from tests.test_gpu_step import build_engine, pad_text, rel, run_hip_step
    name = "step_tiny_bf16.npz"
    z = FX.load(name)
    dims = FX.dims_of(z)
    algo = json.loads(str(z["algo"]))
    text, chosen, rejected = FX.step_inputs(z)
    w = FX.step_weights(z, name, dims)
    B, N = chosen.shape
    eng = build_engine(dims, w, B, max(t.shape[1] for t in text), N)
    logps, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
    ora = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16)
    e = max(rel(logps[:B], ora.chosen_logps), rel(logps[B:], ora.rejected_logps))
    ge = max(rel(grads[k], ora.lora_grads[k]) for k in ora.lora_grads)
    print(f"smoke: loss {loss:.6f} (oracle {float(ora.loss):.6f}) logp rel err {e:.2e} grad rel err {ge:.2e}")
    assert e < 1e-3 and ge < 5e-2, (e, ge)


if __name__ == "__main__":
    run_smoke()
