"""Why the bf16 and fp32 oracles differ by 7 % in loss at step 1 of the trajectory test (verdict r4 item 5).

The trajectory test's workload (bench.simpo_setup(layers=2): 7B widths, 2 decoder layers, 4 ragged pairs,
dropout 0.05), step 1 only, forward: per-sequence log-probs of the HIP path and of the oracle in bf16 and fp32
(HIP masks replayed), the per-pair margins and losses.  Then the same with the weights moved to the CPU and
regenerated there (synthetic_weights on a CPU generator), and with every weight cast through fp32 (bf16 values
either way).  Prints one JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from oracle import simpo_ref as O
    from ospo_amd.simpo import SimPOConfig, SimPOLossBuffers, simpo_forward
    from tests.test_gpu_step import _LazyMasks, _oracle_dims, _unpad

    torch.set_num_threads(16)
    dims, eng, batches, w = bench.simpo_setup(layers=int(os.environ.get("TRAJ_LAYERS", "2")))
    text, chosen, rejected = batches[0]
    B = chosen.shape[0]
    logps = eng.forward(text, chosen, rejected)
    buf = SimPOLossBuffers(B, "cuda")
    _, mean, _ = simpo_forward(logps, B, SimPOConfig(), buf)
    hip = logps.float().cpu()
    call, p, M = eng._drop_call, eng.lora_dropout, eng.M
    wc = {k: v.cpu() for k, v in w.items()}
    del eng, w
    torch.cuda.empty_cache()
    odims = O.JanusDims(**{**_oracle_dims(dims).__dict__, "lora_dropout": p})
    kin = {"qkv": dims.d_model, "o": dims.d_model, "gu": dims.d_model, "down": dims.d_ff}
    masks = _LazyMasks(M, kin, 42, call, p)
    tl, ch, rj = _unpad(text), chosen.cpu().long(), rejected.cpu().long()

    def case(name, ww, with_hip):
        out = {"case": name}
        for dt in (torch.bfloat16, torch.float32):
            o = O.simpo_step(tl, ch, rj, ww, odims, dtype=dt, backward=False, dropout_masks=masks)
            lp = torch.cat([o.chosen_logps, o.rejected_logps]).float()
            out[str(dt).split(".")[-1]] = {"loss": float(o.loss), "logps": [round(float(x), 6) for x in lp],
                                          "losses": [round(float(x), 5) for x in o.losses]}
        l16 = torch.tensor(out["bfloat16"]["logps"])
        l32 = torch.tensor(out["float32"]["logps"])
        out["logp_rel_bf16_vs_fp32"] = [round(float(x), 7) for x in ((l16 - l32) / l32.abs())]
        out["margin_bf16_vs_fp32"] = [round(float(10 * ((l16[i] - l16[B + i]) - (l32[i] - l32[B + i]))), 5)
                                      for i in range(B)]
        if with_hip:
            out["hip"] = {"loss": float(mean.item()), "logps": [round(float(x), 6) for x in hip]}
            out["logp_rel_hip_vs_fp32"] = [round(float(x), 7) for x in ((hip - l32) / l32.abs())]
        print(json.dumps(out), flush=True)

    case("device_weights", wc, True)
    from ospo_amd.engine import synthetic_weights
    wcpu = synthetic_weights(dims, "cpu", seed=0, lora_seed=1)
    case("cpu_generated_weights", wcpu, False)
    # where does the gap enter: the same device weights, with the LoRA B set to zero (frozen base only)
    wz = {k: (torch.zeros_like(v) if k.endswith(".lora_B") else v) for k, v in wc.items()}
    case("device_weights_lora_B_zero", wz, False)


if __name__ == "__main__":
    main()
