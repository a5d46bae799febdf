import sys, torch; sys.path.insert(0, '.')
from oracle import simpo_ref as O
from tests.test_gpu_step import build_engine, run_hip_step, rel
torch.set_num_threads(16)
dims = O.JanusDims(n_layers=2)
w = O.init_weights(dims, seed=3, dtype=torch.bfloat16, lora_b_std=1e-2)
g = torch.Generator().manual_seed(9)
B = 2
text = [torch.randint(0, dims.vocab, (1, 24 - i), generator=g, dtype=torch.int32) for i in range(B)]
chosen = torch.randint(0, dims.img_vocab, (B, 576), generator=g)
rejected = torch.randint(0, dims.img_vocab, (B, 576), generator=g)
algo = {"beta": 10.0, "gamma_beta_ratio": 0.5, "label_smoothing": 0.0, "loss_type": "sigmoid"}
eng = build_engine(dims, w, B, 24, 576)
lp, loss, grads = run_hip_step(eng, text, chosen, rejected, algo)
ob = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.bfloat16)
of = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.float32)
lb = torch.cat([ob.chosen_logps, ob.rejected_logps]); lf = torch.cat([of.chosen_logps, of.rejected_logps])
print("logps hip ", lp.tolist()); print("logps bf16", lb.tolist()); print("logps fp32", lf.tolist())
print("abs err hip-fp32", (lp - lf).abs().max().item(), "oracle_bf16-fp32", (lb - lf).abs().max().item(), "hip-bf16", (lp-lb).abs().max().item())
print("loss hip", loss, "bf16", float(ob.loss), "fp32", float(of.loss))
print("grad rel hip-fp32", max(rel(grads[k], of.lora_grads[k]) for k in of.lora_grads), "bf16-fp32", max(rel(ob.lora_grads[k], of.lora_grads[k]) for k in of.lora_grads))
