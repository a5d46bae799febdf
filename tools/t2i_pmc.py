"""T2I decode traffic pass (run under rocprofv3 --pmc, one counter per pass; tools/gpu/gpu_r04_t2i_pmc.sh): the
bench's generator (Janus-Pro-7B shapes, 16 prompts x (cond, uncond), prompts <= 48 tokens, fused decode Linears)
sampling N_IMG tokens EAGERLY (no hipGraph: the counters are collected per dispatch), so the prefill plus N_IMG - 1
decode steps.  tools/t2i_pmc_summary.py turns the counter CSVs into measured / algorithmic HBM bytes of the
decode kernels."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ospo_amd.engine import JANUS_PRO_7B, synthetic_weights  # noqa: E402
from ospo_amd.generate import T2IGenerator  # noqa: E402

N_IMG = int(os.environ.get("T2I_PMC_TOKENS", "8"))
B, LP = 16, 48


def main():
    dev = torch.device("cuda", 0)
    dims = JANUS_PRO_7B
    w = synthetic_weights(dims, dev, seed=0, lora_seed=1)
    gen = T2IGenerator(dims, w, device=dev, max_batch=B, max_prompt_len=LP, n_img_tokens=N_IMG, cfg_weight=5.0,
                       temperature=1.0, vq_weights=None, fused_layers=True)
    del w
    torch.cuda.empty_cache()
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(0, dims.vocab, (int(torch.randint(LP // 2, LP + 1, (1,), generator=g)),),
                             generator=g).tolist() for _ in range(B)]
    toks, _, lp = gen._prompt_rows(prompts)
    tok = gen.generate(prompts, seed=0, use_graph=False)
    torch.cuda.synchronize()
    print({"n_img": N_IMG, "prompt_len": lp, "rows": 2 * B, "tokens_sum": int(tok.long().sum().item())}, flush=True)


if __name__ == "__main__":
    main()
