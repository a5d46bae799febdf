"""Profile target: a few eager (non-graph) decode steps of the 7B T2I sampler, after a warm-up
generate, so rocprofv3 --kernel-trace shows each kernel of the step separately."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd.engine import JANUS_PRO_7B, synthetic_weights  # noqa: E402
from ospo_amd.generate import T2IGenerator  # noqa: E402

dev = torch.device("cuda", 0)
dims = JANUS_PRO_7B
B, N, Lp = 16, 576, 48
w = synthetic_weights(dims, dev, seed=0, lora_seed=1)
gen = T2IGenerator(dims, w, device=dev, max_batch=B, max_prompt_len=Lp, n_img_tokens=N)
del w
g = torch.Generator().manual_seed(0)
prompts = [torch.randint(0, dims.vocab, (40,), generator=g).tolist() for _ in range(B)]
gen.generate(prompts, seed=0, use_graph=False)
gen.pos.fill_(Lp + N // 2)
gen.step.fill_(N)
for _ in range(int(os.environ.get("T2I_STEPS", "5"))):
    gen._decode_step(2 * B)
torch.cuda.synchronize()
print("done")
