"""Forward attention launches at the step shape (S 8, T 600, 32 heads, d 128) for a rocprofv3 --pmc pass: 20
launches of the ablation build's forward with OSPO_ATTN_FWD3_GM = argv[1] (band size of the workgroup order;
absent: the default), inputs alternated between two seeded sets.  tools/gpu/gpu_r06_attn_pmc.sh summarises."""
import os as _os
import sys

_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
if len(sys.argv) > 1 and sys.argv[1] != "default":
    _os.environ["OSPO_ATTN_FWD3_GM"] = sys.argv[1]
import math  # noqa: E402

import torch  # noqa: E402

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

S, T, H, hd = 8, 600, 32, 128
D = H * hd
g = torch.Generator(device="cuda").manual_seed(0)
qkv = [torch.randn(S * T, 3 * D, device="cuda", generator=g).bfloat16() for _ in range(2)]
o = [torch.empty(S * T, D, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
lse = [torch.empty(S * H * T, device="cuda") for _ in range(2)]
for i in range(20):
    ops.flash_attn_fwd(qkv[i & 1], 0, D, 2 * D, o[i & 1], lse[i & 1], S, T, H, hd, 1 / math.sqrt(hd))
torch.cuda.synchronize()
print("ok")
