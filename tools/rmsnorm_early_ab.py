"""rmsnorm_bwd at the step shape (M 4800, D 4096, with the residual grad), ablation build: one process per form
(OSPO_RMS_EARLY is read once).  Prints the median of 3 x 20 launches (HIP events, inputs alternated between two
sets) and a checksum of the output for the bit-identity check across the two runs."""
import os as _os
import sys
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import hashlib  # noqa: E402
import json  # noqa: E402

import torch  # noqa: E402

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

M, D = 4800, 4096
g = torch.Generator(device="cuda").manual_seed(3)
dy = [torch.randn(M, D, device="cuda", generator=g).bfloat16() for _ in range(2)]
x = [torch.randn(M, D, device="cuda", generator=g).bfloat16() for _ in range(2)]
dres = [torch.randn(M, D, device="cuda", generator=g).bfloat16() for _ in range(2)]
w = (1 + 0.1 * torch.randn(D, device="cuda", generator=g)).bfloat16()
rstd = torch.rand(M, device="cuda", generator=g) + 0.5
dx = [torch.empty(M, D, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
f = lambda i: ops.rmsnorm_bwd(dy[i], x[i], w, rstd, dx[i], dres=dres[i])  # noqa: E731
for i in range(10):
    f(i & 1)
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(20):
        f(i & 1)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 20 * 1e3)
f(0)
torch.cuda.synchronize()
print(json.dumps({"early": _os.environ.get("OSPO_RMS_EARLY", "0"), "us": round(sorted(ts)[1], 2),
                  "GBps": round(4 * M * D * 2 / sorted(ts)[1] / 1e3, 0),
                  "sha": hashlib.sha1(dx[0].view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]}), flush=True)
