"""Decode Linear split-count A/B (ablation library): per shape, cold weights (tools/dlin_warm_ab.py's rotation), the
split count of gemv3_kper pinned by ospo_set_gemv_splits (0 = the default rule) and the pipelined form on
(OSPO_DLIN_PIPE=1: wherever it fits) or off (0).  Prints one JSON line per (shape, splits, pipe)."""
import os as _os
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import json
import os
import subprocess
import sys

if os.environ.get("DLIN_CHILD") is None:  # one process per pipe setting (the knob is read once per process)
    for pipe in ("1", "0"):
        env = dict(os.environ, DLIN_CHILD="1", OSPO_DLIN_PIPE=pipe)
        r = subprocess.run([sys.executable, "-u", __file__], env=env)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

R = 32
SHAPES = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008)]
torch.manual_seed(0)
dev = "cuda"
x = (torch.randn(R, 11008, device=dev) * 0.5).bfloat16()
for name, N, K in SHAPES:
    wbytes = N * K * 2
    ncopy = max(2, -(-(1 << 30) // wbytes))
    ws_ = [ops.tile_decode_weight((torch.rand(N, K, device=dev) * 0.02 - 0.01).bfloat16()) for _ in range(ncopy)]
    out = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    xk = x[:, :K].contiguous()
    for sp in (0, 2, 4, 8, 16):
        if sp > K // 256:
            continue
        call("ospo_set_gemv_splits", sp)
        ws = ops.decode_linear_ws(R, N, K, dev)
        seq = list(range(4 * ncopy))
        for i in seq[:4]:
            ops.decode_linear(xk, ws_[i % ncopy], out, ws)
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in seq:
                ops.decode_linear(xk, ws_[i % ncopy], out, ws)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / len(seq) * 1e3)
        print(json.dumps({"shape": name, "splits": sp, "pipe": os.environ["OSPO_DLIN_PIPE"], "cold_us": round(min(ts), 2),
                          "TBps": round(wbytes / min(ts) / 1e6, 2)}), flush=True)
    call("ospo_set_gemv_splits", 0)
    del ws_
