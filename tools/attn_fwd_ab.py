"""Forward attention A/B at the step shape (S 8, T 600, 32 heads, d 128) on seeded inputs: the output and lse
are saved to gpurun_out/attn_fwd_<tag>.pt and the forward is timed (HIP events).  Run once per kernel
(OSPO_ATTN_FWD8=1 selects the round-1..3 8-wave kernel in the ablation build), then --compare A B."""
import os as _os
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import json
import math
import sys

import torch

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402

S, T, H, hd = 8, 600, 32, 128


def run(tag):
    torch.manual_seed(0)
    D = H * hd
    qkv = torch.randn(S * T, 3 * D, device="cuda").bfloat16()
    o = torch.empty(S * T, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(S * H * T, device="cuda")
    sc = 1 / math.sqrt(hd)
    fn = lambda: ops.flash_attn_fwd(qkv, 0, D, 2 * D, o, lse, S, T, H, hd, sc)  # noqa: E731
    ts = []
    for _ in range(5):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    os_dir = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "gpurun_out")
    _os.makedirs(os_dir, exist_ok=True)
    torch.save({"o": o.cpu(), "lse": lse.cpu()}, _os.path.join(os_dir, f"attn_fwd_{tag}.pt"))
    fl = 4 * S * H * hd * T * (T + 1) / 2
    t = sorted(ts)[2]
    print(json.dumps({"tag": tag, "fwd_us": round(t, 1), "tflops": round(fl / t / 1e6, 1)}), flush=True)


def compare(a, b):
    d = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "gpurun_out")
    x = torch.load(_os.path.join(d, f"attn_fwd_{a}.pt"), weights_only=True)
    y = torch.load(_os.path.join(d, f"attn_fwd_{b}.pt"), weights_only=True)
    print(json.dumps({"o_bit_equal": bool(torch.equal(x["o"], y["o"])),
                      "lse_bit_equal": bool(torch.equal(x["lse"], y["lse"])),
                      "o_max_abs": float((x["o"].float() - y["o"].float()).abs().max())}), flush=True)
    return torch.equal(x["o"], y["o"]) and torch.equal(x["lse"], y["lse"])


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])
