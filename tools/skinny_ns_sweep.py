"""Ring depth x grid size of the forward's u products at the step shape (round 6): run once per OSPO_SK3_NS value
(the ablation build reads it once per process); inside, skinny variant 100 + W pins the target workgroup count.
ospo_lora_skinny with dropout + keep bits (the engine's call), nt = 3 (q|k|v) and 1 (o), M 4800, K 4096; medians of
3 x 20 launches, inputs alternated between two copies."""
import os as _os
import sys
_os.environ.setdefault("OSPO_HIP_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                     "ospo_amd", "libospo_hip_ablation.so"))
import json  # noqa: E402

import torch  # noqa: E402

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from ospo_amd import ops  # noqa: E402
from ospo_amd._lib import call  # noqa: E402

M, K = 4800, 4096


def timeit(f, it=20):
    for i in range(4):
        f(i & 1)
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(it):
            f(i & 1)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / it * 1e3)
    return sorted(ts)[1]


def main():
    torch.manual_seed(0)
    xs = [torch.randn(M, K, device="cuda").bfloat16() for _ in range(2)]
    bits = torch.empty(M * K // 8, dtype=torch.uint8, device="cuda")
    res = {}
    ref = {}
    for nt in (3, 1):
        bt = (torch.randn(16 * nt, K, device="cuda") * 0.05).bfloat16()
        # workspace for the largest split count (64 splits: counters + partials), zeroed once (the counter head
        # stays zero between calls)
        ws = torch.zeros(4096 // 4 + 64 * 4864 * 16 * nt + 16, dtype=torch.float32, device="cuda")
        o = torch.zeros(M, 64, device="cuda", dtype=torch.bfloat16)
        for w in (0, 768, 1024, 1536):
            call("ospo_set_skinny_variant", 100 + w if w else 4)
            f = lambda i: ops.lora_skinny(xs[i], bt, o, M, M, K, nt, 0, 2.0, b_rows=16 * nt, ws=ws,  # noqa: E731
                                          dropout=(12345, 0.05), keep_bits=bits)
            t = timeit(f)
            f(0)
            torch.cuda.synchronize()
            key = f"nt{nt}_wgs{w or 'default'}"
            res[key] = round(t, 1)
            ref.setdefault(nt, o.clone())
            res[key + "_same_as_default"] = bool(torch.equal(o, ref[nt]))
        call("ospo_set_skinny_variant", 4)
    print(json.dumps({"NS": _os.environ.get("OSPO_SK3_NS", "2"), "us": res}), flush=True)


if __name__ == "__main__":
    main()
