"""Golden vectors for the learning-rate schedules of step 5, from the REFERENCE's own code (this container only).

Run:  python tests/golden/make_golden_sched.py        (needs /root/reference)

What runs is the reference's ``CosineDecayWarmUpRestarts`` (ospo/utils/train.py:119-148; the module is
exec'd with make_golden.py's stubs for the absent pytorch_lightning) and torch's ``ConstantLR`` as
``configure_optimizers`` builds them (ospo/wrapper/train.py:107-130): the optimizer's lr after
construction and after every ``scheduler.step()`` (PL calls it once per optimizer step, interval
"step"), for the warm-up ratios / lengths below, with and without an ``lr_scale`` param group.
Output: tests/golden/sched_golden.json (numbers only -- never reference source).
"""
from __future__ import annotations

import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (stubs + the reference module loader)

CASES = [  # (max_training_steps, warmup_ratio, init_lr, min_lr, steps, lr_scale)
    (100, 0.1, 1.5e-4, 1e-6, 110, None),
    (30, 0.05, 2e-5, 0.0, 35, None),
    (12, 0.0, 1e-4, 1e-5, 14, None),
    (40, 0.25, 3e-4, 3e-5, 45, 0.5),
]


def main():
    MG.install_stubs()
    ref = MG.load_ref_module("ref_utils_train", "ospo/utils/train.py")
    out = {"cosine": [], "constant": []}
    for max_steps, ratio, init_lr, min_lr, steps, lr_scale in CASES:
        p = torch.nn.Parameter(torch.zeros(2))
        group = {"params": [p]}
        if lr_scale is not None:
            group["lr_scale"] = lr_scale
        opt = torch.optim.AdamW([group], lr=init_lr)
        sch = ref.CosineDecayWarmUpRestarts(opt, warmup_iter=max_steps * ratio, max_iter=max_steps,
                                            eta_min=min_lr, eta_max=init_lr)
        lrs = [opt.param_groups[0]["lr"]]
        for _ in range(steps):
            opt.step()
            sch.step()
            lrs.append(opt.param_groups[0]["lr"])
        out["cosine"].append({"max_training_steps": max_steps, "warmup_ratio": ratio, "init_lr": init_lr,
                              "min_lr": min_lr, "lr_scale": lr_scale, "lrs": lrs})
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.AdamW([p], lr=2e-5)
    sch = torch.optim.lr_scheduler.ConstantLR(opt, factor=1.0, total_iters=20)
    lrs = [opt.param_groups[0]["lr"]]
    for _ in range(25):
        opt.step()
        sch.step()
        lrs.append(opt.param_groups[0]["lr"])
    out["constant"].append({"init_lr": 2e-5, "total_iters": 20, "lrs": lrs})
    with open(os.path.join(HERE, "sched_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote sched_golden.json:", {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
