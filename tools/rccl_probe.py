"""RCCL (torch.distributed "nccl") probe on a ONE-GPU box: every rank binds cuda:0.

Launched as ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
--master-port P tools/rccl_probe.py``.  Checks, with real RCCL collectives, what the DP path
(ospo_amd/dist.py) issues per step: the bucketed GradAllReduce (plain and overlapped
begin/push/finish forms, with ranges pushed in reverse layer order as the backward does) and the
fused scalar all-reduce of the logged metrics.  Prints one JSON line from rank 0.

RCCL refuses two ranks on one device ("Duplicate GPU detected", measured on the 1-GPU box), so on
such a box run it with --nproc-per-node 1: RCCL then initialises and runs every collective of the
step on a one-rank communicator (GradAllReduce's buckets are issued directly, since the product
class skips the collective at world 1).
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import dist as odist  # noqa: E402


def main():
    world, rank, _ = odist.env_world()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.time()
    dist.init_process_group("nccl", device_id=dev)
    init_s = time.time() - t0
    out = {"world": world, "backend": dist.get_backend(), "init_s": round(init_s, 2)}
    n = 37_480_000  # flat LoRA grads at r = 16 (37.48 M params)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    flat = torch.randn(n, device=dev, generator=g)
    # expected average: regenerate every rank's buffer locally
    ref = torch.zeros(n, device=dev)
    for r in range(world):
        gr = torch.Generator(device=dev).manual_seed(1234 + r)
        ref += torch.randn(n, device=dev, generator=gr)
    ref /= world
    a = flat.clone()
    if world > 1:
        odist.GradAllReduce(world)(a)
    else:  # the same bucket calls on a one-rank RCCL communicator
        works = [dist.all_reduce(a[i:i + 16 * 1024 * 1024], async_op=True) for i in range(0, n, 16 * 1024 * 1024)]
        for w in works:
            w.wait()
    torch.cuda.synchronize()
    out["bucketed_max_err"] = (a - ref).abs().max().item()
    # overlapped form: 30 layer ranges pushed in reverse order on the current stream
    b = flat.clone()
    ar = odist.GradAllReduce(world)
    ar.begin(b)
    edges = [round(i * n / 30) for i in range(31)]
    for i in reversed(range(30)):
        ar.push(edges[i], edges[i + 1])
    ar.finish()
    torch.cuda.synchronize()
    out["overlapped_max_err"] = (b - ref).abs().max().item()
    s = torch.tensor([float(rank), 2.0 * rank, 1.0], device=dev)
    dist.all_reduce(s)
    s.mul_(1.0 / world)
    odist.broadcast_(flat[:16], 0)
    out["scalars"] = s.tolist()
    # timing of the per-step gradient all-reduce (150 MB fp32)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(5):
        odist.GradAllReduce(world)(flat)
    torch.cuda.synchronize()
    out["allreduce_ms"] = round((time.time() - t0) / 5 * 1e3, 2)
    ok = out["bucketed_max_err"] < 1e-5 and out["overlapped_max_err"] < 1e-5
    out["ok"] = ok
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
