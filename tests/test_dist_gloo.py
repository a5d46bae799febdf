"""Data-parallel path on CPU: world_size 2 over gloo (127.0.0.1).

(1) GradAllReduce = mean of the per-rank flat buffers, bucketed.
(2) The reference's DP semantics: each rank takes half of the pairs, computes the
    SimPO LoRA gradient of its local mean loss; the all-reduced mean equals the
    single-process gradient over the union batch (oracle, fp32, tiny model)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import simpo_ref as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from ospo_amd import dist as odist
    odist.init(backend="gloo")
    try:
        # (1) bucketed all-reduce mean
        flat = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        odist.GradAllReduce(world, bucket_elems=128)(flat)
        exp = torch.arange(1000, dtype=torch.float32) * (1 + 2) / 2
        ok1 = torch.allclose(flat, exp)
        # (1b) the overlapped form: ranges pushed in reverse-layer order, merged into buckets
        ar = odist.GradAllReduce(world, bucket_elems=300)
        flat2 = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        ar.begin(flat2)
        for lo in range(900, -1, -100):  # ten "layers" of 100, last layer first
            ar.push(lo, lo + 100)
        ar.finish()
        ok1 = ok1 and torch.allclose(flat2, exp)
        # (2) DP SimPO grads == union-batch grads
        from tests import fixtures as FX
        from ospo_amd.lora import LoraLayout
        z = FX.load("step_tiny_fp32.npz")
        dims = FX.dims_of(z)
        text, chosen, rejected = FX.step_inputs(z)
        text = [t[:, :5] for t in text]  # equal prompt lengths: no cross-pair padding difference
        w = {k: v.float() for k, v in FX.step_weights(z, "step_tiny_fp32.npz", dims).items()}
        out = O.simpo_step([text[rank]], chosen[rank:rank + 1], rejected[rank:rank + 1], w, dims,
                           dtype=torch.float32)
        lay = LoraLayout(dims.n_layers, dims.d_model, dims.d_ff, dims.lora_r)
        g = torch.zeros(lay.numel)
        lay.to_flat(out.lora_grads, g)
        odist.GradAllReduce(world)(g)
        q.put((rank, ok1, g))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_dp_grads_equal_union_batch():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    g0, g1 = res[0][2], res[1][2]
    assert torch.equal(g0, g1)  # every rank holds the same averaged gradient
    from tests import fixtures as FX
    from ospo_amd.lora import LoraLayout
    z = FX.load("step_tiny_fp32.npz")
    dims = FX.dims_of(z)
    text, chosen, rejected = FX.step_inputs(z)
    text = [t[:, :5] for t in text]
    w = {k: v.float() for k, v in FX.step_weights(z, "step_tiny_fp32.npz", dims).items()}
    full = O.simpo_step(text, chosen, rejected, w, dims, dtype=torch.float32)
    lay = LoraLayout(dims.n_layers, dims.d_model, dims.d_ff, dims.lora_r)
    gf = torch.zeros(lay.numel)
    lay.to_flat(full.lora_grads, gf)
    assert float((g0 - gf).norm() / gf.norm()) < 1e-5
