"""The drop-in Trainer's data-parallel step on CPU (gloo, world 2): Trainer.fit overlaps the LoRA-grad all-reduce
with the backward (GradAllReduce.begin / push from the engine's layer hook / finish, as simpo.train_step does on the
timed path) and the result must be BIT-equal to the post-backward all-reduce of the same per-rank gradients
(VERDICT r5 item 7).  The engine is a stand-in with the HIP engine's backward contract: backward(g, on_layer_grads)
accumulates each layer's flat LoRA-gradient range, last layer first, and calls on_layer_grads(lo, hi) once that range
is final; the per-rank gradients are the oracle's SimPO LoRA grads of that rank's pair (fp32, tiny model)."""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Engine:
    """backward(g, on_layer_grads) as SimPOEngine.backward: grads += this rank's flat grads (scaled by the upstream
    gradient), layer by layer in reverse, each layer's range announced once final."""

    def __init__(self, flat, per_layer, n_layers):
        self.flat, self.per_layer, self.n_layers = flat, per_layer, n_layers
        self.grads = torch.zeros_like(flat)
        self.layer_grads_hook = None
        self.calls = 0

    def forward(self, text, chosen, rejected):
        return torch.zeros(2 * chosen.shape[0])

    def backward(self, g, on_layer_grads=None):
        self.calls += 1
        s = float(g.sum())
        for i in reversed(range(self.n_layers)):
            lo, hi = i * self.per_layer, (i + 1) * self.per_layer
            self.grads[lo:hi] += s * self.flat[lo:hi]
            if on_layer_grads is not None:
                on_layer_grads(lo, hi)


class _Opt:
    def __init__(self, eng):
        self.eng, self.seen = eng, []

    def step(self):
        self.seen.append(self.eng.grads.clone())

    def zero_grad(self):
        self.eng.grads.zero_()


class _Sched:
    def step(self):
        pass


class _Wrapper:
    def __init__(self, eng):
        self.engine, self.logged = eng, {}
        self.anchor = torch.zeros(1, requires_grad=True)
        self.opt = _Opt(eng)

    def setup(self, stage, log_dir):
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)

    def configure_optimizers(self):
        return [self.opt], [{"scheduler": _Sched()}]

    def training_step(self, batch, idx):
        from ospo_amd.simpo import PolicyLogps
        text, chosen, rejected = batch
        logps = PolicyLogps.apply(self.anchor, self.engine, text, chosen, rejected)
        return logps.sum() * 0.5  # d loss / d logps = 0.5 each: one backward adds 1.0 x the rank's grads

    def on_before_optimizer_step(self):
        pass


def _worker(rank, world, port, accum, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from oracle import simpo_ref as O
    from ospo_amd import dist as odist
    from ospo_amd.lora import LoraLayout
    from ospo_amd.trainer import Trainer
    from tests import fixtures as FX
    odist.init(backend="gloo")
    try:
        z = FX.load("step_tiny_fp32.npz")
        dims = FX.dims_of(z)
        text, chosen, rejected = FX.step_inputs(z)
        w = {k: v.float() for k, v in FX.step_weights(z, "step_tiny_fp32.npz", dims).items()}
        out = O.simpo_step([text[rank][:, :5]], chosen[rank:rank + 1], rejected[rank:rank + 1], w, dims,
                           dtype=torch.float32)
        lay = LoraLayout(dims.n_layers, dims.d_model, dims.d_ff, dims.lora_r)
        flat = torch.zeros(lay.numel)
        lay.to_flat(out.lora_grads, flat)
        assert lay.per_layer * dims.n_layers == lay.numel
        eng = _Engine(flat, lay.per_layer, dims.n_layers)
        wrapper = _Wrapper(eng)
        cfg = {"base": {"save_path": tmp, "exp_name": "dp"},
               "experiment": {"max_training_steps": 2, "gradient_accumulation_steps": accum,
                              "enable_checkpointing": False, "log_steps": 1}}
        tr = Trainer(cfg, world=world, rank=rank)
        # buckets smaller than a layer: the overlapped form issues several collectives per step
        tr.allreduce = odist.GradAllReduce(world, bucket_elems=max(1, lay.per_layer // 3))
        batch = (torch.zeros(1, 5, dtype=torch.int32), chosen[rank:rank + 1], rejected[rank:rank + 1])
        tr.fit(wrapper, [batch] * 4)
        # the post-backward form on the same per-rank gradients (accum micro-batches of flat / accum each: the loss
        # is divided by accum, so d loss / d logps sums to 1 / accum per micro-batch)
        ref = flat * 0.0
        for _ in range(accum):
            ref += (1.0 / accum) * flat
        odist.GradAllReduce(world)(ref)
        # numpy copies: pickled by value (a torch tensor's shared-memory fd dies with the worker that sent it)
        q.put((rank, [t.numpy().copy() for t in wrapper.opt.seen], ref.numpy().copy(), eng.calls))
    finally:
        dist.destroy_process_group()


def _run(accum):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as tmp:
        procs = [ctx.Process(target=_worker, args=(r, world, port, accum, tmp, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    return res


def test_trainer_fit_overlapped_allreduce_bit_equal_post_backward():
    for accum in (1, 2):
        res = _run(accum)
        for rank, seen, ref, calls in res:
            assert len(seen) == 2 and calls == 2 * accum
            for g in seen:  # every optimizer step saw exactly the post-backward all-reduced mean
                assert np.array_equal(g, ref), (accum, rank, float(np.abs(g - ref).max()))
        assert np.array_equal(res[0][1][0], res[1][1][0])  # and every rank the same
