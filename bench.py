"""Throughput of the Janus-Pro-7B SimPO training step on MI355X (BASELINE.json metric).

python bench.py [--gpus N --steps K --warmup W]    (N>1: launched by torch.distributed.run)

A step = forward of 2B sequences (chosen | rejected, T = 24 text + 576 image
tokens) through the LoRA'd Janus-Pro-7B LLM and gen_head, SimPO loss, backward
to the LoRA adapters, RCCL all-reduce of the LoRA grads (N>1), clip + AdamW.
Synthetic data (random-init weights of the 7B architecture, random prompt and
VQ ids; there is no checkpoint or dataset offline).  Prints ONE JSON line on
rank 0.  See DESIGN.md "Measurement".
"""
from __future__ import annotations

import argparse
import contextlib
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_FP8_TFLOPS = 5000.0   # MI355X dense fp8 (MX-scaled e4m3) MFMA, same table
METRIC = "preference-pairs/sec (whole node), Janus-Pro-7B SimPO @576 img tokens, 1/2/4/8 GPU"


def algorithmic_flops_per_pair(T=600, N=576, L=30, D=4096, F=11008, r=16, Dg=4096, V=16384, A_in=8):
    """fwd + bwd (activation grads + LoRA grads), no recompute, no text lm_head."""
    p_lin = L * (4 * D * D + 3 * D * F)
    p_lora = L * r * (4 * (D + D) + 2 * (D + F) + (F + D))
    p_gh = D * Dg + Dg * V
    p_al = A_in * D + D * D
    attn_f = 2 * L * D * T * (T + 1)  # causal QK^T + PV
    fwd = 2 * T * p_lin + attn_f + 2 * T * p_lora + 2 * N * p_gh + 2 * N * p_al
    bwd = 2 * T * p_lin + 2 * attn_f + 4 * T * p_lora + 2 * N * p_gh
    return 2 * (fwd + bwd)  # two sequences per pair


def synthetic_batch(B, Lt, N, vocab, img_vocab, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    lens = torch.randint(Lt // 2, Lt + 1, (B,), generator=g)
    lens[0] = Lt
    text = torch.full((B, Lt), -1, dtype=torch.int32)
    for i in range(B):
        text[i, : lens[i]] = torch.randint(0, vocab, (int(lens[i]),), generator=g, dtype=torch.int32)
    chosen = torch.randint(0, img_vocab, (B, N), generator=g, dtype=torch.int32)
    rejected = torch.randint(0, img_vocab, (B, N), generator=g, dtype=torch.int32)
    return text.to(device), chosen.to(device), rejected.to(device)


def cpu_baseline(Lt=24, N=576):
    """The CPU oracle (oracle/simpo_ref.py, bf16 CPU path) on a bounded sample:
    one pair, full 7B shapes, fwd+bwd with 1 and with 2 decoder layers;
    t_layer = t2 - t1, t_head = t1 - t_layer, per-pair = t_head + 30 * t_layer."""
    from oracle import simpo_ref as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    text = [torch.randint(0, 4096, (1, Lt), generator=g, dtype=torch.int32)]
    ch = torch.randint(0, 16384, (1, N), generator=g)
    rj = torch.randint(0, 16384, (1, N), generator=g)
    times = {}
    for L in (1, 2):
        dims = O.JanusDims(n_layers=L, vocab=4096)
        w = O.init_weights(dims, seed=1, dtype=torch.bfloat16)
        t0 = time.perf_counter()
        O.simpo_step(text, ch, rj, w, dims, dtype=torch.bfloat16)
        times[L] = time.perf_counter() - t0
        del w
    t_layer = max(times[2] - times[1], 1e-6)
    t_head = max(times[1] - t_layer, 0.0)
    t_pair = t_head + 30 * t_layer
    return {"value": round(1.0 / t_pair, 5), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"1 pair (T={Lt + N}), oracle bf16 fwd+bwd with 1 and 2 full-size 7B decoder layers "
                      f"({times[1]:.1f}s, {times[2]:.1f}s): t_layer {t_layer:.2f}s, head+loss {t_head:.2f}s, "
                      f"scaled to 30 layers = {t_pair:.1f}s/pair"}


def t2i_bytes_per_step(dims, R, T_keys):
    """Algorithmic HBM bytes of one decode step: every weight once (decoder
    Linears, gen_head, aligner W2; bf16), the KV cache read by attention (K and V of T_keys
    positions per row, layer and head), the new K/V written, activations negligible."""
    D, Fd, L, H = dims.d_model, dims.d_ff, dims.n_layers, dims.n_heads
    w = L * (4 * D * D + 3 * D * Fd) + D * dims.gen_head_dim + dims.gen_head_dim * dims.img_vocab + D * D
    kv = L * R * H * 128 * 2 * (T_keys + 1)
    return 2.0 * (w + kv)


def bench_t2i(args):
    """BASELINE config 4: step-3 AR T2I sampling, Janus-Pro-7B, 576 tokens, cfg 5, parallel_size 16
    (32 cond/uncond rows), hipGraph-captured decode.  One 'step' = one generate() call."""
    from ospo_amd.engine import JANUS_PRO_7B, synthetic_weights
    from ospo_amd.generate import T2IGenerator
    dev = torch.device("cuda", 0)
    dims = JANUS_PRO_7B.__class__(**{**JANUS_PRO_7B.__dict__, "n_layers": args.layers})
    B, N, Lp = args.t2i_batch, args.img_tokens, args.t2i_prompt_len
    w = synthetic_weights(dims, dev, seed=0, lora_seed=1)
    gen = T2IGenerator(dims, w, device=dev, max_batch=B, max_prompt_len=Lp, n_img_tokens=N, cfg_weight=5.0,
                       temperature=1.0)
    del w
    torch.cuda.empty_cache()
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(0, dims.vocab, (int(torch.randint(Lp // 2, Lp + 1, (1,), generator=g)),),
                             generator=g).tolist() for _ in range(B)]
    for i in range(args.warmup):
        gen.generate(prompts, seed=i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        tok = gen.generate(prompts, seed=100 + i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # decode-step roofline: graph replays of one step timed with HIP events on the replay stream
    R = 2 * B
    gen.pos.fill_(Lp + N // 2)
    gen.step.fill_(N)  # past the last token: the sampler writes nothing, the rest runs as usual
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record(st)
    for _ in range(reps):
        gen._graph.replay()
    e1.record(st)
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / reps
    nbytes = t2i_bytes_per_step(dims, R, Lp + N // 2 + reps // 2)
    achieved = nbytes / (step_ms * 1e-3) / 1e9
    value = B * args.steps / dt
    line = {
        "metric": "images/sec, Janus-Pro-7B step-3 T2I sampling (576 tokens, cfg 5, parallel_size 16)",
        "value": round(value, 3), "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 1), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random-init Janus-Pro-7B weights, random prompt ids)",
        "config": {"workload": f"Janus-Pro-{'7B' if dims.n_layers == 30 else str(dims.n_layers) + 'L'} T2I sampling, "
                               f"{B} prompts x (cond, uncond), {N} image tokens, hipGraph decode step",
                   "prompt_len_max": Lp, "decode_steps": N - 1, "tokens_per_s": round(value * N, 1)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(achieved / 8000.0, 4), "traffic": None,
                     "kernel": "decode step (hipGraph: 30 x (4 decode_gemv + attn_cache + norms) + gen_head + sampler)",
                     "algorithmic_bytes_per_step": round(nbytes), "avg_step_us": round(step_ms * 1e3, 1)},
        "tokens_checksum": int(tok.long().sum().item()),
    }
    print(json.dumps(line), flush=True)


def vq_flops_per_image(H=384, W=384):
    """Algorithmic FLOPs of the VQ-16 encoder + quant_conv on one H x W image: every convolution
    2 * Ho * Wo * Cout * Cin * KH * KW, the AttnBlock products 2 * 2 * n^2 * C (n = tokens)."""
    ch, mult = 128, (1, 1, 2, 2, 4)
    h, w = H, W
    f = 2 * h * w * ch * 3 * 9  # conv_in
    cin = ch
    for i, m in enumerate(mult):
        cout = ch * m
        for j in range(2):
            f += 2 * h * w * cout * cin * 9 + 2 * h * w * cout * cout * 9
            if cin != cout:
                f += 2 * h * w * cout * cin
            cin = cout
            if i == len(mult) - 1:
                f += 4 * 2 * h * w * cin * cin + 4 * (h * w) ** 2 * cin
        if i != len(mult) - 1:
            h, w = h // 2, w // 2
            f += 2 * h * w * cin * cin * 9
    f += 2 * (2 * h * w * cin * cin * 9) * 2 + 4 * 2 * h * w * cin * cin + 4 * (h * w) ** 2 * cin  # mid
    f += 2 * h * w * 256 * cin * 9 + 2 * h * w * 8 * 256  # conv_out, quant_conv
    return f


def bench_vq(args):
    """VQ-16 image tokenizer (gen_vision_model.encode), fp32, 384 px, a batch of
    images per call; value = images/s.  Roofline: f32 MFMA (157.3 TF dense, MI355X_MICROARCH.md)."""
    from ospo_amd.vq import VQEncoder, synthetic_vq_weights
    dev = torch.device("cuda", 0)
    w = synthetic_vq_weights(0)
    enc = VQEncoder(w, device=dev)
    B = args.vq_batch
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(B, 3, 384, 384, generator=g) * 2 - 1).to(dev)
    for _ in range(args.warmup):
        enc.encode(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ids = enc.encode(x)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    value = B * args.steps / dt
    fl = vq_flops_per_image()
    achieved = value * fl / 1e12
    line = {
        "metric": "images/sec, Janus-Pro VQ-16 tokenizer encode (384 px -> 576 ids), fp32",
        "value": round(value, 2), "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded VQ-16 weights, random pixels)",
        "config": {"workload": f"VQ-16 encode + quantize, {B} images of 384x384 per call",
                   "algorithmic_gflop_per_image": round(fl / 1e9, 1)},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 1), "peak": 157.3, "unit": "TFLOP/s",
                     "frac": round(achieved / 157.3, 4), "traffic": None,
                     "kernel": "whole encode (conv_f32_kernel implicit GEMM on v_mfma_f32_32x32x2_f32 dominates)"},
        "ids_checksum": int(ids.long().sum().item()),
    }
    if not args.no_cpu_baseline:
        from oracle import vq_ref as V
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
        t0 = time.perf_counter()
        V.encode_ref(x[:1].cpu(), w)
        tc = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": round(1.0 / tc, 4), "unit": "images/s", "cores": torch.get_num_threads(),
                                "kind": "port", "sample": f"1 image, oracle/vq_ref.py encode_ref fp32 ({tc:.2f} s)"}
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs-per-gpu", type=int, default=4)
    ap.add_argument("--text-len", type=int, default=24)
    ap.add_argument("--img-tokens", type=int, default=576)
    ap.add_argument("--layers", type=int, default=30)
    ap.add_argument("--lora-r", type=int, default=16)
    # dropout 0 for parity runs, configs/peft/lora.yaml's 0.05 for throughput
    ap.add_argument("--lora-dropout", type=float, default=0.05)
    # BASELINE config 5: the frozen decoder Linears on MXFP8 block-scaled fp8 MFMA (use with --lora-r 32)
    ap.add_argument("--linear-dtype", choices=("bf16", "mx8"), default="bf16")
    ap.add_argument("--workload", choices=("simpo", "t2i", "vq"), default="simpo")  # t2i: config 4; vq: §8f-3
    ap.add_argument("--vq-batch", type=int, default=16)
    ap.add_argument("--t2i-batch", type=int, default=16)       # parallel_size: prompts (x2 rows with CFG)
    ap.add_argument("--t2i-prompt-len", type=int, default=48)  # max prompt tokens (left-padded)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timer", action="store_true")
    args = ap.parse_args()
    if args.workload == "t2i":
        return bench_t2i(args)
    if args.workload == "vq":
        return bench_vq(args)

    from ospo_amd import dist as odist
    from ospo_amd import ops
    from ospo_amd.engine import JANUS_PRO_7B, SimPOEngine, synthetic_weights
    from ospo_amd.simpo import SimPOConfig, SimPOLossBuffers, train_step

    world, rank, local = odist.init()
    dev = torch.device("cuda", local)
    dims = JANUS_PRO_7B.__class__(**{**JANUS_PRO_7B.__dict__, "n_layers": args.layers, "lora_r": args.lora_r,
                                     "lora_alpha": 2 * args.lora_r})
    B, Lt, N = args.pairs_per_gpu, args.text_len, args.img_tokens
    weights = synthetic_weights(dims, dev, seed=0, lora_seed=1)  # identical on every rank (same seeds)
    eng = SimPOEngine(dims, weights, device=dev, max_pairs=B, max_text_len=Lt, n_img_tokens=N,
                      lora_dropout=args.lora_dropout, dropout_seed=42, linear_dtype=args.linear_dtype)
    del weights
    torch.cuda.empty_cache()
    cfg = SimPOConfig()
    buf = SimPOLossBuffers(B, dev)
    allreduce = odist.GradAllReduce(world) if world > 1 else None
    batches = [synthetic_batch(B, Lt, N, dims.vocab, dims.img_vocab, seed=1000 * rank + i, device=dev)
               for i in range(4)]

    # OSPO_MAIN_PRIO < 0 (A/B knob): the step's main stream is a high-priority HIP stream, so its GEMMs
    # are dispatched ahead of the side stream's LoRA dA/dB products
    prio = int(os.environ.get("OSPO_MAIN_PRIO", "0"))
    hp = torch.cuda.Stream(device=dev, priority=prio) if prio else None
    if hp is not None:
        hp.wait_stream(torch.cuda.current_stream(dev))
    stream_ctx = torch.cuda.stream(hp) if hp is not None else contextlib.nullcontext()
    stream_ctx.__enter__()
    for i in range(args.warmup):
        train_step(eng, *batches[i % 4], cfg, buf, allreduce=allreduce)
    timer = None if args.no_kernel_timer else ops.KernelTimer()
    odist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - 1:
            # per-launch HIP events on the last timed step only: an event pair around every GEMM
            # costs ~1 % of the step (128.8 vs 127.5 ms), so recording them on all K steps would
            # depress `value`; one step holds ~245 GEMM launches, enough for the average
            ops.set_kernel_timer(timer)
        out = train_step(eng, *batches[i % 4], cfg, buf, allreduce=allreduce)
    odist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stream_ctx.__exit__(None, None, None)
    ops.set_kernel_timer(None)
    loss = float(out["loss"].item())
    if not math.isfinite(loss):
        raise RuntimeError(f"non-finite loss {loss}")
    t = torch.tensor([dt], device=dev)
    if world > 1:
        import torch.distributed as tdist
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    dt = float(t.item())
    if rank != 0:
        return
    global_batch = B * world
    value = global_batch * args.steps / dt
    ms = dt / args.steps * 1e3
    T = Lt + N
    flops_pair = algorithmic_flops_per_pair(T=T, N=N, L=dims.n_layers, r=dims.lora_r)
    roof = None
    kern = {}
    if timer is not None:
        kern = timer.summary()
        dom = max(kern, key=lambda k: kern[k]["ms"])
        d = kern[dom]
        achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "gemm_pmc.json")
        if os.path.exists(pmc):
            traffic = json.load(open(pmc)).get(dom, {}).get("hbm_bytes_per_launch")
        mx = dom.startswith("gemm_nt_mx8")
        peak = PEAK_FP8_TFLOPS if mx else PEAK_BF16_TFLOPS
        roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "traffic_note": "HBM+Infinity-Cache bytes per launch (2*FETCH_SIZE+WRITE_SIZE, profiles/gemm_pmc.json)",
                "algorithmic_bytes_per_launch": round(d["bytes"] / d["count"]),
                "kernel": f"{dom} (gemm_nt_v5_kernel SP-schedule MFMA {'MXFP8 e4m3' if mx else 'bf16'} + split-K fixup)",
                "launches": d["count"],
                "avg_launch_us": round(d["ms"] * 1e3 / d["count"], 2),
                "step_mfma_frac": round(flops_pair * value / world / 1e12 / PEAK_BF16_TFLOPS, 4)}
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16" if args.linear_dtype == "bf16" else "mxfp8-e4m3 linears, bf16 rest",
        "data": "synthetic (random-init Janus-Pro-7B-shaped weights, random prompt/VQ token ids)",
        "config": {"workload": f"Janus-Pro-{'7B' if dims.n_layers == 30 else str(dims.n_layers) + 'L'} SimPO "
                               f"train step, LoRA r={dims.lora_r} dropout {args.lora_dropout}, {N} image tokens, "
                               f"{B} pairs/GPU" + (", MXFP8 decoder Linears (config 5)" if args.linear_dtype == "mx8" else ""),
                   "lora_dropout": args.lora_dropout, "linear_dtype": args.linear_dtype,
                   "global_batch": global_batch, "seq_len": T, "parallelism": f"dp{world}",
                   "algorithmic_tflop_per_pair": round(flops_pair / 1e12, 3)},
        "roofline": roof,
        "loss": round(loss, 5),
        "gemm_kernels": {k: {"count": v["count"], "ms": round(v["ms"], 2),
                             "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)} for k, v in kern.items()},
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(Lt=Lt, N=N)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
