"""Step-3 text-to-image sampling on the MI355X (BASELINE config 4).

The loop of ``ospo/wrapper/image_generation.py:109-171`` (``JanusProImageGenWrapper.generate_image``;
the same loop is ``ospo/inference.py:110-163``), run over a KV cache:

* the B prompts are left-padded with ``pad_id`` to one length Lp; row 2b is prompt b, row 2b+1 its
  unconditional copy with every token but the first and the last replaced by ``pad_id``
  (image_generation.py:132-141); padding is an attention mask, positions run 0..T-1 through it
  (HF 4.38 ``LlamaModel`` builds position ids from ``past_key_values_length`` only);
* step 0 is the prompt (prefill), steps 1..n-1 one token each; every step takes gen_head on the last
  position, ``logits = uncond + cfg_weight * (cond - uncond)``, ``softmax(logits / temperature)`` and
  samples one VQ id per image (:156-165), which ``prepare_gen_img_embeds`` turns into the next
  input for both rows of the pair (:166-169).

MI355X-first structure: the prefill reuses the training kernels (256x256 MFMA GEMM with the RoPE
epilogue, RMSNorm, SwiGLU); each decode step is weight streaming (``ospo_decode_gemv``) plus cached
attention (``ospo_attn_cache``); every step-dependent value is a device counter, so one decode step is
captured as a hipGraph (``torch.cuda.CUDAGraph`` over the HIP launches) and replayed n-1 times.
Sampling: inverse CDF on the bf16 probabilities with a seeded uniform per image and step
(``ospo_cfg_sample``) -- the distribution ``torch.multinomial`` draws from, with a generator whose
draws the oracle can replay.  ``generate`` returns the image-token ids; ``generate_images`` adds the
VQ pixel decoder (``decode_code``, image_generation.py:174) and the uint8 conversion of :175-181, so a
batch of prompts becomes the [B, 384, 384, 3] images step 3 saves.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch

from . import ops
from .engine import ModelDims

BF16 = torch.bfloat16
PAD_ID = 100015  # "<｜▁pad▁｜>" of the Janus-Pro tokenizer (VLChatProcessor.pad_id)


def _dev(t, device):
    return t.to(device=device, dtype=BF16).contiguous()


class T2IGenerator:
    """Device-resident Janus-Pro sampler (one per GPU).  ``weights``: the names of
    ``engine.synthetic_weights`` / ``oracle.simpo_ref.init_weights``; LoRA A/B present in them are
    merged (W + s B A, as ``inference.py`` merges the trained adapter before sampling)."""

    def __init__(self, dims: ModelDims, weights: Dict[str, torch.Tensor], device="cuda", max_batch: int = 16,
                 max_prompt_len: int = 64, n_img_tokens: int = 576, cfg_weight: float = 5.0,
                 temperature: float = 1.0, pad_id: int = PAD_ID, vq_weights: Optional[Dict[str, torch.Tensor]] = None,
                 tiled_weights: bool = True, fused_layers: bool = True, mlp_one_launch: bool = True,
                 head_split: bool = False, attn_o_one_launch: bool = False):
        if dims.head_dim != 128:
            raise ValueError("head_dim must be 128 (Janus-Pro)")
        if 2 * max_batch > 64:
            raise ValueError("at most 32 prompts per batch (64 cond/uncond rows)")
        if not temperature > 0:
            raise ValueError("temperature must be > 0")
        self.dims, self.device = dims, torch.device(device)
        self.cfg_weight, self.temperature, self.pad_id = float(cfg_weight), float(temperature), int(pad_id)
        self.n_img = n_img_tokens
        D, Fd, L, H = dims.d_model, dims.d_ff, dims.n_layers, dims.n_heads
        dev, w = self.device, weights
        s = dims.lora_scale

        def merged(name):
            W = w[name].to(device=dev, dtype=torch.float32)
            A, B = w.get(name + ".lora_A"), w.get(name + ".lora_B")
            if A is not None and B is not None:
                W = W + s * (B.to(dev, torch.float32) @ A.to(dev, torch.float32))
            return W.to(BF16)

        self.embed = _dev(w["embed_tokens"], dev)
        self.layers = []
        for i in range(L):
            p = f"layers.{i}."
            self.layers.append({
                "ln_in": _dev(w[p + "input_layernorm"], dev), "ln_post": _dev(w[p + "post_attention_layernorm"], dev),
                "qkv": torch.cat([merged(p + "q_proj"), merged(p + "k_proj"), merged(p + "v_proj")], 0).contiguous(),
                "o": merged(p + "o_proj").contiguous(),
                "gu": torch.cat([merged(p + "gate_proj"), merged(p + "up_proj")], 0).contiguous(),
                "down": merged(p + "down_proj").contiguous(),
            })
        self.norm = _dev(w["norm"], dev)
        self.gh_w1, self.gh_b1 = _dev(w["gen_head.w1"], dev), _dev(w["gen_head.b1"], dev)
        self.gh_w2, self.gh_b2 = _dev(w["gen_head.w2"], dev), _dev(w["gen_head.b2"], dev)
        self.al_w1, self.al_b1 = _dev(w["gen_aligner.w1"], dev), _dev(w["gen_aligner.b1"], dev)
        self.al_w2, self.al_b2 = _dev(w["gen_aligner.w2"], dev), _dev(w["gen_aligner.b2"], dev)
        self.gen_embed = _dev(w["gen_embed"], dev)
        # decode-step copies of the weight streams in the MFMA-tiled layout (ops.tile_decode_weight: every
        # fragment load reads whole 128-B lines; bit-identical results).  The prefill keeps the row-major
        # weights (256x256 GEMM).  Needs R = 2 max_batch <= 32 and N % 128 == 0, else row-major.
        self.tiled = bool(tiled_weights) and 2 * max_batch <= 32

        def dw(t):
            return ops.tile_decode_weight(t) if self.tiled and t.shape[0] % 128 == 0 and t.shape[1] % 32 == 0 else t

        # one launch per Linear (ops.decode_linear, round 3): the RMSNorms folded into the q|k|v and gate|up
        # stagings, split sums and consumers in the launch; needs every decode weight tiled (N % 128)
        Dg, Fa = dims.gen_head_dim, self.al_w2.shape[1]
        # (the folded RMSNorm reads one sum-of-squares partial per 128 input columns, <= 32 of them: D, Dg <= 4096;
        # the in-launch split sums keep one counter per 128 output rows, <= 1024 of them)
        self.fused = (bool(fused_layers) and self.tiled and all(n % 128 == 0 for n in (D, 3 * D, 2 * Fd, Dg))
                      and dims.img_vocab % 128 == 0 and all(k % 32 == 0 for k in (D, Fd, Dg, Fa))
                      and D // 128 <= 32 and Dg // 128 <= 32
                      and all(n // 128 <= 1024 for n in (3 * D, 2 * Fd, D, Dg, dims.img_vocab)))
        # the attention of one half of the heads overlapped with the q|k|v projection of the other half (round 5):
        # head-major q|k|v rows, two head-range launches, the second half on a side stream of the same graph
        self.head_split = bool(head_split) and self.fused and dims.n_heads % 2 == 0
        for lw in self.layers:
            for k in ("qkv", "o", "gu", "down"):
                src = ops.interleave_gate_up(lw[k]) if (k == "gu" and self.fused) else lw[k]
                if k == "qkv" and self.head_split:
                    src = ops.head_major_qkv(lw[k], dims.n_heads)
                lw[k + "_d"] = dw(src)
        self.gh_w1_d, self.gh_w2_d, self.al_w2_d = dw(self.gh_w1), dw(self.gh_w2), dw(self.al_w2)
        # ---- KV cache and decode-step buffers (R = 2 * max_batch rows)
        self.max_batch, self.max_prompt = max_batch, max_prompt_len
        self.Tmax = max_prompt_len + n_img_tokens
        R = 2 * max_batch
        z = lambda *sh, dt=BF16: torch.zeros(*sh, dtype=dt, device=dev)  # noqa: E731
        self.kc = [z(R, H, self.Tmax, 128) for _ in range(L)]
        self.vc = [z(R, H, self.Tmax, 128) for _ in range(L)]
        V, Dg = dims.img_vocab, dims.gen_head_dim
        self.x, self.xn, self.qkv, self.q = z(R, D), z(R, D), z(R, 3 * D), z(R, D)
        self.attn, self.xmid, self.xn2 = z(R, D), z(R, D), z(R, D)
        self.gu, self.h, self.xo = z(R, 2 * Fd), z(R, Fd), z(R, D)
        self.hf, self.zg, self.logits, self.e1 = z(R, D), z(R, Dg), z(R, V), z(R, D)
        self.rstd = z(R, dt=torch.float32)
        self.next_ids = torch.zeros(R, dtype=torch.int32, device=dev)
        self.start = torch.zeros(R, dtype=torch.int32, device=dev)
        self.pos = torch.zeros(1, dtype=torch.int32, device=dev)
        self.step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tokens = torch.zeros(max_batch, n_img_tokens, dtype=torch.int32, device=dev)
        self.u = torch.zeros(n_img_tokens * max_batch, dtype=torch.float32, device=dev)  # [n, B] of this batch
        shapes = [(3 * D, D), (D, D), (2 * Fd, D), (D, Fd), (Dg, D), (V, Dg), (D, D)]
        self.gws = torch.zeros(max(ops.query("ospo_decode_gemv_ws_bytes", R, n, k) for n, k in shapes) // 4 + 4,
                               dtype=torch.float32, device=dev)
        self.cos, self.sin = ops.rope_tables(self.Tmax, 128, dims.rope_theta, dev)
        if self.fused:
            self.lws = torch.zeros(max(ops.query("ospo_decode_linear_ws_bytes", R, n, k) for n, k in shapes) // 4 + 4,
                                   dtype=torch.float32, device=dev)
            # row sums of squares of the residual stream for the folded RMSNorms: [D / 128, 32] per buffer
            # (x, xo: the layer stack ping-pongs them; xmid)
            self.ss_x, self.ss_xo, self.ss_mid = (torch.zeros(D // 128, 32, dtype=torch.float32, device=dev)
                                                  for _ in range(3))
        # the decode MLP in one launch (ops.decode_mlp, round 5): per gate|up row group an h-ready flag tagged
        # with (step, layer), zeroed before every generate(); tmo: nonzero if a down workgroup's wait gave up
        self.mlp_one_launch = bool(mlp_one_launch) and self.fused and dims.n_layers < 63
        self.mlp_flags = torch.zeros(max(2 * Fd // 128, 1), dtype=torch.int32, device=dev)
        self.mlp_tmo = torch.zeros(1, dtype=torch.int32, device=dev)
        self._side = torch.cuda.Stream(device=dev) if self.head_split else None
        # the cached attention and o in one launch (ops.decode_attn_o, round 5; an A/B option, measured 1.6-2.7 %
        # slower than the two launches): a flag and a ticket per head, the same epochs; tmo shared with the MLP's waits
        self.attn_o_one_launch = (bool(attn_o_one_launch) and self.fused and not self.head_split
                                  and dims.n_layers < 63)
        self.attn_o_used = False  # (set when a decode step took the one-launch form: its shapes fit)
        self.mlp_used = False  # (set when a decode step ran the MLP as one launch: ops.decode_mlp took the shape)
        self.attn_flags = torch.zeros(2 * dims.n_heads, dtype=torch.int32, device=dev)
        self._graph = None
        self._graph_B = None
        self.probs = None  # [n, B, V] fp32 when record_probs
        # gen_vision_model's pixel decoder (VQ-16 weights: post_quant_conv.*, decoder.*, quantize.*)
        self.vq_decoder = None
        if vq_weights is not None:
            from .vq import VQDecoder
            self.vq_decoder = VQDecoder(vq_weights, device=dev)

    # ------------------------------------------------------------------ prefill
    def _prompt_rows(self, prompts: Sequence[Sequence[int]]):
        """Token matrix [2B, Lp] and pad lengths exactly as image_generation.py:124-141."""
        B = len(prompts)
        Lp = max(len(p) for p in prompts)
        toks = torch.full((2 * B, Lp), self.pad_id, dtype=torch.int32)
        start = torch.zeros(2 * B, dtype=torch.int32)
        for i in range(2 * B):
            ids = torch.tensor(list(prompts[i // 2]), dtype=torch.int32)
            pad = Lp - ids.numel()
            toks[i, pad:] = ids
            start[i] = pad
            if i % 2 != 0:
                toks[i, pad + 1: Lp - 1] = self.pad_id
        return toks, start, Lp

    def _prefill(self, toks: torch.Tensor, Lp: int):
        dims, dev = self.dims, self.device
        D, Fd, H = dims.d_model, dims.d_ff, dims.n_heads
        R = toks.shape[0]
        M = R * Lp
        ids = toks.reshape(-1).to(dev)
        z = lambda *sh, dt=BF16: torch.empty(*sh, dtype=dt, device=dev)  # noqa: E731
        x, xn, qkv, attn = z(M, D), z(M, D), z(M, 3 * D), z(M, D)
        xmid, gu, h, rstd = z(M, D), z(M, 2 * Fd), z(M, Fd), z(M, dt=torch.float32)
        ops.embed_rows(ids, self.embed, x)
        cos, sin = self.cos[:Lp].contiguous(), self.sin[:Lp].contiguous()
        scale = 1.0 / math.sqrt(128)
        for i, lw in enumerate(self.layers):
            ops.rmsnorm_fwd(x, lw["ln_in"], xn, rstd, dims.rms_eps)
            if (3 * D) % 256 == 0:  # q|k RoPE in the projection epilogue; position = row % Lp
                ops.gemm_nt(xn, lw["qkv"], qkv, rope=(cos, sin, Lp, 2 * D))
            else:
                ops.gemm_nt(xn, lw["qkv"], qkv)
                ops.rope(qkv, 0, D, R, Lp, H, 128, cos, sin)
            ops.kv_store(qkv, R, Lp, None, self.kc[i], self.vc[i], H, self.Tmax)
            ops.attn_cache(qkv, self.kc[i], self.vc[i], R, Lp, H, self.Tmax, self.start, None, scale, attn)
            ops.gemm_nt(attn, lw["o"], xmid, residual=x)
            ops.rmsnorm_fwd(xmid, lw["ln_post"], xn, rstd, dims.rms_eps)
            ops.gemm_nt(xn, lw["gu"], gu)
            ops.swiglu_fwd(gu, h)
            ops.gemm_nt(h, lw["down"], x, residual=xmid)
        last = x.view(R, Lp, D)[:, Lp - 1].contiguous()
        self._head_and_sample(last, R)

    # ---------------------------------------------------------------- one step
    def _head_and_sample(self, last: torch.Tensor, R: int, ss: Optional[torch.Tensor] = None):
        """gen_head on the last position, CFG + sampling, next input embeds (aligner).  ss: the row sums of
        squares of ``last`` (fused path), so the final RMSNorm folds into gen_head's first Linear."""
        dims = self.dims
        if self.fused and ss is not None:
            ops.decode_linear(last, self.gh_w1_d, self.zg[:R], self.lws, norm=(ss, self.norm, dims.rms_eps),
                              bias=self.gh_b1, gelu=True)
        else:
            ops.rmsnorm_fwd(last, self.norm, self.hf[:R], self.rstd[:R], dims.rms_eps)
            ops.decode_gemv(self.hf[:R], self.gh_w1_d, self.zg[:R], bias=self.gh_b1, gelu=True, ws=self.gws)
        if self.fused:
            ops.decode_linear(self.zg[:R], self.gh_w2_d, self.logits[:R], self.lws, bias=self.gh_b2)
        else:
            ops.decode_gemv(self.zg[:R], self.gh_w2_d, self.logits[:R], bias=self.gh_b2, ws=self.gws)
        B = R // 2
        probs = None
        if self.probs is not None:
            probs = self.probs[self._host_step]
        ops.cfg_sample(self.logits[:R], B, self.cfg_weight, self.temperature, self.u, self.step, self.n_img,
                       self.tokens[:B], self.next_ids[:R], probs)
        ops.gen_aligner_in(self.next_ids[:R], self.gen_embed, self.al_w1, self.al_b1, self.e1[:R])
        if self.fused:  # the next step's input and its row sums of squares (layer 0's folded RMSNorm)
            ops.decode_linear(self.e1[:R], self.al_w2_d, self.x[:R], self.lws, bias=self.al_b2, ss_out=self.ss_x)
        else:
            ops.decode_gemv(self.e1[:R], self.al_w2_d, self.x[:R], bias=self.al_b2, ws=self.gws)
        ops.decode_advance(self.pos, self.step)

    def _decode_step(self, R: int):
        """One token for every row at position *pos: the layer stack ping-pongs the residual
        stream between self.x and self.xo; the aligner writes the next input into self.x."""
        dims = self.dims
        H = dims.n_heads
        scale = 1.0 / math.sqrt(128)
        g = self.gws
        x, xo = self.x[:R], self.xo[:R]
        D, Fd = dims.d_model, dims.d_ff
        if self.fused:
            self._decode_step_fused(R)
            return
        fuse_qkv = ops.decode_gemv_fusable(R, 3 * D, D)  # split sum + RoPE/KV store in one kernel
        fuse_gu = ops.decode_gemv_fusable(R, 2 * Fd, D)  # split sum + SwiGLU in one kernel
        for i, lw in enumerate(self.layers):
            ops.rmsnorm_fwd(x, lw["ln_in"], self.xn[:R], self.rstd[:R], dims.rms_eps)
            if fuse_qkv:
                ops.decode_gemv_kv(self.xn[:R], lw["qkv_d"], g, self.pos, (self.cos, self.sin), self.kc[i], self.vc[i],
                                   H, self.Tmax, self.q[:R])
            else:
                ops.decode_gemv(self.xn[:R], lw["qkv_d"], self.qkv[:R], ws=g)
                ops.kv_store(self.qkv[:R], R, 1, self.pos, self.kc[i], self.vc[i], H, self.Tmax,
                             rope=(self.cos, self.sin), q_out=self.q[:R])
            ops.attn_cache(self.q[:R], self.kc[i], self.vc[i], R, 1, H, self.Tmax, self.start, self.pos, scale,
                           self.attn[:R])
            ops.decode_gemv(self.attn[:R], lw["o_d"], self.xmid[:R], residual=x, ws=g)
            ops.rmsnorm_fwd(self.xmid[:R], lw["ln_post"], self.xn2[:R], self.rstd[:R], dims.rms_eps)
            if fuse_gu:
                ops.decode_gemv_swiglu(self.xn2[:R], lw["gu_d"], g, self.h[:R])
            else:
                ops.decode_gemv(self.xn2[:R], lw["gu_d"], self.gu[:R], ws=g)
                ops.swiglu_fwd(self.gu[:R], self.h[:R])
            ops.decode_gemv(self.h[:R], lw["down_d"], xo, residual=self.xmid[:R], ws=g)
            x, xo = xo, x
        self._head_and_sample(x, R)

    def _decode_step_fused(self, R: int):
        """_decode_step in 5 launches per layer (ops.decode_linear): q|k|v with the input RMSNorm folded in
        + RoPE / KV store, cached attention, o + residual (+ its row sums of squares), gate|up with the
        post-attention RMSNorm folded in + SwiGLU, down + residual (+ row sums of squares)."""
        dims = self.dims
        H, eps = dims.n_heads, dims.rms_eps
        scale = 1.0 / math.sqrt(128)
        ws = self.lws
        x, xo = self.x[:R], self.xo[:R]
        ss, sso = self.ss_x, self.ss_xo
        for i, lw in enumerate(self.layers):
            kv = (self.pos, (self.cos, self.sin), self.kc[i], self.vc[i], H, self.Tmax)
            if self.head_split:
                # q|k|v of heads [0, H/2) -> (attention of [0, H/2) on this stream | q|k|v + attention of [H/2, H)
                # on the side stream) -> o: the first half's attention streams the KV cache while the second
                # half's projection streams its weights
                H2 = H // 2
                main = torch.cuda.current_stream(self.device)
                ops.decode_qkv_heads(x, lw["qkv_d"], self.q[:R], ws, norm=(ss, lw["ln_in"], eps), kv=kv, h0=0, nh=H2)
                ev_q = torch.cuda.Event()
                ev_q.record(main)
                self._side.wait_event(ev_q)
                with torch.cuda.stream(self._side):
                    ops.decode_qkv_heads(x, lw["qkv_d"], self.q[:R], ws, norm=(ss, lw["ln_in"], eps), kv=kv, h0=H2,
                                         nh=H - H2)
                    ops.attn_cache_heads(self.q[:R], self.kc[i], self.vc[i], R, 1, H, self.Tmax, self.start, self.pos,
                                         scale, self.attn[:R], H2, H - H2)
                    ev_s = torch.cuda.Event()
                    ev_s.record(self._side)
                ops.attn_cache_heads(self.q[:R], self.kc[i], self.vc[i], R, 1, H, self.Tmax, self.start, self.pos,
                                     scale, self.attn[:R], 0, H2)
                main.wait_event(ev_s)
            else:
                ops.decode_linear(x, lw["qkv_d"], self.q[:R], ws, epi="kv", norm=(ss, lw["ln_in"], eps), kv=kv)
            if self.attn_o_one_launch and ops.decode_attn_o(
                    self.q[:R], self.kc[i], self.vc[i], R, H, self.Tmax, self.start, self.pos, scale, self.attn[:R],
                    lw["o_d"], x, self.xmid[:R], self.ss_mid, ws, step=self.step, layer=i, flags=self.attn_flags,
                    tmo=self.mlp_tmo):
                self.attn_o_used = True
            else:
                if not self.head_split:
                    ops.attn_cache(self.q[:R], self.kc[i], self.vc[i], R, 1, H, self.Tmax, self.start, self.pos,
                                   scale, self.attn[:R])
                ops.decode_linear(self.attn[:R], lw["o_d"], self.xmid[:R], ws, residual=x, ss_out=self.ss_mid)
            if self.mlp_one_launch and ops.decode_mlp(
                    self.xmid[:R], lw["gu_d"], lw["down_d"], self.h[:R], xo, ws, norm=(self.ss_mid, lw["ln_post"], eps),
                    ss_out=sso, step=self.step, layer=i, flags=self.mlp_flags, tmo=self.mlp_tmo):
                self.mlp_used = True
            else:
                ops.decode_linear(self.xmid[:R], lw["gu_d"], self.h[:R], ws, epi="swiglu",
                                  norm=(self.ss_mid, lw["ln_post"], eps))
                ops.decode_linear(self.h[:R], lw["down_d"], xo, ws, residual=self.xmid[:R], ss_out=sso)
            x, xo = xo, x
            ss, sso = sso, ss
        self._head_and_sample(x, R, ss)

    # ----------------------------------------------------------------- generate
    @torch.inference_mode()
    def generate_images(self, prompts: Sequence[Sequence[int]], seed: int = 0, use_graph: bool = True,
                        img_size: int = 384, patch_size: int = 16) -> torch.Tensor:
        """generate_image (image_generation.py:109-181) up to the saved pixels: the image tokens, then
        ``decode_code`` with shape [B, 8, img_size / patch_size, img_size / patch_size] and the uint8
        conversion.  Returns uint8 [B, img_size, img_size, 3] on the device."""
        if self.vq_decoder is None:
            raise RuntimeError("T2IGenerator was built without vq_weights: no pixel decoder")
        hw = img_size // patch_size
        if hw * hw != self.n_img:
            raise ValueError(f"{self.n_img} image tokens do not tile a {hw} x {hw} grid")
        tok = self.generate(prompts, seed=seed, use_graph=use_graph)
        dec = self.vq_decoder.decode_code(tok, hw, hw)
        return self.vq_decoder.to_images(dec)

    def uniforms(self, seed: int, B: int) -> torch.Tensor:
        """The sampler's uniforms [n_img_tokens, B] for a seed (set_seed(seed) in the reference
        seeds torch.multinomial; here a CPU generator seeds the inverse-CDF draws)."""
        g = torch.Generator(device="cpu").manual_seed(int(seed))
        return torch.rand(self.n_img, B, generator=g)

    @torch.inference_mode()
    def generate(self, prompts: Sequence[Sequence[int]], seed: int = 0, use_graph: bool = True,
                 record_probs: bool = False) -> torch.Tensor:
        """prompts: B lists of token ids (tokenizer.encode of the formatted prompt, BOS included).
        Returns the image-token ids int32 [B, n_img_tokens] (on the device)."""
        dims = self.dims
        B = len(prompts)
        if not 1 <= B <= self.max_batch:
            raise ValueError(f"batch of {B} prompts, capacity {self.max_batch}")
        for p in prompts:
            if not 1 <= len(p) <= self.max_prompt:
                raise ValueError(f"prompt length {len(p)} outside [1, {self.max_prompt}]")
            if min(p) < 0 or max(p) >= dims.vocab:
                raise ValueError(f"token id out of range [0, {dims.vocab})")
        R = 2 * B
        toks, start, Lp = self._prompt_rows(prompts)
        self.u.zero_()
        self.u[: self.n_img * B].copy_(self.uniforms(seed, B).reshape(-1))
        self.start[:R].copy_(start)
        self.pos.fill_(Lp)      # the first decoded token sits at position Lp
        self.step.fill_(0)
        self.mlp_flags.zero_()  # (the flags' epochs restart with the step counter)
        self.attn_flags.zero_()
        self.mlp_tmo.zero_()  # a wait that gave up in an earlier generate() does not fail this one
        if self.fused:
            ops.zero_ws_counters(self.lws, ops.WS_DECODE_LINEAR)  # split-sum counters, left zero by every call
        self.tokens.zero_()
        self.probs = (torch.zeros(self.n_img, B, dims.img_vocab, dtype=torch.float32, device=self.device)
                      if record_probs else None)
        self._host_step = 0
        self._prefill(toks, Lp)          # step 0 (+ advance: pos = Lp, step = 1 after it)
        self.pos.fill_(Lp)
        n_rest = self.n_img - 1
        if use_graph and not record_probs:
            if self._graph is None or self._graph_B != B:
                torch.cuda.synchronize(self.device)
                self._graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._graph):
                    self._decode_step(R)
                self._graph_B = B
            for _ in range(n_rest):
                self._graph.replay()
        else:
            for s in range(n_rest):
                self._host_step = s + 1
                self._decode_step(R)
        if (self.mlp_one_launch or self.attn_o_one_launch) and int(self.mlp_tmo.item()) != 0:
            raise RuntimeError("decode_mlp / decode_attn_o: a consumer workgroup's wait gave up (outputs invalid)")
        return self.tokens[:B]
