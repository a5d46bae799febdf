"""The SimPO policy engine: Janus-Pro LLM + LoRA + gen_head on the HIP kernels.

One call of ``forward`` runs what the reference runs from ``preprocess_batch``
(ospo/wrapper/train.py:219-279, minus VQ encode: token ids are given) through
``concatenated_forward`` (:345-372) and ``get_batch_logps`` (:375-396) and
returns the per-sequence mean log-prob of the 2B sequences (chosen first).
``backward`` takes d(loss)/d(logps) and accumulates the LoRA gradients into the
flat fp32 buffer (ospo_amd/lora.py layout) -- the autograd of train.py:448-456
+ PL's backward, written out explicitly.

MI355X-first memory plan (288 GB HBM3E per GPU):
  * frozen weights are stored twice, W [out,in] and W^T [in,out], so every
    forward AND backward product is an "NT" MFMA GEMM with K contiguous on
    both operands (7B: +13 GB);
  * q|k|v and gate|up are fused into single GEMMs (N = 3D, 2F);
  * every activation the backward needs stays resident (7B, B=4 pairs:
    ~19 GB) -- no gradient-checkpoint recompute (the reference recomputes:
    ospo/utils/model.py:45-46), and the [2B, T, 102400] text lm_head the
    reference evaluates and discards is never computed;
  * LoRA runs as a K-extension of the frozen GEMM (A2 = s*x.A^T, B2 =
    block-diagonal packed B), and its gradients land in the flat buffer by
    fp32-atomic transposed GEMMs.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import dropout, ops
from .lora import LoraLayout, roundup

BF16 = torch.bfloat16
F32 = torch.float32


@dataclass
class ModelDims:
    n_layers: int
    d_model: int
    d_ff: int
    n_heads: int
    head_dim: int
    vocab: int
    img_vocab: int
    img_embed: int
    gen_head_dim: int
    rope_theta: float = 10000.0
    rms_eps: float = 1e-6
    lora_r: int = 16
    lora_alpha: int = 32

    @classmethod
    def from_any(cls, d) -> "ModelDims":
        keys = cls.__dataclass_fields__.keys()
        src = d if isinstance(d, dict) else d.__dict__
        return cls(**{k: src[k] for k in keys if k in src})

    @property
    def lora_scale(self) -> float:
        return self.lora_alpha / self.lora_r


JANUS_PRO_7B = ModelDims(30, 4096, 11008, 32, 128, 102400, 16384, 8, 4096)
JANUS_PRO_1B = ModelDims(24, 2048, 5632, 16, 128, 102400, 16384, 8, 2048)


def _dev(t: torch.Tensor, device) -> torch.Tensor:
    return t.to(device=device, dtype=BF16).contiguous()


class SimPOEngine:
    """Device-resident Janus-Pro SimPO policy (one per GPU / rank)."""

    def __init__(self, dims: ModelDims, weights: Dict[str, torch.Tensor], device="cuda", max_pairs: int = 4,
                 max_text_len: int = 64, n_img_tokens: int = 576, lora_dropout: float = 0.0,
                 dropout_seed: int = 42, linear_dtype: str = "bf16", fuse_swiglu_bwd: bool = False,
                 dadb_splits=(8, 4, 4, 8), side_priority: int = -1, wgrad_wgs: int = 0, fuse_gdb: bool = True,
                 fuse_swiglu_gdb: bool = True,
                 da_stream: bool = True, keep_bits: bool = True, fuse_swiglu_u: bool = True,
                 side_after_norm: bool = True, gdb_groups=("qkv", "o", "gu", "down"), side_main=()):
        if not 0.0 <= float(lora_dropout) < 1.0:
            raise ValueError(f"lora_dropout must be in [0, 1), got {lora_dropout}")
        if linear_dtype not in ("bf16", "mx8"):
            raise ValueError(f"linear_dtype must be 'bf16' or 'mx8', got {linear_dtype!r}")
        # "mx8": the frozen decoder Linears (q|k|v, o, gate|up, down; forward and dX) run as MXFP8
        # block-scaled fp8 MFMA GEMMs (BASELINE config 5; oracle/mx8_ref.py defines the arithmetic)
        self.linear_dtype = linear_dtype
        # fuse_swiglu_bwd (bf16): the down_proj dX GEMM writes the SwiGLU backward (dgate | dup) from its
        # epilogue and dh is never stored (ospo_gemm_nt_swiglu_bwd_bf16, bit-identical).  Off by default: the
        # step time is the same (the epilogue's gu/dgu traffic is not overlapped with MFMA)
        self.fuse_swiglu_bwd = linear_dtype == "bf16" and bool(fuse_swiglu_bwd)
        # peft lora_dropout on the adapter inputs (ospo_amd/dropout.py: counter-based masks, one per input)
        self.lora_dropout = float(lora_dropout)
        self._kbits = {}  # (layer, group) -> the forward's dropout keep bits (_keep_bits)
        self.training = True
        self._drop_base = int(dropout_seed)
        self._drop_call = 0
        self.layer_grads_hook = None  # on_layer_grads for backward() reached through autograd (Trainer.fit)
        if dims.head_dim != 128:
            raise ValueError("head_dim must be 128 (Janus-Pro)")
        if dims.d_model % 256 or dims.d_ff % 256 or dims.gen_head_dim % 256 or dims.img_vocab % 256:
            raise ValueError("d_model, d_ff, gen_head_dim and img_vocab must be multiples of 256")
        self.dims, self.device = dims, torch.device(device)
        D, Fd, L = dims.d_model, dims.d_ff, dims.n_layers
        self.layout = LoraLayout(L, D, Fd, dims.lora_r)
        self.scale = dims.lora_scale
        dev = self.device
        w = weights
        # ---- frozen weights, fused and transposed copies
        self.embed = _dev(w["embed_tokens"], dev)
        self.layers = []
        for i in range(L):
            p = f"layers.{i}."
            wqkv = torch.cat([w[p + "q_proj"], w[p + "k_proj"], w[p + "v_proj"]], 0)
            wgu = torch.cat([w[p + "gate_proj"], w[p + "up_proj"]], 0)
            lay = {
                "ln_in": _dev(w[p + "input_layernorm"], dev), "ln_post": _dev(w[p + "post_attention_layernorm"], dev),
                "qkv": _dev(wqkv, dev), "o": _dev(w[p + "o_proj"], dev), "gu": _dev(wgu, dev),
                "down": _dev(w[p + "down_proj"], dev),
            }
            for k in ("qkv", "o", "gu", "down"):
                lay[k + "T"] = lay[k].t().contiguous()
                if linear_dtype == "mx8":  # fp8 copies replace the bf16 ones (quantized once: frozen)
                    lay[k] = ops.MX8.of(lay[k])
                    lay[k + "T"] = ops.MX8.of(lay[k + "T"])
            self.layers.append(lay)
        self.norm = _dev(w["norm"], dev)
        self.gh_w1, self.gh_b1 = _dev(w["gen_head.w1"], dev), _dev(w["gen_head.b1"], dev)
        self.gh_w2, self.gh_b2 = _dev(w["gen_head.w2"], dev), _dev(w["gen_head.b2"], dev)
        self.gh_w1T, self.gh_w2T = self.gh_w1.t().contiguous(), self.gh_w2.t().contiguous()
        self.al_w1, self.al_b1 = _dev(w["gen_aligner.w1"], dev), _dev(w["gen_aligner.b1"], dev)
        self.al_w2, self.al_b2 = _dev(w["gen_aligner.w2"], dev), _dev(w["gen_aligner.b2"], dev)
        self.gen_embed = _dev(w["gen_embed"], dev)
        # ---- LoRA flat state
        n = self.layout.numel
        self.lora = torch.zeros(n, dtype=BF16, device=dev)
        lora_src = {k: v for k, v in w.items() if ".lora_" in k}
        if lora_src:
            staging = torch.zeros(n, dtype=BF16)
            self.layout.to_flat({k: v.to(BF16).cpu() for k, v in lora_src.items()}, staging)
            self.lora.copy_(staging)
        self.grads = torch.zeros(n, dtype=F32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=BF16, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=BF16, device=dev)
        self.opt_step = 0
        self._sumsq = torch.zeros(1, dtype=F32, device=dev)
        self._sumsq_ws = torch.zeros(2048, dtype=F32, device=dev)
        # packed LoRA operands, per group contiguous over layers ([L][...], one pack launch per group)
        r = self.layout.r
        self._packed_all = {
            gname: (torch.zeros(max(L, 1), g.Rp, g.Kin, dtype=BF16, device=dev),
                    torch.zeros(max(L, 1), g.Kin, g.Rp, dtype=BF16, device=dev),
                    torch.zeros(max(L, 1), g.nmods * g.Nmod, g.Rp, dtype=BF16, device=dev),
                    torch.zeros(max(L, 1), g.nmods * r, g.Nmod, dtype=BF16, device=dev))
            for gname, g in self.layout.groups.items()}
        self.packed = [{gname: tuple(t[i] for t in ts) for gname, ts in self._packed_all.items()} for i in range(L)]
        # fuse_gdb (LoRA r = 16, or 32 since round 6): g = s dy.B and dB += dy^T u of a group in one stream over dy
        # on the main stream (ospo_lora_gdb_r); the side stream then runs only dA.  Off: g on the main stream, dB with
        # dA on the side.
        self.fuse_gdb = bool(fuse_gdb) and dims.lora_r in (16, 32)
        # fuse_swiglu_gdb (with fuse_gdb, bf16): the SwiGLU backward and the gate|up group's g / dB in one stream
        # over (dh, gu) -- dgu written once, never read back by a separate g / dB pass (ospo_swiglu_lora_gdb)
        self.fuse_swiglu_gdb = bool(fuse_swiglu_gdb) and self.fuse_gdb
        # gdb_groups (round 5 A/B): the groups whose g / dB run as the fused ospo_lora_gdb stream; the others take
        # g from the skinny product on the main stream (no separate split-sum launch) and dB on the side stream
        self.gdb_groups = frozenset(gdb_groups)
        self.pack_lora()
        self._alloc(max_pairs, max_text_len, n_img_tokens)
        self._rope_T = -1
        # The LoRA weight-gradient side stream runs at high HIP priority (-1): its short memory-bound dA/dB
        # launches are dispatched ahead of the main stream's GEMM workgroups and get out of their way
        # (+0.3 %, profiles/r01/stream_priority_ab.log; main-stream high priority instead: -0.2 %).
        # K splits of the LoRA dA / dB products: dA (Kin <= 8192, > 8192), dB (multi-module, single-module)
        # (8, 4, 4, 8 measured best, profiles/r01/dadb_splits_ab_highprio.log)
        self._dadb_splits = tuple(int(v) for v in dadb_splits)
        # > 0: the LoRA weight gradients as ospo_lora_wgrad streams of ~wgrad_wgs workgroups; 0: the 64 x 64
        # f32-atomic tiles (faster in isolation, 180.8 vs 198.8 us per layer, tools/lora_grads_bench.py)
        self.wgrad_wgs = int(wgrad_wgs)
        # da_stream: dA as one stream over the adapter input with the forward's keep bits (ops.lora_da, round 3:
        # 5.2 ms of side-stream kernel time per step against 5.6 for the 64 x 64 f32-atomic tiles re-hashing the
        # mask, profiles/r03/step_lora_variants_breakdown_v2.txt); off: those tiles (ops.gemm_f32acc(b_dropout=...)),
        # which re-hash (their byte-wise keep-bit reads cost more than the hashes: 66.7 vs 47 us per launch)
        self.da_stream = bool(da_stream)
        # keep_bits: the forward's u products store each dropout mask as bits, which the dX GEMMs and dA read
        # instead of re-hashing it (round 3); off: every consumer re-hashes
        self.use_keep_bits = bool(keep_bits)
        # fuse_swiglu_u: the SwiGLU forward and the down adapter's u product in one stream over gu (round 3;
        # bit-identical; 95.7 us against 50.4 + ~44 + 5 us unfused once silu uses the hardware reciprocal)
        self.fuse_swiglu_u = bool(fuse_swiglu_u)
        # side_after_norm: a layer's dA work is enqueued after its input-norm backward, so it overlaps the next
        # layer's down dX GEMM instead of that memory-bound norm (+0.4 % at the step, 3 of 3 alternating rounds,
        # profiles/r03/step_side_order_ab.jsonl); off: enqueued right after the q|k|v dX GEMM
        self.side_after_norm = bool(side_after_norm)
        # side_main: the groups whose dA / dB run on the main stream instead of the side stream (A/B, round 5)
        self.side_main = tuple(side_main)
        if len(self._dadb_splits) != 4 or min(self._dadb_splits) < 1:
            raise ValueError("dadb_splits must be four positive split counts")
        self._side = torch.cuda.Stream(device=self.device, priority=int(side_priority))

    def ensure_capacity(self, pairs: int, text_len: int):
        """Grow the activation buffers when a batch exceeds them (ragged prompts)."""
        if pairs > self.cap_pairs or text_len + self.N > self.cap_T:
            self._alloc(max(pairs, self.cap_pairs), max(text_len, self.cap_T - self.N), self.N)

    # ------------------------------------------------------------ setup
    def _alloc(self, max_pairs, max_text_len, N):
        dims, dev = self.dims, self.device
        D, Fd, L, H = dims.d_model, dims.d_ff, dims.n_layers, dims.n_heads
        S = 2 * max_pairs
        Tm = max_text_len + N
        self.cap_pairs, self.cap_T, self.N = max_pairs, Tm, N
        Mc = roundup(S * Tm, 64)
        self.Mcap = Mc
        Rmax = max(g.Rp for g in self.layout.groups.values())
        z = lambda *s, dt=BF16: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        self.acts = []
        for _ in range(L):
            self.acts.append({
                "x": z(Mc, D), "xn1": z(Mc, D), "rstd1": z(Mc, dt=F32), "u_qkv": z(Mc, self.layout.groups["qkv"].Rp),
                "qkv": z(Mc, 3 * D), "lse": z(S * H * Tm, dt=F32), "attn": z(Mc, D),
                "u_o": z(Mc, self.layout.groups["o"].Rp), "xmid": z(Mc, D), "xn2": z(Mc, D), "rstd2": z(Mc, dt=F32),
                "u_gu": z(Mc, self.layout.groups["gu"].Rp), "gu": z(Mc, 2 * Fd), "h": z(Mc, Fd),
                "u_d": z(Mc, self.layout.groups["down"].Rp),
            })
        self.x_final = z(Mc, D)
        self.hf = z(Mc, D)
        self.rstd_f = z(Mc, dt=F32)
        R = S * N
        Dg, V = dims.gen_head_dim, dims.img_vocab
        self.img_ids = torch.zeros(R, dtype=torch.int32, device=dev)
        self.text_ids = torch.zeros(max_pairs * max(max_text_len, 1), dtype=torch.int32, device=dev)
        self.e1 = z(R, D)
        self.img_emb = z(R, D)
        self.hsel = z(R, D)
        self.zpre = z(R, Dg)
        self.zact = z(R, Dg)
        self.logits = z(R, V)
        self.lse_tok = z(R, dt=F32)
        self.tok_logp = z(R, dt=F32)
        self.seq_logps = z(S, dt=F32)
        # backward scratch (shared by all layers)
        self.u32_flat = z(Mc * Rmax, dt=F32)
        # Every buffer the side stream's dA/dB read (a group's g buffer and its dy) comes in two copies,
        # used by layer parity: main rewrites a copy in layer i only after the side stream finished
        # layer i+2's products, so the guards below practically never stall the main stream.
        self.gsc2 = {name: [z(Mc, g.Rp), z(Mc, g.Rp)] for name, g in self.layout.groups.items()}
        # the gradient w.r.t. each layer's output, three copies (round 5; two before): layer i's copy is read by its
        # side-stream dB / dA work and rewritten by layer i-2's input-norm backward, so main waits for the side work
        # of the layer two above (as for every other side operand) instead of the layer just above
        self.dx2 = [z(Mc, D), z(Mc, D), z(Mc, D)]
        self.dxmid2 = [z(Mc, D), z(Mc, D)]
        self.dqkv2 = [z(Mc, 3 * D), z(Mc, 3 * D)]
        self.dgu2 = [z(Mc, 2 * Fd), z(Mc, 2 * Fd)]
        self.dxn = z(Mc, D)
        self.dattn = z(Mc, D)
        self.dh = None if self.fuse_swiglu_bwd else z(Mc, Fd)
        self.delta_ws = z(S * H * Tm, dt=F32)
        # dS^T of one layer's attention backward (bf16, ~210 MB at 8 sequences x T = 600): the dK/dV kernel
        # writes it, dQ = dS.K reads it, so S and dP are not recomputed for dQ (5 MFMA products, not 7)
        self.ds_ws = ops.flash_attn_bwd_ws(S, Tm, H, dev)
        self.dz = z(R, Dg)
        self.dhsel = z(R, D)
        # fp32 g partials of the fused g / dB stream (ospo_lora_gdb_r), sized once for the capacity
        # (the size grows with the rows); every group's call fits
        self._gdb_ws = None
        if self.fuse_gdb:
            nb = max((ops.query_gdb_ws(Mc, g.nmods, g.Nmod, dims.lora_r) for g in self.layout.groups.values()
                      if g.Nmod % 128 == 0 and g.nmods <= 4), default=0)
            if nb > 0:
                self._gdb_ws = torch.zeros((nb + 15) // 16 * 4, dtype=F32, device=dev)  # (counters: zero)
        # MXFP8 activation operands, one per contraction size (main-stream GEMMs only, reused in order)
        self._mx = {K: ops.MX8(Mc, K, dev) for K in {D, Fd, 2 * Fd, 3 * D}} if self.linear_dtype == "mx8" else {}

    def pack_lora(self):
        """Rebuild the packed A / A^T / block-diagonal B / B^T operands from the flat params
        (one launch per module group, all layers)."""
        L, r = self.dims.n_layers, self.layout.r
        if L == 0:
            return
        for gname, g in self.layout.groups.items():
            Acat, AcatT, Bcat, BT = self._packed_all[gname]
            A = self.lora[g.a_off:]
            B = self.lora[g.b_off:]
            ops.lora_pack(A, B, g.nmods, r, g.Kin, g.Nmod, g.Rp, Acat, AcatT, Bcat, BT, n_layers=L,
                          layer_stride=self.layout.per_layer)

    def _mxo(self, K: int):
        """mx8 mode: the MXFP8 operand a producer kernel (norm / SwiGLU) fills next to its bf16
        output, so the following _lin(..., pre=True) skips its quantize pass; bf16 mode: None."""
        return self._mx.get(K)

    def _lin(self, x: torch.Tensor, w, out: torch.Tensor, pre: bool = False, **kw) -> torch.Tensor:
        """A frozen decoder Linear (+ LoRA K-extension / bias / residual / RoPE / dropout epilogues):
        the bf16 MFMA GEMM, or in mx8 mode: quantize x (MXFP8, one pass) + the block-scaled fp8 GEMM.
        pre=True: x's producer already wrote its MXFP8 copy into self._mxo(K) (no quantize pass)."""
        if self.linear_dtype == "mx8":
            a = self._mx[x.shape[1]]
            if not pre:
                ops.quant_mx8(x, a)
            elif a.m != x.shape[0]:
                raise RuntimeError(f"pre-quantized operand holds {a.m} rows, the Linear needs {x.shape[0]}")
            kw.pop("keep_bits", None)  # (the MXFP8 GEMM re-hashes the dropout mask)
            return ops.gemm_nt_mx8(a, w, out, **kw)
        return ops.gemm_nt(x, w, out, **kw)

    def lora_tensors(self) -> Dict[str, torch.Tensor]:
        return self.layout.from_flat(self.lora)

    def grad_tensors(self) -> Dict[str, torch.Tensor]:
        return self.layout.from_flat(self.grads)

    def _rope(self, T):
        if T != self._rope_T:
            self.cos, self.sin = ops.rope_tables(T, self.dims.head_dim, self.dims.rope_theta, self.device)
            self._rope_T = T

    # ------------------------------------------------------------ LoRA helpers
    def _u32(self, Rp: int) -> torch.Tensor:
        return self.u32_flat[: self.Mcap * Rp].view(self.Mcap, Rp)

    def _skinny_ws(self, K: int, n_tiles: int) -> torch.Tensor:
        """Split-K workspace of ospo_lora_skinny (grown on demand, never shared across streams)."""
        need = ops.lora_skinny_ws_bytes(self.Mk, K, n_tiles)
        ws = getattr(self, "_sk_ws", None)
        if ws is None or ws.numel() * 4 < need:
            ws = self._sk_ws = ops.lora_skinny_ws(self.Mk, K, max(n_tiles, 8), self.device)
        return ws

    def _bits_bwd(self, layer: int, group: str, drop, K: int):
        """The keep bits the forward wrote for this adapter input (None: the consumer re-hashes)."""
        if drop is None or not self.use_keep_bits or (layer, group) not in self._kbits:
            return None
        return self._keep_bits(layer, group, K)

    # u-product tile counts whose streaming kernel writes keep bits (ospo_lora_skinny refuses the others)
    _BITS_TILES = (1, 2, 3, 4, 6, 8)

    def _bits_fwd(self, layer: int, group: str, K: int):
        if not self.use_keep_bits or self._drop(layer, group) is None:
            return None
        nt = (self.layout.groups[group].nmods * self.layout.r + 15) // 16
        if nt not in self._BITS_TILES:
            return None  # (no bits written: the backward's consumers re-hash the mask)
        return self._keep_bits(layer, group, K)

    def _drop(self, layer: int, group: str):
        """(seed, p) of one adapter input's dropout mask in the current step, or None."""
        if self.lora_dropout <= 0 or not self.training:
            return None
        return (dropout.layer_seed(self._drop_base, self._drop_call, layer, group), self.lora_dropout)

    def _keep_bits(self, layer: int, group: str, K: int):
        """The keep bits of one adapter input's dropout mask ([Mcap, K] bits, row-major), written by the
        forward's u product and read by the backward's dA (ops.lora_da) instead of re-hashing; None where
        the streaming kernels do not apply (then dA re-hashes)."""
        if K % 128 or self.Mcap * K * 2 >= 2 ** 31:
            return None
        key = (layer, group)
        t = self._kbits.get(key)
        if t is None or t.numel() * 8 < self.Mcap * K:
            t = self._kbits[key] = torch.empty(self.Mcap * K // 8, dtype=torch.uint8, device=self.device)
        return t

    def _lora_down(self, x, Acat, out_bf16, M, nmods, drop=None, xd=None, bits=None):
        """out = bf16(scale * dropout(x) . Acat^T)  ([Mcap, Rp]; rows M..Mk-1 and unused columns zero).
        With drop=(seed, p) and xd given, the masked x is also written to xd (the engine passes none:
        the backward's dA recomputes the mask); bits: the mask's keep bits for that dA (_keep_bits)."""
        Rp, K = Acat.shape
        used = nmods * self.layout.r
        nt = (used + 15) // 16
        ops.lora_skinny(x, Acat, out_bf16, M, self.Mk, K, nt, 0, self.scale, b_rows=used, ws=self._skinny_ws(K, nt),
                        dropout=drop, xd=xd if drop else None, keep_bits=bits if drop else None)

    def _lora_g_db(self, dy, g, Bcat, BT, M, par, u, gbase):
        """(g_s, dB done): with fuse_gdb, g_s = bf16(scale * dy . Bcat) and dB += dy^T . u in one stream over dy
        (ospo_lora_gdb); else _lora_g and the side stream computes dB."""
        r = self.layout.r
        if not (self.fuse_gdb and g.name in self.gdb_groups and self._gdb_ws is not None and r in (16, 32)
                and g.Nmod % 128 == 0 and g.nmods <= 4 and g.nmods * r <= g.Rp):
            return self._lora_g(dy, g, Bcat, BT, M, par), False
        out = self.gsc2[g.name][par]
        b_off = gbase + g.b_off
        dB = self.grads[b_off: b_off + g.nmods * g.Nmod * r].view(g.nmods * g.Nmod, r)
        ops.lora_gdb(dy, BT, u, out, dB, M, self.Mk, g.nmods, g.Nmod, self.scale, ws=self._gdb_ws, r=r)
        return out, True

    def _swiglu_g_db(self, g, M, par, a, dgu, gbase, BT):
        """dgu = swiglu_bwd(dh, gu) with the gate|up group's g_s and dB in one stream (ospo_swiglu_lora_gdb);
        None when the shapes do not fit it (the caller then runs swiglu_bwd and _lora_g_db)."""
        r = self.layout.r
        if not (self.fuse_swiglu_gdb and self._gdb_ws is not None and r in (16, 32) and g.nmods == 2
                and g.Nmod % 128 == 0 and self.dh is not None and self._mxo(2 * g.Nmod) is None
                and dgu.shape[0] * dgu.stride(0) * 2 < 2 ** 31):
            return None
        out = self.gsc2[g.name][par]
        b_off = gbase + g.b_off
        dB = self.grads[b_off: b_off + g.nmods * g.Nmod * r].view(g.nmods * g.Nmod, r)
        ops.swiglu_lora_gdb(self.dh, a["gu"], dgu, BT, a["u_gu"], out, dB, M, self.Mk, self.scale, ws=self._gdb_ws,
                            r=r)
        return out

    def _lora_g(self, dy, g, Bcat, BT, M, par=0):
        """g_s = bf16(scale * dy . Bcat)  ([Mcap, Rp]; rows M..Mk-1 zero), into g buffer copy `par`."""
        r = self.layout.r
        out = self.gsc2[g.name][par]
        if g.nmods == 1:
            nt = (r + 15) // 16
            ops.lora_skinny(dy, BT, out, M, self.Mk, g.Nmod, nt, 0, self.scale, b_rows=r,
                            ws=self._skinny_ws(g.Nmod, nt))
        elif r % 16 == 0:  # block-diagonal: n-tile j reduces over module j // (r/16) of dy
            nt = g.nmods * r // 16
            ops.lora_skinny(dy, BT, out, M, self.Mk, g.Nmod, nt, g.Nmod, self.scale,
                            ws=self._skinny_ws(g.Nmod, nt), module_tiles=r // 16)
        else:  # block-diagonal with r % 16 != 0: split-K fp32 path
            K = Bcat.shape[0]
            u32 = self._u32(g.Rp)
            u32.zero_()
            ops.gemm_f32acc(dy[:M], Bcat, u32, a_kmajor=False, b_kmajor=True, k_splits=max(1, min(K // 512, 8)))
            ops.f32_to_bf16(u32, out, self.scale)
        return out

    # ------------------------------------------------------------ forward
    def forward(self, text_ids: torch.Tensor, chosen_ids: torch.Tensor, rejected_ids: torch.Tensor) -> torch.Tensor:
        """text_ids int32 [B, Lt] (-1 = right padding, ragged prompts), chosen/rejected
        int [B, N] VQ token ids.  Returns seq_logps fp32 [2B] (chosen first)."""
        dims = self.dims
        B, Lt = text_ids.shape
        N = chosen_ids.shape[1]
        self.ensure_capacity(B, Lt)
        # the in-launch split sums' counters (workspace heads, sized by the library: ops.ws_counter_bytes) are
        # left zero by every call that completes; re-zeroing them once per step (two small fills) bounds the damage of
        # one that did not (an aborted step) to that step
        if getattr(self, "_sk_ws", None) is not None:
            ops.zero_ws_counters(self._sk_ws, ops.WS_SKINNY)
        if getattr(self, "_gdb_ws", None) is not None:
            ops.zero_ws_counters(self._gdb_ws, ops.WS_LORA_GDB)
        if N != self.N:
            raise ValueError(f"batch (B={B}, Lt={Lt}, N={N}) exceeds engine capacity "
                             f"(pairs={self.cap_pairs}, T={self.cap_T}, N={self.N})")
        if Lt < 1:
            raise ValueError("need at least one text token (the <begin_of_image> tag)")
        for t, hi, name in ((text_ids, dims.vocab, "text id"), (chosen_ids, dims.img_vocab, "chosen VQ id"),
                            (rejected_ids, dims.img_vocab, "rejected VQ id")):
            if not t.is_cuda and t.numel() and (int(t.max()) >= hi or int(t.min()) < (-1 if t is text_ids else 0)):
                raise ValueError(f"{name} out of range [0, {hi})")
        S, T = 2 * B, Lt + N
        M = S * T
        if self.lora_dropout > 0 and self.training:
            self._drop_call += 1  # fresh masks per forward; backward() reuses this call's
            if M * max(self.dims.d_model, self.dims.d_ff) >= 2 ** 32:
                raise ValueError("LoRA dropout mask index exceeds 32 bits")
        self.B, self.S, self.T, self.Lt, self.M = B, S, T, Lt, M
        self.Mk = roundup(M, 64)
        D, Fd, H, hd = dims.d_model, dims.d_ff, dims.n_heads, dims.head_dim
        self._rope(T)
        ids = self.img_ids[: S * N].view(S, N)
        ids[:B].copy_(chosen_ids, non_blocking=True)
        ids[B:].copy_(rejected_ids, non_blocking=True)
        tids = self.text_ids[: B * Lt].view(B, Lt)
        tids.copy_(text_ids, non_blocking=True)
        R = S * N
        # gen_aligner(gen_embed(ids)) -> image embeds; assemble [text | img] rows (train.py:267-277, 286-312)
        ops.gen_aligner_in(self.img_ids[:R], self.gen_embed, self.al_w1, self.al_b1, self.e1[:R])
        ops.gemm_nt(self.e1[:R], self.al_w2, self.img_emb[:R], bias=self.al_b2)
        x = self.acts[0]["x"] if dims.n_layers else self.x_final
        ops.assemble_inputs(tids, B, Lt, self.embed, self.img_emb[:R], N, D, x)
        lay = self.layout
        scale_attn = 1.0 / math.sqrt(hd)
        for i in range(dims.n_layers):
            a, lw, pk = self.acts[i], self.layers[i], self.packed[i]
            x = a["x"]
            ops.rmsnorm_fwd(x[:M], lw["ln_in"], a["xn1"][:M], a["rstd1"][:M], dims.rms_eps, mx=self._mxo(D))
            Acat, _, Bcat, _ = pk["qkv"]
            self._lora_down(a["xn1"], Acat, a["u_qkv"], M, lay.groups["qkv"].nmods, self._drop(i, "qkv"),
                            bits=self._bits_fwd(i, "qkv", D))
            if (3 * D) % 256 == 0:  # q|k RoPE fused into the projection's epilogue
                self._lin(a["xn1"][:M], lw["qkv"], a["qkv"][:M], pre=True, a2=a["u_qkv"][:M], b2=Bcat,
                          rope=(self.cos, self.sin, T, 2 * D))
            else:
                self._lin(a["xn1"][:M], lw["qkv"], a["qkv"][:M], pre=True, a2=a["u_qkv"][:M], b2=Bcat)
                ops.rope(a["qkv"], 0, D, S, T, H, hd, self.cos, self.sin)
            ops.flash_attn_fwd(a["qkv"], 0, D, 2 * D, a["attn"], a["lse"], S, T, H, hd, scale_attn, mx=self._mxo(D))
            Acat, _, Bcat, _ = pk["o"]
            self._lora_down(a["attn"], Acat, a["u_o"], M, lay.groups["o"].nmods, self._drop(i, "o"),
                            bits=self._bits_fwd(i, "o", D))
            self._lin(a["attn"][:M], lw["o"], a["xmid"][:M], pre=True, a2=a["u_o"][:M], b2=Bcat, residual=x[:M])
            ops.rmsnorm_fwd(a["xmid"][:M], lw["ln_post"], a["xn2"][:M], a["rstd2"][:M], dims.rms_eps,
                            mx=self._mxo(D))
            Acat, _, Bcat, _ = pk["gu"]
            self._lora_down(a["xn2"], Acat, a["u_gu"], M, lay.groups["gu"].nmods, self._drop(i, "gu"),
                            bits=self._bits_fwd(i, "gu", D))
            self._lin(a["xn2"][:M], lw["gu"], a["gu"][:M], pre=True, a2=a["u_gu"][:M], b2=Bcat)
            Acat, _, Bcat, _ = pk["down"]
            used_d = lay.groups["down"].nmods * lay.r
            if self.fuse_swiglu_u and self._mxo(Fd) is None and Fd % 64 == 0 and used_d <= 64:
                # SwiGLU fused with the down adapter's u product: one stream over gu, h never re-read
                nt = (used_d + 15) // 16
                ops.swiglu_fwd_lora_down(a["gu"], a["h"], Acat, a["u_d"], M, self.Mk, Fd, nt, self.scale,
                                         b_rows=used_d, ws=self._skinny_ws(Fd, nt), dropout=self._drop(i, "down"),
                                         keep_bits=self._bits_fwd(i, "down", Fd))
            else:
                ops.swiglu_fwd(a["gu"][:M], a["h"][:M], mx=self._mxo(Fd))
                self._lora_down(a["h"], Acat, a["u_d"], M, lay.groups["down"].nmods, self._drop(i, "down"),
                                bits=self._bits_fwd(i, "down", Fd))
            xn = self.acts[i + 1]["x"] if i + 1 < dims.n_layers else self.x_final
            self._lin(a["h"][:M], lw["down"], xn[:M], pre=True, a2=a["u_d"][:M], b2=Bcat, residual=a["xmid"][:M])
        ops.rmsnorm_fwd(self.x_final[:M], self.norm, self.hf[:M], self.rstd_f[:M], dims.rms_eps)
        # gen_head on the N positions that predict image tokens: t = Lt-1 .. T-2 (train.py:385-391)
        ops.gather_rows(self.hf, S, T, Lt - 1, N, self.hsel[:R])
        ops.gemm_nt(self.hsel[:R], self.gh_w1, self.zpre[:R], bias=self.gh_b1)
        ops.gelu_fwd(self.zpre[:R], self.zact[:R])
        ops.gemm_nt(self.zact[:R], self.gh_w2, self.logits[:R], bias=self.gh_b2)
        ops.logprob_fwd(self.logits[:R], self.img_ids[:R], N, self.lse_tok[:R], self.tok_logp[:R],
                        self.seq_logps[:S])
        return self.seq_logps[:S]

    def logit_sums(self, skip_last: bool = False) -> torch.Tensor:
        """fp32 [S]: per sequence, the sum of the gen_head logits over every position and code --
        what the reference's ``all_logits[:B].mean()`` logging reduces (train.py:441-442) -- without
        the [S, T, V] tensor: sum_v (z W2^T + b2)_v = z . colsum(W2) + sum(b2), z = GELU(h W1^T + b1).
        The N predicting positions reuse the forward's z; the Lt other positions (text, and the
        last, whose logits no loss term reads) run gen_head's first Linear here.  skip_last: leave
        position T-1 out (train.py:422 rebinds the logits to [..., :-1, :] when sft_weight > 0).
        Call after forward() and before backward()."""
        S, T, Lt, N, D = self.S, self.T, self.Lt, self.N, self.dims.d_model
        Dg, V, dev = self.dims.gen_head_dim, self.dims.img_vocab, self.device
        if not hasattr(self, "_w2sum"):  # colsum(W2) = rows of W2^T . 1, sum(b2) (frozen: once)
            ones = torch.ones(V, dtype=F32, device=dev)
            self._w2sum = torch.empty(Dg, dtype=F32, device=dev)
            self._b2sum = torch.empty(1, dtype=F32, device=dev)
            ops.row_dot_sum(self.gh_w2T, ones, self._w2sum, 1)
            ops.row_dot_sum(self.gh_b2.view(1, V), ones, self._b2sum, 1)
        nt = Lt - 1  # text positions 0 .. Lt-2 (position Lt-1 is the first predicting one)
        nl = 0 if skip_last else 1
        seq = torch.empty(S, dtype=F32, device=dev)
        ops.row_dot_sum(self.zact[: S * N], self._w2sum, seq, N, add=self._b2sum, add_scale=float(N + nt + nl))
        rows = S * (nt + nl)
        if rows:
            hx = torch.empty(rows, D, dtype=BF16, device=dev)
            if nt:
                ops.gather_rows(self.hf, S, T, 0, nt, hx[: S * nt])
            if nl:
                ops.gather_rows(self.hf, S, T, T - 1, 1, hx[S * nt:])
            zp = torch.empty(rows, Dg, dtype=BF16, device=dev)
            ops.gemm_nt(hx, self.gh_w1, zp, bias=self.gh_b1)
            za = torch.empty_like(zp)
            ops.gelu_fwd(zp, za)
            if nt:
                ops.row_dot_sum(za[: S * nt], self._w2sum, seq, nt, accumulate=True)
            if nl:
                ops.row_dot_sum(za[S * nt:], self._w2sum, seq, 1, accumulate=True)
        return seq

    def full_logits(self) -> torch.Tensor:
        """gen_head over EVERY position: bf16 [S, T, V], what the reference's concatenated_forward
        returns (train.py:356-357, 367-368).  A new tensor; call after forward() (backward() leaves
        the final hidden state alone).  The loss path never needs it: the N predicting positions'
        logits are computed in forward() and the logits/* metrics come from logit_sums()."""
        S, T, Dg, V, dev = self.S, self.T, self.dims.gen_head_dim, self.dims.img_vocab, self.device
        M = S * T
        zp = torch.empty(M, Dg, dtype=BF16, device=dev)
        ops.gemm_nt(self.hf[:M], self.gh_w1, zp, bias=self.gh_b1)
        za = torch.empty_like(zp)
        ops.gelu_fwd(zp, za)
        out = torch.empty(M, V, dtype=BF16, device=dev)
        ops.gemm_nt(za, self.gh_w2, out, bias=self.gh_b2)
        return out.view(S, T, V)

    # ------------------------------------------------------------ backward
    def zero_grad(self):
        self.grads.zero_()

    def backward(self, g_seq: torch.Tensor, on_layer_grads=None):
        """g_seq fp32 [2B] = dL/d seq_logps.  Accumulates LoRA grads into self.grads.
        on_layer_grads(lo, hi): called (on the side stream, after that layer's dA/dB were
        enqueued) when grads[lo:hi] of a layer are final -- e.g. GradAllReduce.push, so the
        data-parallel all-reduce overlaps the rest of the backward."""
        dims = self.dims
        S, T, Lt, M, Mk, N = self.S, self.T, self.Lt, self.M, self.Mk, self.N
        D, Fd, H, hd = dims.d_model, dims.d_ff, dims.n_heads, dims.head_dim
        R = S * N
        g_seq = g_seq.to(device=self.device, dtype=F32).contiguous()
        # log-softmax/gather backward, in place over the logits buffer
        ops.logprob_bwd(self.logits[:R], self.img_ids[:R], self.lse_tok[:R], N, g_seq, self.logits[:R])
        ops.gemm_nt(self.logits[:R], self.gh_w2T, self.dz[:R])
        ops.gelu_bwd(self.dz[:R], self.zpre[:R], self.dz[:R])
        ops.gemm_nt(self.dz[:R], self.gh_w1T, self.dhsel[:R])
        ops.scatter_rows(self.dhsel[:R], S, T, Lt - 1, N, self.dxn[:M])
        L = dims.n_layers
        ops.rmsnorm_bwd(self.dxn[:M], self.x_final[:M], self.norm, self.rstd_f[:M], self.dx2[(L - 1) % 3][:M],
                        mx=self._mxo(D))
        scale_attn = 1.0 / math.sqrt(hd)
        lay = self.layout
        # LoRA weight grads (dA = g^T x, dB = dy^T u) of a layer run on a side stream, enqueued once the
        # layer's backward is on the main stream (one event each way per layer: an event record costs the
        # recording stream ~3.5 us and a wait ~1.4 us, tools/event_cost_probe.py; per-group events cost
        # ~0.4 ms per step).  Main waits before rewriting what pending side work reads: the g / dy copies of
        # parity q (layer i+2's) at the start of layer i, and the dx copy (i - 1) % 3 (layer i+2's, three copies)
        # before the input-norm backward that rewrites it.
        main, side = torch.cuda.current_stream(self.device), self._side
        side.wait_stream(main)
        done = {}  # layer -> event after that layer's side work was enqueued

        def wait_done(layer):
            ev = done.get(layer)
            if ev is not None:
                main.wait_event(ev)

        for i in reversed(range(dims.n_layers)):
            a, lw, pk = self.acts[i], self.layers[i], self.packed[i]
            gbase = lay.layer_off(i)
            q = i % 2  # copy of every side-stream operand this layer writes (dx: i % 3)
            wait_done(i + 2)  # layer i+2's side work read the copies this layer rewrites
            dx = self.dx2[i % 3]  # gradient w.r.t. this layer's output (bf16)
            dgu, dxmid, dqkv = self.dgu2[q], self.dxmid2[q], self.dqkv2[q]
            pending = []  # (group, g_s, x_in, dy, u, dropout, dB done on main)
            # ---- down_proj: out = xmid + h W_d^T + s (h A_d^T) B_d^T
            Acat, AcatT, Bcat, BT = pk["down"]
            gs, fdb = self._lora_g_db(dx, lay.groups["down"], Bcat, BT, M, q, a["u_d"], gbase)
            dr = self._drop(i, "down")
            if self.fuse_swiglu_bwd:
                ops.gemm_nt_swiglu_bwd(dx[:M], lw["downT"], a["gu"][:M], dgu[:M], a2=gs[:M], b2=AcatT, dropout=dr)
            else:
                self._lin(dx[:M], lw["downT"], self.dh[:M], pre=True, a2=gs[:M], b2=AcatT, dropout=dr,
                          keep_bits=self._bits_bwd(i, "down", dr, Fd))
            pending.append(("down", gs, a["h"], dx, a["u_d"], dr, fdb))
            # ---- gate/up
            Acat, AcatT, Bcat, BT = pk["gu"]
            gs = None if self.fuse_swiglu_bwd else self._swiglu_g_db(lay.groups["gu"], M, q, a, dgu, gbase, BT)
            if gs is not None:
                fdb = True
            else:
                if not self.fuse_swiglu_bwd:
                    ops.swiglu_bwd(self.dh[:M], a["gu"][:M], dgu[:M], mx=self._mxo(2 * Fd))
                gs, fdb = self._lora_g_db(dgu, lay.groups["gu"], Bcat, BT, M, q, a["u_gu"], gbase)
            dr = self._drop(i, "gu")
            self._lin(dgu[:M], lw["guT"], self.dxn[:M], pre=True, a2=gs[:M], b2=AcatT, dropout=dr,
                      keep_bits=self._bits_bwd(i, "gu", dr, D))
            pending.append(("gu", gs, a["xn2"], dgu, a["u_gu"], dr, fdb))
            ops.rmsnorm_bwd(self.dxn[:M], a["xmid"][:M], lw["ln_post"], a["rstd2"][:M], dxmid[:M],
                            dres=dx[:M], mx=self._mxo(D))
            # ---- o_proj
            Acat, AcatT, Bcat, BT = pk["o"]
            gs, fdb = self._lora_g_db(dxmid, lay.groups["o"], Bcat, BT, M, q, a["u_o"], gbase)
            dr = self._drop(i, "o")
            self._lin(dxmid[:M], lw["oT"], self.dattn[:M], pre=True, a2=gs[:M], b2=AcatT, dropout=dr,
                      keep_bits=self._bits_bwd(i, "o", dr, D))
            pending.append(("o", gs, a["attn"], dxmid, a["u_o"], dr, fdb))
            # ---- attention + RoPE
            ops.flash_attn_bwd(a["qkv"], 0, D, 2 * D, a["attn"], self.dattn, a["lse"], self.delta_ws, self.ds_ws,
                               dqkv, S, T, H, hd, scale_attn, rope_cos=self.cos, rope_sin=self.sin,
                               mx=self._mxo(3 * D) if i > 0 else None)  # layer 0 runs no q|k|v dX GEMM
            # ---- q/k/v
            Acat, AcatT, Bcat, BT = pk["qkv"]
            gs, fdb = self._lora_g_db(dqkv, lay.groups["qkv"], Bcat, BT, M, q, a["u_qkv"], gbase)
            dr = self._drop(i, "qkv")
            if i > 0:
                self._lin(dqkv[:M], lw["qkvT"], self.dxn[:M], pre=True, a2=gs[:M], b2=AcatT, dropout=dr,
                          keep_bits=self._bits_bwd(i, "qkv", dr, D))
            pending.append(("qkv", gs, a["xn1"], dqkv, a["u_qkv"], dr, fdb))
            def enqueue_side():
                # this layer's LoRA weight grads on the side stream (one event from main); side_main groups on
                # main, in the same order (the grads of a group are summed by the same kernels either way)
                for name, gs_, x_in, dy, u, dr_, fdb_ in pending:
                    if name in self.side_main:
                        self._lora_grads(gs_, x_in, dy, u, lay.groups[name], gbase, dr_, fdb_,
                                         self._bits_bwd(i, name, dr_, x_in.shape[1]))
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    for name, gs_, x_in, dy, u, dr_, fdb_ in pending:
                        if name not in self.side_main:
                            self._lora_grads(gs_, x_in, dy, u, lay.groups[name], gbase, dr_, fdb_,
                                             self._bits_bwd(i, name, dr_, x_in.shape[1]))
                    if on_layer_grads is not None:  # this layer's dA/dB are the last side-stream work so far
                        on_layer_grads(gbase, gbase + lay.per_layer)
                ev2 = torch.cuda.Event()
                ev2.record(side)
                done[i] = ev2

            late = self.side_after_norm and i > 0
            if not late:
                enqueue_side()
            if i > 0:
                # (writes dxn and dx copy (i - 1) % 3 = (i + 2) % 3, whose last reader, layer i+2's side work, main
                # waited for at this layer's start; neither is read by this layer's side work)
                ops.rmsnorm_bwd(self.dxn[:M], a["x"][:M], lw["ln_in"], a["rstd1"][:M], self.dx2[(i - 1) % 3][:M],
                                dres=dxmid[:M], mx=self._mxo(D))
            if late:
                enqueue_side()
            # layer 0: the gradient w.r.t. its input (the text / image embeddings) feeds nothing that
            # trains -- the embedding tables and gen_aligner are frozen (train.py:148-216) -- so its q|k|v dX
            # GEMM and the input RMSNorm backward are not run
        main.wait_stream(side)

    def _lora_grads(self, gs, x_in, dy, u, g, gbase, drop=None, skip_db=False, bits=None):
        """dA = g_s^T . dropout(x_in)  -> rows [nmods*r, Kin];  dB = dy^T . u_s (block diagonal).  dA: the
        f32-atomic tile product (or, da_stream, one stream over x_in: ops.lora_da), its dropout mask from the
        forward's keep bits (else re-hashed on x_in: the forward keeps no masked copy); dB, when not fused into
        ospo_lora_gdb, is the f32-atomic tile product."""
        r = self.layout.r
        Mk = self.Mk
        used = g.nmods * r
        a_off = gbase + g.a_off
        dA = self.grads[a_off: a_off + used * g.Kin].view(used, g.Kin)
        b_off = gbase + g.b_off
        dB = self.grads[b_off: b_off + g.nmods * g.Nmod * r].view(g.nmods * g.Nmod, r)
        if self.da_stream and g.Kin % 128 == 0 and g.Rp in (64, 128) and Mk * g.Kin * 2 < 2 ** 31:
            for c0 in range(0, used, 64):
                ops.lora_da(x_in[:Mk], gs[:Mk, c0:], dA[c0:c0 + 64], s_cols=min(64, used - c0), dropout=drop,
                            keep_bits=bits)
            if not skip_db:
                sa_small, sa_big, sb_multi, sb_single = self._dadb_splits
                ops.gemm_f32acc(dy[:Mk], u[:Mk], dB, a_kmajor=True, b_kmajor=True,
                                k_splits=sb_multi if g.nmods > 1 else sb_single, diag=(g.Nmod, r))
            return
        if self.wgrad_wgs > 0 and r % 16 == 0 and g.Rp in (64, 128):
            sa, sb = self._wgrad_splits(g.Kin), self._wgrad_splits(g.nmods * g.Nmod)
            ops.lora_wgrad(x_in[:Mk], gs[:Mk], dA, mode=0, s_cols=used, splits=sa, dropout=drop)
            if not skip_db:
                ops.lora_wgrad(dy[:Mk], u[:Mk], dB, mode=1, s_cols=used, splits=sb, nmod=g.Nmod, r=r)
            return
        # other ranks: the 64 x 64 f32-atomic tiles (K splits measured on the 7B shapes, profiles/r01/
        # lora_grads_sweep.jsonl)
        sa_small, sa_big, sb_multi, sb_single = self._dadb_splits
        ops.gemm_f32acc(gs[:Mk, :used], x_in[:Mk], dA, a_kmajor=True, b_kmajor=True,
                        k_splits=sa_big if g.Kin > 8192 else sa_small, b_dropout=drop)
        if not skip_db:  # (with fuse_gdb, ospo_lora_gdb produced dB with g on the main stream)
            ops.gemm_f32acc(dy[:Mk], u[:Mk], dB, a_kmajor=True, b_kmajor=True,
                            k_splits=sb_multi if g.nmods > 1 else sb_single, diag=(g.Nmod, r))

    def _wgrad_splits(self, N: int) -> int:
        """K-range splits of a LoRA weight-gradient stream: ~wgrad_wgs workgroups of 256-column stripes."""
        stripes = max(1, N // 256)
        return max(1, min(self.Mk // 64 // 4, round(self.wgrad_wgs / stripes)))

    # ------------------------------------------------------------ optimizer
    def grad_norm_sq(self) -> torch.Tensor:
        self._sumsq.zero_()
        ops.sumsq(self.grads, self._sumsq, self._sumsq_ws)
        return self._sumsq

    def optimizer_step(self, lr=4e-5, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.0, max_norm=1.0):
        """PL clip (gradient_clip_val) + AdamW on the flat bf16 LoRA params, then repack.
        The pre-clip norm stays on device (``self._sumsq``); no host sync."""
        self.opt_step += 1
        self.grad_norm_sq()
        ops.adamw_clip(self.lora, self.grads, self.exp_avg, self.exp_avg_sq, lr, betas[0], betas[1], eps,
                       weight_decay, self.opt_step, self._sumsq, max_norm if max_norm else 0.0)
        self.pack_lora()


def synthetic_weights(dims: ModelDims, device, seed: int = 0, lora_seed: int = 1, std: float = 0.02,
                      lora_b_std: float = 1e-3) -> Dict[str, torch.Tensor]:
    """Random-init weights of the Janus-Pro architecture, generated ON the device
    (no checkpoint exists offline).  Same names/statistics as oracle.init_weights:
    N(0, 0.02) linears, norms ~1, LoRA A kaiming-uniform, LoRA B ~ N(0, 1e-3)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    D, Fd = dims.d_model, dims.d_ff

    def n(*shape, s=std):
        return (torch.randn(*shape, generator=g, device=dev) * s).to(BF16)

    def norm(*shape):
        return (1.0 + torch.randn(*shape, generator=g, device=dev) * 0.05).to(BF16)

    shapes = {"q_proj": (D, D), "k_proj": (D, D), "v_proj": (D, D), "o_proj": (D, D),
              "gate_proj": (Fd, D), "up_proj": (Fd, D), "down_proj": (D, Fd)}
    w = {"embed_tokens": n(dims.vocab, D), "norm": norm(D)}
    for i in range(dims.n_layers):
        w[f"layers.{i}.input_layernorm"] = norm(D)
        w[f"layers.{i}.post_attention_layernorm"] = norm(D)
        for p, s in shapes.items():
            w[f"layers.{i}.{p}"] = n(*s)
    w["gen_head.w1"], w["gen_head.b1"] = n(dims.gen_head_dim, D), n(dims.gen_head_dim)
    w["gen_head.w2"], w["gen_head.b2"] = n(dims.img_vocab, dims.gen_head_dim), n(dims.img_vocab)
    w["gen_aligner.w1"], w["gen_aligner.b1"] = n(D, dims.img_embed, s=0.3), n(D)
    w["gen_aligner.w2"], w["gen_aligner.b2"] = n(D, D), n(D)
    w["gen_embed"] = n(dims.img_vocab, dims.img_embed, s=1.0)
    gl = torch.Generator(device=dev).manual_seed(lora_seed)
    r = dims.lora_r
    for i in range(dims.n_layers):
        for p, (o, k) in shapes.items():
            bound = 1.0 / math.sqrt(k)
            w[f"layers.{i}.{p}.lora_A"] = ((torch.rand(r, k, generator=gl, device=dev) * 2 - 1) * bound).to(BF16)
            w[f"layers.{i}.{p}.lora_B"] = (torch.randn(o, r, generator=gl, device=dev) * lora_b_std).to(BF16)
    return w
