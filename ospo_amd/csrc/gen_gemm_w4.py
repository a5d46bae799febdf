#!/usr/bin/env python3
"""Generates gemm_w4_asm.inc: the hand-placed K-loop programs of the 4-wave 256x256 bf16 GEMM
(gemm_nt_w4_kernel in gemm_w4.h).  Build-time only (the Makefile runs it); the output is committed.

Structure (one wave per SIMD, each wave a 128 x 128 quadrant of the 256 x 256 tile, 8 x 8 blocks of
v_mfma_f32_16x16x32_bf16, 256 accumulators in a[0:255]):

  * a K-tile (64 deep) is 128 MFMAs: substep 0 (k 0..31) for all 64 blocks, then substep 1 (k 32..63);
    block (i, j) = B fragment i (srcA, 16 output columns) x A fragment j (srcB, 16 output rows).
  * every fragment of a K-tile lives in registers (2 substeps x 16 fragments x 4 VGPRs = v[128:255]):
    substep-0 fragments of tile t+1 are read in the last MFMA gaps of tile t, substep-1 fragments of tile
    t in its first 16 gaps.  After the first 16 gaps the wave holds tile t whole, so one barrier
    (barrier 1) frees tile t's LDS stage and tile t+2's 16 LDS-DMA pieces go into it, spread over the
    following MFMAs (A pieces in substep 0, B pieces in substep 1).
  * barrier 2 (near the end of the tile) is preceded by a counted vmcnt that leaves tile t+2's pieces in
    flight and retires tile t+1's, whose substep-0 fragments are then read.
  * LDS: 2 stages x 64 KiB ([A 256 rows][B 256 rows] x 128 B, chunk XOR row&7 swizzle applied on the
    DMA source address), so each piece has ~1-1.5 K-tiles of load latency.

Every MFMA gap holds at most one ds_read or one LDS-DMA issue plus SALU, so the MFMA pipe stays fed
(MI355X_MICROARCH.md: 16x16x32 holds the SIMD's issue for 8 of its 16 cycles).  Accumulation order per
output element is that of gemm_nt_v5_kernel (K-tiles in order, substep 0 then 1; LoRA extension tiles
last, or first with dropout), so results are bit-identical to it.

Programs (runtime-selected by the kernel; each one asm statement):
  plain_E (E = 0, 1, 2 extension tiles at the end): prologue, tile 0, loop over main tiles 1..nm-3,
      tail tiles nm-2 .. nm-1+E.  Needs nm >= 4 main tiles.
  drop_E (E = 1, 2 extension tiles first, dropout mask applied to the accumulators after them):
      prologue, the E extension tiles, mask pass, loop over main tiles E..nt-3, the last two tiles.
      Needs nm >= 3.
"""
import sys

MFMA = "v_mfma_f32_16x16x32_bf16"
# staged programs: a block's bf16 staging runs this many MFMAs after its final MFMA (>= 4 x 16 cycles: past the
# 8-pass MFMA's result latency, which inline asm does not pad for the v_accvgpr_read)
STAGE_LAG = 4
RD_ORDER = [("X", 0)] + [("Y", j) for j in range(8)] + [("X", i) for i in range(1, 8)]


def X(s, i):
    b = 128 + 64 * s + 4 * i
    return f"v[{b}:{b + 3}]"


def Y(s, j):
    b = 160 + 64 * s + 4 * j
    return f"v[{b}:{b + 3}]"


def ACC(i, j):
    b = 4 * (8 * i + j)
    return f"a[{b}:{b + 3}]"


# m0_early: each piece's M0 is set one MFMA gap before its LDS-DMA (that gap also covers the M0 -> DMA wait
# state); 1.3 % faster over the step shapes than M0 + s_nop + DMA in one gap (profiles/r04/w4_variants_v1.log)
DEFAULT = dict(m0_early=True, sc1=True, a_slots=[24 + 4 * k for k in range(8)],
               b_slots=[64 + 5 * k for k in range(8)], bar2=108,
               # decompositions (ablation only, results invalid): vm_wait overrides barrier 2's vmcnt,
               # no_bar1 / no_bar2 drop those barriers (and bar1's lgkmcnt(0)), no_reads drops the fragment reads
               vm_wait=None, no_bar1=False, no_bar2=False, no_reads=False)


class Prog:
    def __init__(self, noload=False, opt=None):
        self.opt = dict(DEFAULT, **(opt or {}))
        self.lines = []
        self.lgkm = []        # outstanding LDS reads (dest register names), in issue order
        self.done = 0         # reads [0, done) of self.lgkm known complete
        self.noload = noload  # ablation: no LDS-DMA after the prologue (results invalid)

    def emit(self, s):
        self.lines.append(s)

    def read(self, kind, s, idx):
        if self.opt["no_reads"]:
            return
        reg = X(s, idx) if kind == "X" else Y(s, idx)
        base = ("%[rB" if kind == "X" else "%[rA") + f"{s}]"
        off = 2048 * idx
        self.emit(f"ds_read_b128 {reg}, {base}" + (f" offset:{off}" if off else ""))
        self.lgkm.append(reg)

    def need(self, regs):
        last = -1
        for n, r in enumerate(self.lgkm):
            if r in regs:
                last = n
        if last < self.done:
            return
        after = len(self.lgkm) - 1 - last
        n = min(after, 15)
        self.emit(f"s_waitcnt lgkmcnt({n})")
        self.done = len(self.lgkm) - n

    def wait_all_lgkm(self):
        self.emit("s_waitcnt lgkmcnt(0)")
        self.done = len(self.lgkm)

    def set_m0(self, op, k):
        off = (32768 if op == "B" else 0) + 4096 * k
        self.emit(f"s_add_u32 m0, %[sM], {off}")

    def piece(self, op, k, src, m0=True):
        """LDS-DMA piece k (0..7) of operand op ('A'/'B') of a K-tile into the current load stage (m0 base
        %[sM]); src 'm' (main operand, k offset %[sK]) or 'e0' / 'e1' (LoRA extension tile 0 / 1).
        m0=False: M0 was set one MFMA gap earlier (set_m0), which also covers the M0 -> LDS-DMA wait state."""
        if m0:
            self.set_m0(op, k)
            self.emit("s_nop 0")
        c = " sc1" if self.opt["sc1"] else ""
        if src == "m":
            self.emit(f"buffer_load_dwordx4 %[o{op}{k}], %[rs{op}], %[sK] offen{c} lds")
        else:
            so = "0" if src == "e0" else "%[sE1]"
            self.emit(f"buffer_load_dwordx4 %[e{op}{k}], %[rs{op}2], {so} offen{c} lds")

    def tile(self, first=False, load=None, has_next=True, vm_next=None, loop=None, stage=False):
        """One K-tile.  load: the source of the tile two ahead ('m', 'e0', 'e1') or None.  vm_next: the
        vmcnt that retires the next tile's pieces (pieces issued after them).  loop: label to branch back
        to while --%[cnt] != 0.  stage (the last tile of a staged program, round 5): once every wave has read
        the tile's fragments (a barrier at gap 24; no LDS-DMA is in flight in the last tile), each accumulator
        block is rounded to bf16 and written to the epilogue's LDS staging rows STAGE_LAG MFMAs after its final
        MFMA (64 + n for block n), in the MFMA gaps; the blocks whose slot falls past the tile are staged by
        epilogue(stage=True)."""
        if self.noload and not first:
            load = None
            vm_next = 0
        post = {k: [] for k in range(128)}
        pre = {k: [] for k in range(128)}
        # substep-1 fragments of this tile (stage t): gaps 0..15
        for n, (kind, idx) in enumerate(RD_ORDER):
            post[n].append(("read", kind, 1, idx))
        # read-base toggles: rA0/rB0 (substep 0, next tile) and rA1/rB1 (substep 1, next tile)
        post[18].append(("v_xor_b32 %[rA0], %[tA0], %[rA0]",))
        post[19].append(("v_xor_b32 %[rB0], %[tB0], %[rB0]",))
        post[20].append(("v_xor_b32 %[rA1], %[tA1], %[rA1]",))
        post[21].append(("v_xor_b32 %[rB1], %[tB1], %[rB1]",))
        if (load is not None and not self.opt["no_bar1"]) or stage:
            pre[24].append(("lgkm0",))
            pre[24].append(("s_barrier",))
        if stage:
            assert load is None and not has_next
            self.deferred = []
            for n in range(64):
                k = 64 + n + STAGE_LAG
                if k <= 127:
                    post[k].append(("stage", n))
                else:
                    self.deferred.append(n)
        if load is not None:
            early = self.opt["m0_early"]
            for op, slots in (("A", self.opt["a_slots"]), ("B", self.opt["b_slots"])):
                for k, sl in enumerate(slots):
                    if early:
                        post[sl - 1].append(("m0", op, k))
                    post[sl].append(("piece", op, k, load, not early))
            if load == "m":
                post[103].append(("s_add_u32 %[sK], %[sK], 128",))
        post[102].append(("s_xor_b32 %[sM], %[sM], %[sMT]",))
        if has_next:
            b2 = self.opt["bar2"]
            vw = vm_next if self.opt["vm_wait"] is None else self.opt["vm_wait"]
            pre[b2].append((f"s_waitcnt vmcnt({vw})",))
            if not self.opt["no_bar2"]:
                pre[b2].append(("s_barrier",))
            for n, (kind, idx) in enumerate(RD_ORDER):
                post[min(b2 + n, 127)].append(("read", kind, 0, idx))
        for k in range(128):
            for it in pre[k]:
                self._item(it)
            s, r = divmod(k, 64)
            i, j = divmod(r, 8)
            if j == 0:  # one wait per row of 8 blocks: fragment X(s, i) and every Y(s, *)
                self.need({X(s, i)} | {Y(s, jj) for jj in range(8)})
            self.need({X(s, i), Y(s, j)})
            c = "0" if (first and s == 0) else ACC(i, j)
            self.emit(f"{MFMA} {ACC(i, j)}, {X(s, i)}, {Y(s, j)}, {c}")
            for it in post[k]:
                self._item(it)
        if loop is not None:
            self.emit("s_sub_u32 %[cnt], %[cnt], 1")
            self.emit("s_cmp_lg_u32 %[cnt], 0")
            self.emit(f"s_cbranch_scc1 {loop}")

    def stage_block(self, n):
        """Block n = 8 i + j of the accumulators -> bf16 (v_cvt_pk_bf16_f32, RNE) -> the staging rows at %[sb] +
        8448 j + 32 i (w4_stage_bf16's layout and instructions, one block)."""
        i, j = divmod(n, 8)
        b = 120 + 4 * (n % 2)
        for e in range(4):
            self.emit(f"v_accvgpr_read_b32 v{b + e}, a{4 * n + e}")
        self.emit(f"v_cvt_pk_bf16_f32 v{b}, v{b}, v{b + 1}")
        self.emit(f"v_cvt_pk_bf16_f32 v{b + 1}, v{b + 2}, v{b + 3}")
        off = 8448 * j + 32 * i
        self.emit(f"ds_write_b64 %[sb], v[{b}:{b + 1}]" + (f" offset:{off}" if off else ""))

    def _item(self, it):
        if it[0] == "stage":
            self.stage_block(it[1])
            return
        if it[0] == "read":
            self.read(it[1], it[2], it[3])
        elif it[0] == "lgkm0":
            self.wait_all_lgkm()
        elif it[0] == "piece":
            self.piece(it[1], it[2], it[3], it[4] if len(it) > 4 else True)
        elif it[0] == "m0":
            self.set_m0(it[1], it[2])
        else:
            self.emit(it[0])

    def prologue(self, src0, src1):
        self.emit("s_mov_b32 %[sSave], m0")
        self.emit("s_nop 4")
        for t, src in ((0, src0), (1, src1)):
            for op in "AB":
                for k in range(8):
                    self.piece(op, k, src)
            if src == "m":
                self.emit("s_add_u32 %[sK], %[sK], 128")
            self.emit("s_xor_b32 %[sM], %[sM], %[sMT]")
        self.emit("s_waitcnt vmcnt(16)")
        self.emit("s_barrier")
        for kind, idx in RD_ORDER:
            self.read(kind, 0, idx)

    def mask_pass(self):
        """Dropout on the extension product held in the accumulators: acc *= keep ? scale : 0.
        Mask word %[mk<j>] bit 4i+e keeps element e of block (i, j)."""
        self.emit("s_nop 15")
        self.emit("s_nop 15")
        for i in range(8):
            for j in range(8):
                for e in range(4):
                    a = f"a{4 * (8 * i + j) + e}"
                    self.emit(f"v_accvgpr_read_b32 v120, {a}")
                    self.emit(f"v_bfe_i32 v121, %[mk{j}], {4 * i + e}, 1")
                    self.emit("v_mul_f32 v120, %[dsc], v120")
                    self.emit("v_and_b32 v120, v121, v120")
                    self.emit(f"v_accvgpr_write_b32 {a}, v120")
        self.emit("s_nop 7")

    def epilogue(self, stage=False):
        self.emit("s_waitcnt vmcnt(0) lgkmcnt(0)")
        self.emit("s_nop 15")
        self.emit("s_nop 15")
        if stage:  # the blocks whose staging slot fell past the last MFMA, then every staging write retired
            for n in self.deferred:
                self.stage_block(n)
            self.emit("s_waitcnt lgkmcnt(0)")
        self.emit("s_barrier")
        self.emit("s_mov_b32 m0, %[sSave]")


def prog_plain(E, noload=False, opt=None, stage=False):
    p = Prog(noload, opt)
    p.prologue("m", "m")
    p.tile(first=True, load="m", vm_next=16)
    p.emit("L_w4loop_%=:")
    p.tile(load="m", vm_next=16, loop="L_w4loop_%=")
    # tail: main tiles nm-2, nm-1, then the E extension tiles; loads of the tile two ahead
    seq = ["m", "m"] + ["e0", "e1"][:E]
    for n in range(len(seq)):
        ld = seq[n + 2] if n + 2 < len(seq) else None
        nxt = n + 1 < len(seq)
        p.tile(load=ld, has_next=nxt, vm_next=(16 if ld else 0), stage=stage and not nxt)
    p.epilogue(stage)
    return p


def prog_drop(E, noload=False, stage=False):
    p = Prog(noload)
    seq0 = ["e0", "e1"][:E] + ["m", "m"]
    p.prologue(seq0[0], seq0[1])
    for n in range(E):
        p.tile(first=(n == 0), load=seq0[n + 2], vm_next=16)
    p.mask_pass()
    p.emit("L_w4loop_%=:")
    p.tile(load="m", vm_next=16, loop="L_w4loop_%=")
    p.tile(load=None, has_next=True, vm_next=0)
    p.tile(load=None, has_next=False, stage=stage)
    p.epilogue(stage)
    return p


# ------------------------------------------------------------------------------------------------------
# MXFP8 programs (gemm_nt_w4_kernel<.., MX = true>): main K-tiles of 128 e4m3 per row (the same 128-B LDS
# rows as a bf16 K-tile) run 64 v_mfma_scale_f32_16x16x128_f8f6f4 per tile, one per 16 x 16 block; the
# LoRA extension tiles (bf16) run 128 v_mfma_f32_16x16x32_bf16 as in the bf16 programs.  A fragment is the
# lo (16-B chunk g) and hi (chunk 4 + g) halves of its 16 rows = the bf16 substep-0 and substep-1 fragments,
# so both tile kinds share one read pattern and one register map:
#   X_i = v[128 + 8 i .. +7] (B rows wn*128 + 16 i, srcA), Y_j = v[192 + 8 j .. +7] (A rows, srcB);
#   E8M0 scale words sX0 v112, sX1 v113 (B blocks 2 wn, 2 wn + 1), sY0 v114, sY1 v115 (A blocks), byte
#   (i & 3) / (j & 3) picked by op_sel / op_sel_hi.
# With a whole tile of fragments in 128 VGPRs there is no room for a second copy, so the next tile's
# fragments replace the current ones as they retire.  MFMA order: half 0 (X_0..3 x every Y_j), then half 1
# (X_4..7 x every Y_j), so X_0..3 retire at MFMA 31, Y_j at 35 + 4 j, X_4..7 at 60..63:
#   gaps 30..37: X_0..3 of tile t+1; 37 + 4 j: Y_j of t+1 (j < 7); gaps 1..10 of t+1: Y_7, X_4..7 and the
#   scale words sX1 / sY1 of t+1 (sX0 at gap 33, sY0 at gap 50 of t: their last uses are 31 / 47).
# Every read lands >= 2 MFMAs after the last use of its registers.  Barrier 1 (gap 11) frees tile t's stage
# (its last reads were X_4..7 / scales at gaps 2..9); tile t+2's 16 pieces (+ 2 scale pieces) follow at
# gaps 13..30; barrier 2 (gap 29) retires tile t+1's pieces (vmcnt = the t+2 pieces already issued).
# Accumulation order per output element: main tiles in order, then the extension tiles (substep 0, 1) --
# that of gemm_nt_v5_kernel<.., MX = true>, so the results are bit-identical to it.
MX_MFMA = "v_mfma_scale_f32_16x16x128_f8f6f4"


def XM(i, h=None):
    b = 128 + 8 * i
    return f"v[{b}:{b + 7}]" if h is None else f"v[{b + 4 * h}:{b + 4 * h + 3}]"


def YM(j, h=None):
    b = 192 + 8 * j
    return f"v[{b}:{b + 7}]" if h is None else f"v[{b + 4 * h}:{b + 4 * h + 3}]"


SX = ["v112", "v113"]
SY = ["v114", "v115"]


class ProgMX(Prog):
    def __init__(self):
        super().__init__(False, None)

    def rd_frag(self, kind, idx, h):
        reg = XM(idx, h) if kind == "X" else YM(idx, h)
        base = ("%[rB" if kind == "X" else "%[rA") + f"{h}]"
        off = 2048 * idx
        self.emit(f"ds_read_b128 {reg}, {base}" + (f" offset:{off}" if off else ""))
        self.lgkm.append(reg)

    def rd_scale(self, kind, w):
        reg = (SX if kind == "X" else SY)[w]
        base = "%[rSX]" if kind == "X" else "%[rSY]"
        self.emit(f"ds_read_b32 {reg}, {base}" + (" offset:256" if w else ""))
        self.lgkm.append(reg)

    def scale_piece(self, op):
        """The E8M0 scale block of this wave (A: rows block m0/64 + wave; B: n0/64 + wave) of the tile two ahead:
        one 4-B LDS-DMA per lane into the scale stage (M0 = %[sMS] (+1024 for B))."""
        self.emit(f"s_add_u32 m0, %[sMS], {1024 if op == 'B' else 0}")
        self.emit("s_nop 0")
        self.emit(f"buffer_load_dword %[oS{op}], %[rsS{op}], %[sKS] offen sc1 lds")

    @staticmethod
    def order(kind):
        """MFMA list of a tile: (i, j, h) with h = None (MX) or the bf16 substep."""
        seq = []
        for h in ([None] if kind == "x" else [0, 1]):
            for half in (0, 1):
                for j in range(8):
                    for i in range(4 * half, 4 * half + 4):
                        seq.append((i, j, h))
        return seq

    def tile(self, kind, first=False, load=None, load_kind=None, nxt=None, loop=None):
        """kind 'x' (MX main tile) or 'b' (bf16 extension tile).  load: source of the tile two ahead ('m', 'e0',
        'e1') or None, load_kind its kind; nxt: the next tile's kind (None: last tile)."""
        seq = self.order(kind)
        G = len(seq)
        sc = 1 if kind == "x" else 2  # gap scale: the bf16 tile's last-use pattern sits in its substep 1
        off = 0 if kind == "x" else 64
        post = {k: [] for k in range(G)}
        pre = {k: [] for k in range(G)}
        if not first:  # Y_7, X_4..7 (and sX1 / sY1 for an MX tile) of THIS tile, from its stage: their registers
            # retired with the previous tile's last MFMAs (>= 2 MFMAs back)
            post[1].append(("frag", "Y", 7, 0))
            post[2].append(("frag", "Y", 7, 1))
            for n, i in enumerate(range(4, 8)):
                post[3 + 2 * n].append(("frag", "X", i, 0))
                post[4 + 2 * n].append(("frag", "X", i, 1))
            if kind == "x":
                post[2].append(("scale", "X", 1))
                post[3].append(("scale", "Y", 1))
        # barrier 1: this tile's stage is free (every wave's reads of it are done) -> tile t+2's pieces
        if load is not None:
            pre[11].append(("lgkm0",))
            pre[11].append(("s_barrier",))
        post[12].append(("v_xor_b32 %[rA0], %[tA0], %[rA0]",))
        post[12].append(("v_xor_b32 %[rB0], %[tB0], %[rB0]",))
        post[13].append(("v_xor_b32 %[rA1], %[tA1], %[rA1]",))
        post[13].append(("v_xor_b32 %[rB1], %[tB1], %[rB1]",))
        post[14].append(("v_xor_b32 %[rSX], %[tSX], %[rSX]",))
        post[14].append(("v_xor_b32 %[rSY], %[tSY], %[rSY]",))
        npieces = 0
        if load is not None:
            slots = list(range(13, 29))
            for n, (op, k) in enumerate([("A", k) for k in range(8)] + [("B", k) for k in range(8)]):
                post[slots[n] - 1].append(("m0", op, k))
                post[slots[n]].append(("piece", op, k, load, False))
            npieces = 16
            if load_kind == "x":
                post[29].append(("spiece", "A"))
                post[30].append(("spiece", "B"))
                post[31].append(("s_add_u32 %[sKS], %[sKS], 256",))
            if load == "m":
                post[31].append(("s_add_u32 %[sK], %[sK], 128",))
            post[32].append(("s_xor_b32 %[sM], %[sM], %[sMT]",))
            post[32].append(("s_xor_b32 %[sMS], %[sMS], %[sMST]",))
        if nxt is not None:
            # barrier 2: the next tile's pieces (issued during the previous tile) retired in every wave
            pre[off + 29].append((f"s_waitcnt vmcnt({npieces})",))
            pre[off + 29].append(("s_barrier",))
            reads = {}
            for i in range(4):  # X_0..3 of the next tile, after their last use (MFMA 28 + i)
                reads.setdefault(off + 30 + 2 * i, []).append(("frag", "X", i, 0))
                reads.setdefault(off + 31 + 2 * i, []).append(("frag", "X", i, 1))
            for j in range(7):  # Y_j, after its last use 35 + 4 j
                reads.setdefault(off + 37 + 4 * j, []).append(("frag", "Y", j, 0))
                reads.setdefault(off + 38 + 4 * j, []).append(("frag", "Y", j, 1))
            if nxt == "x":
                reads.setdefault(off + 33, []).append(("scale", "X", 0))
                reads.setdefault(off + 50, []).append(("scale", "Y", 0))
            for k, its in reads.items():
                post[k].extend(its)
        for k, (i, j, h) in enumerate(seq):
            for it in pre[k]:
                self._item(it)
            if h is None:
                self.need({XM(i, 0), XM(i, 1), YM(j, 0), YM(j, 1), SX[i >> 2], SY[j >> 2]})
                c = "0" if first else ACC(i, j)
                bi, bj = i & 3, j & 3
                self.emit(f"{MX_MFMA} {ACC(i, j)}, {XM(i)}, {YM(j)}, {c}, {SX[i >> 2]}, {SY[j >> 2]} "
                          f"op_sel:[{bi & 1},{bj & 1},0] op_sel_hi:[{bi >> 1},{bj >> 1},0]")
            else:
                self.need({XM(i, h), YM(j, h)})
                c = "0" if (first and h == 0) else ACC(i, j)
                self.emit(f"{MFMA} {ACC(i, j)}, {XM(i, h)}, {YM(j, h)}, {c}")
            for it in post[k]:
                self._item(it)
        if loop is not None:
            self.emit("s_sub_u32 %[cnt], %[cnt], 1")
            self.emit("s_cmp_lg_u32 %[cnt], 0")
            self.emit(f"s_cbranch_scc1 {loop}")

    def _item(self, it):
        if it[0] == "frag":
            self.rd_frag(it[1], it[2], it[3])
        elif it[0] == "scale":
            self.rd_scale(it[1], it[2])
        elif it[0] == "spiece":
            self.scale_piece(it[1])
        else:
            super()._item(it)

    def prologue_mx(self):
        """Tiles 0 and 1 (both main) into stages 0 / 1 with their scales; every fragment and scale word of
        tile 0 read."""
        self.emit("s_mov_b32 %[sSave], m0")
        self.emit("s_nop 4")
        for _ in range(2):
            for op in "AB":
                for k in range(8):
                    self.piece(op, k, "m")
            self.scale_piece("A")
            self.scale_piece("B")
            self.emit("s_add_u32 %[sK], %[sK], 128")
            self.emit("s_add_u32 %[sKS], %[sKS], 256")
            self.emit("s_xor_b32 %[sM], %[sM], %[sMT]")
            self.emit("s_xor_b32 %[sMS], %[sMS], %[sMST]")
        self.emit("s_waitcnt vmcnt(18)")
        self.emit("s_barrier")
        for i in range(8):
            self.rd_frag("X", i, 0)
            self.rd_frag("X", i, 1)
        for j in range(8):
            self.rd_frag("Y", j, 0)
            self.rd_frag("Y", j, 1)
        for w in range(2):
            self.rd_scale("X", w)
            self.rd_scale("Y", w)


def prog_mx(E):
    """MX main tiles (nm >= 4) then E bf16 extension tiles.  Loop over main tiles 1 .. nm-3."""
    p = ProgMX()
    p.prologue_mx()
    p.tile("x", first=True, load="m", load_kind="x", nxt="x")
    p.emit("L_w4mx_%=:")
    p.tile("x", load="m", load_kind="x", nxt="x", loop="L_w4mx_%=")
    seq = [("m", "x"), ("m", "x")] + [("e0", "b"), ("e1", "b")][:E]
    for n in range(len(seq)):
        ld = seq[n + 2] if n + 2 < len(seq) else None
        nk = seq[n + 1][1] if n + 1 < len(seq) else None
        p.tile(seq[n][1], load=ld[0] if ld else None, load_kind=ld[1] if ld else None, nxt=nk)
    p.epilogue()
    return p


HEADER = """// GENERATED by gen_gemm_w4.py -- do not edit.  The hand-placed K-loop programs of gemm_nt_w4_kernel
// (gemm_w4.h): see the generator's docstring for the schedule.
"""


def asm_fn(name, prog, drop, stage=False):
    outs = ['[sSave] "=&s"(o.save)', '[cnt] "+s"(o.cnt)', '[sK] "+s"(o.sK)', '[sM] "+s"(o.sM)',
            '[rA0] "+v"(o.rA0)', '[rA1] "+v"(o.rA1)', '[rB0] "+v"(o.rB0)', '[rB1] "+v"(o.rB1)']
    ins = ['[rsA] "s"(o.rsA)', '[rsB] "s"(o.rsB)', '[rsA2] "s"(o.rsA2)', '[rsB2] "s"(o.rsB2)',
           '[sE1] "s"(o.sE1)', '[sMT] "s"(o.sMT)',
           '[tA0] "v"(o.tA0)', '[tA1] "v"(o.tA1)', '[tB0] "v"(o.tB0)', '[tB1] "v"(o.tB1)']
    ins += [f'[oA{k}] "v"(o.oA[{k}])' for k in range(8)] + [f'[oB{k}] "v"(o.oB[{k}])' for k in range(8)]
    ins += [f'[eA{k}] "v"(o.eA[{k}])' for k in range(8)] + [f'[eB{k}] "v"(o.eB[{k}])' for k in range(8)]
    if drop:
        ins += [f'[mk{j}] "v"(o.mk[{j}])' for j in range(8)] + ['[dsc] "s"(o.dsc)']
    if stage:
        ins += ['[sb] "v"(o.sb)']
    scratch = range(120, 128) if stage else (120, 121)
    clob = ['"memory"', '"scc"'] + [f'"v{r}"' for r in scratch] + [f'"v{r}"' for r in range(128, 256)] + \
        [f'"a{r}"' for r in range(256)]
    body = "\n".join(f'      "{l}\\n"' for l in prog.lines)
    return (f"__device__ __forceinline__ void {name}(W4Ops& o) {{\n  asm volatile(\n{body}\n"
            f"      : {', '.join(outs)}\n      : {', '.join(ins)}\n      : {', '.join(clob)});\n}}\n")


def asm_fn_mx(name, prog):
    outs = ['[sSave] "=&s"(o.save)', '[cnt] "+s"(o.cnt)', '[sK] "+s"(o.sK)', '[sM] "+s"(o.sM)',
            '[sKS] "+s"(o.sKS)', '[sMS] "+s"(o.sMS)',
            '[rA0] "+v"(o.rA0)', '[rA1] "+v"(o.rA1)', '[rB0] "+v"(o.rB0)', '[rB1] "+v"(o.rB1)',
            '[rSX] "+v"(o.rSX)', '[rSY] "+v"(o.rSY)']
    ins = ['[rsA] "s"(o.rsA)', '[rsB] "s"(o.rsB)', '[rsA2] "s"(o.rsA2)', '[rsB2] "s"(o.rsB2)',
           '[rsSA] "s"(o.rsSA)', '[rsSB] "s"(o.rsSB)',
           '[sE1] "s"(o.sE1)', '[sMT] "s"(o.sMT)', '[sMST] "s"(o.sMST)',
           '[tA0] "v"(o.tA0)', '[tA1] "v"(o.tA1)', '[tB0] "v"(o.tB0)', '[tB1] "v"(o.tB1)',
           '[tSX] "v"(o.tSX)', '[tSY] "v"(o.tSY)', '[oSA] "v"(o.oSA)', '[oSB] "v"(o.oSB)']
    ins += [f'[oA{k}] "v"(o.oA[{k}])' for k in range(8)] + [f'[oB{k}] "v"(o.oB[{k}])' for k in range(8)]
    ins += [f'[eA{k}] "v"(o.eA[{k}])' for k in range(8)] + [f'[eB{k}] "v"(o.eB[{k}])' for k in range(8)]
    clob = ['"memory"', '"scc"'] + [f'"v{r}"' for r in range(112, 256)] + [f'"a{r}"' for r in range(256)]
    body = "\n".join(f'      "{l}\\n"' for l in prog.lines)
    return (f"__device__ __forceinline__ void {name}(W4Ops& o) {{\n  asm volatile(\n{body}\n"
            f"      : {', '.join(outs)}\n      : {', '.join(ins)}\n      : {', '.join(clob)});\n}}\n")


# ablation schedule variants (gemm_nt_w4_kernel<false, DBG, V>, library variants 42..)
ABL_VARIANTS = {
    1: dict(m0_early=False),
    2: dict(sc1=False),
    3: dict(m0_early=True, a_slots=[25 + 3 * k for k in range(8)], b_slots=[49 + 3 * k for k in range(8)]),
    4: dict(m0_early=True, a_slots=[25 + 3 * k for k in range(8)], b_slots=[49 + 3 * k for k in range(8)], bar2=112),
    5: dict(a_slots=[26, 26, 34, 34, 42, 42, 50, 50], b_slots=[66, 66, 74, 74, 82, 82, 90, 90]),
    6: dict(vm_wait=63),      # decomposition: no wait for the next tile's pieces
    7: dict(no_bar1=True),    # decomposition: no barrier 1
    8: dict(no_bar2=True),    # decomposition: no barrier 2
    9: dict(no_reads=True),   # decomposition: no fragment reads
}


def acc_reader():
    """w4_acc(N): accumulator block N (= 8 i + j) of a[0:255] as f32x4; N folds to a constant."""
    cases = []
    for n in range(64):
        b = 4 * n
        cases.append(f'    case {n}: asm volatile("v_accvgpr_read_b32 %0, a{b}\\n\\tv_accvgpr_read_b32 %1, a{b + 1}\\n\\t'
                     f'v_accvgpr_read_b32 %2, a{b + 2}\\n\\tv_accvgpr_read_b32 %3, a{b + 3}" '
                     f': "=v"(x), "=v"(y), "=v"(z), "=v"(w)); break;')
    return ("__device__ __forceinline__ f32x4 w4_acc(int n) {\n  float x = 0.f, y = 0.f, z = 0.f, w = 0.f;\n"
            "  switch (n) {\n" + "\n".join(cases) + "\n    default: break;\n  }\n  return f32x4{x, y, z, w};\n}\n")


def acc_writer():
    """w4_acc_set(N, v): accumulator block N of a[0:255] := v (round 5: the in-launch split-K combine writes the
    summed tile back before the epilogue); N folds to a constant.  The trailing s_nop keeps a later
    v_accvgpr_read of the same registers clear of the write."""
    cases = []
    for n in range(64):
        b = 4 * n
        cases.append(f'    case {n}: asm volatile("v_accvgpr_write_b32 a{b}, %0\\n\\tv_accvgpr_write_b32 a{b + 1}, %1\\n\\t'
                     f'v_accvgpr_write_b32 a{b + 2}, %2\\n\\tv_accvgpr_write_b32 a{b + 3}, %3\\n\\ts_nop 1" '
                     f':: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a{b}", "a{b + 1}", "a{b + 2}", "a{b + 3}"); break;')
    return ("__device__ __forceinline__ void w4_acc_set(int n, const f32x4& v) {\n  switch (n) {\n" + "\n".join(cases) +
            "\n    default: break;\n  }\n}\n")


def stage_fn():
    """w4_stage_bf16: every accumulator block rounded to bf16 (v_cvt_pk_bf16_f32, RNE, as the C++ epilogue's
    pack2) and written to the epilogue's LDS staging rows (ml * 528 + nl * 2; %[sb] = this lane's block-(0,0)
    address, block (i, j) at +8448 j + 32 i).  The plain epilogue (alpha 1, no bias): 7 instructions per block
    instead of the compiler's ~16 (one wave per SIMD: every VALU instruction costs its full issue)."""
    lines = []
    for n in range(64):
        i, j = divmod(n, 8)
        b = 120 + 4 * (n % 2)
        for e in range(4):
            lines.append(f"v_accvgpr_read_b32 v{b + e}, a{4 * n + e}")
        lines.append(f"v_cvt_pk_bf16_f32 v{b}, v{b}, v{b + 1}")
        lines.append(f"v_cvt_pk_bf16_f32 v{b + 1}, v{b + 2}, v{b + 3}")
        off = 8448 * j + 32 * i
        lines.append(f"ds_write_b64 %[sb], v[{b}:{b + 1}]" + (f" offset:{off}" if off else ""))
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    clob = ", ".join(['"memory"'] + [f'"v{r}"' for r in range(120, 128)])
    return ("__device__ __forceinline__ void w4_stage_bf16(uint32_t sb) {\n  asm volatile(\n" + body +
            f"\n      :\n      : [sb] \"v\"(sb)\n      : {clob});\n}}\n")


def main(out):
    parts = [HEADER, acc_reader(), acc_writer(), stage_fn()]
    for E in (0, 1, 2):
        parts.append(asm_fn(f"w4_plain{E}", prog_plain(E), False))
    for E in (1, 2):
        parts.append(asm_fn(f"w4_drop{E}", prog_drop(E), True))
    for E in (0, 1, 2):
        parts.append(asm_fn_mx(f"w4_mx{E}", prog_mx(E)))
    parts.append("#ifdef OSPO_ABLATION\n// decomposition (results invalid): no LDS-DMA after the prologue\n")
    # round 5, measured and rejected (same bytes, 0.3 % slower in the step: profiles/r05/gemm_epi_ab.log,
    # bench_ab_r5c_hash_*.json): the plain bf16 epilogue's staging inside the last tile's MFMA gaps
    parts.append("// staged programs (OSPO_GEMM_EPI=10)\n")
    for E in (0, 1, 2):
        parts.append(asm_fn(f"w4_plain{E}_st", prog_plain(E, stage=True), False, stage=True))
    for E in (1, 2):
        parts.append(asm_fn(f"w4_drop{E}_st", prog_drop(E, stage=True), True, stage=True))
    parts.append(asm_fn("w4_plain0_noload", prog_plain(0, noload=True), False))
    parts.append("// schedule variants for A/B (w4v<V>_plain<E>, bf16 without dropout)\n")
    for v, opt in ABL_VARIANTS.items():
        for E in (0, 1, 2):
            parts.append(asm_fn(f"w4v{v}_plain{E}", prog_plain(E, opt=opt), False))
    parts.append("#endif\n")
    with open(out, "w") as f:
        f.write("".join(parts))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gemm_w4_asm.inc")
