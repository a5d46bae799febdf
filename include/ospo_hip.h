/*
 * libospo_hip.so -- C ABI of the MI355X-native (gfx950 / CDNA4) SimPO training
 * path for Janus-Pro (OSPO step 5).  Plain pointers, sizes and a hipStream_t;
 * no framework types.  Every function validates shapes/alignment BEFORE any
 * launch and returns an ospo_status (0 = OK).  The library allocates nothing:
 * every buffer (workspaces included) is owned by the caller.  All work is
 * enqueued asynchronously on `stream`; no function synchronises the host.
 *
 * Each entry point names the reference interface it replaces (file:line under
 * the reference tree OSPO-NeurIPS2025/OSPO; "HF" = transformers 4.38.2 Llama,
 * "peft" = peft 0.7.1 lora.Linear, both upstream of the reference).
 *
 * Conventions: bf16 = IEEE bfloat16 (2 bytes), row-major, leading dimensions in
 * ELEMENTS.  Token rows of a batch are laid out sequence-major: row = s*T + t.
 */
#ifndef OSPO_HIP_H
#define OSPO_HIP_H

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  OSPO_OK = 0,
  OSPO_ERR_SHAPE = 1,       /* shape / leading-dimension / tile-multiple violation */
  OSPO_ERR_ALIGN = 2,       /* pointer not 16-byte aligned where required */
  OSPO_ERR_HIP = 3,         /* launch failed (hipGetLastError) */
  OSPO_ERR_UNSUPPORTED = 4, /* configuration not built */
  OSPO_ERR_ARG = 5          /* bad scalar argument (loss type, null pointer) */
} ospo_status;

const char* ospo_strerror(int status);

/* ABI revision; bumped whenever a signature, a workspace layout or the dropout masks a seed produces change.
 * 2 (round 6): ospo_lora_gdb's partials sit behind a zero-at-allocation counter head (OSPO_WS_LORA_GDB), the
 * round-5 dropout hash (new masks for every seed), ospo_ws_counter_bytes and ospo_gemm_clock_probe_bf16.
 * 3 (round 6): ospo_lora_gdb_r / ospo_swiglu_lora_gdb_r (LoRA rank 16 or 32; the rank-16 entry points are
 * their r = 16 forms).
 * Bindings check it when they load the library (ospo_amd/_lib.py). */
#define OSPO_ABI_VERSION 3
int ospo_abi_version(void);

/* Box probe (measurement aid, no reference counterpart): C = A . B^T with the product's bf16 256 x 256 K loop,
 * unsplit, M % 256 == N % 256 == 0, K % 64 == 0, K >= 256, each 256 x 256 tile's workgroup writing 8 uint64
 * stamps (stamps_bytes >= (M/256)(N/256) * 64): [0] s_memtime at the K loop's start, [1] s_memrealtime at entry,
 * [2] s_memrealtime at the loop's start, [3] s_memtime and [4] s_memrealtime at its end, [5..7] s_memrealtime
 * after the epilogue's staging, store issue and drain.  In-kernel clock = ([3]-[0]) / ([4]-[2]) x 100 MHz. */
int ospo_gemm_clock_probe_bf16(const void* A, const void* B, void* C, int M, int N, int K, void* stamps,
                               size_t stamps_bytes, hipStream_t stream);

/* Counter heads at the START of a caller-owned workspace: they must be zero when the workspace is allocated and
 * every call leaves them zero again (a host-side reset after an aborted stream zeroes exactly this many bytes). */
typedef enum {
  OSPO_WS_GEMM_TAIL = 0,      /* 4 KiB at the END of a split-K workspace, read only by the ablation build's
                                 in-launch combine (the product library ignores them) */
  OSPO_WS_SKINNY = 1,         /* ospo_lora_skinny / ospo_swiglu_fwd_lora_down: 4 KiB of row-block counters */
  OSPO_WS_LORA_GDB = 2,       /* ospo_lora_gdb / ospo_swiglu_lora_gdb: 8 KiB of column-block counters + 16 B */
  OSPO_WS_DECODE_LINEAR = 3   /* ospo_decode_linear / ospo_decode_mlp / ospo_decode_attn_o: 4 KiB */
} ospo_ws_kind;
#define OSPO_WS_GEMM_TAIL_CNT_BYTES 4096
#define OSPO_WS_SKINNY_CNT_BYTES 4096
#define OSPO_WS_LORA_GDB_CNT_BYTES (8192 + 16)
#define OSPO_WS_DECODE_LINEAR_CNT_BYTES 4096
/* bytes of that head (0 for an unknown kind) */
size_t ospo_ws_counter_bytes(int kind);

/* ------------------------------------------------------------------ GEMM ---
 * Linear layers of the Llama decoder with fused peft LoRA (peft lora.Linear
 * .forward, reached from ospo/utils/model.py:50-60; call sites HF
 * LlamaAttention/LlamaMLP q,k,v,o,gate,up,down) and the frozen Linear layers
 * of gen_head (janus/models/modeling_vlm.py:47-51) / gen_aligner
 * (janus/models/projector.py:39-45).
 *
 * C[M,N] (bf16) = round( alpha * (A[M,K] . B[N,K]^T + A2[M,K2] . B2[N,K2]^T) + bias[N] )
 *                 [+ residual[M,N], added after rounding and rounded again]
 * A, A2 row-major with K contiguous; B, B2 row-major with K contiguous (the
 * nn.Linear weight layout [out,in]).  A2/B2 is the LoRA K-extension
 * (A2 = scaling * lora_A(x), B2 = block-diagonal lora_B), may be NULL (K2 = 0).
 * Requires N % 256 == 0 (or N % 64 == 0 for N <= 256), K % 64 == 0, K2 % 64 == 0;
 * M arbitrary.  MFMA bf16 (v_mfma_f32_16x16x32_bf16), fp32 accumulation.
 *
 * Split-K tail (every 256x256 GEMM entry point below): the tiles of the last, partial
 * round (tiles % CUs) may be split along K into fp32 partial tiles that a fixup launch sums
 * and epilogues.  ws (16-B aligned, >= ospo_gemm_nt_ws_bytes(M, N, K, K2, mx, tail_split)
 * bytes) holds the partials; NULL or too small = no split.  The caller owns it; calls
 * sharing a ws must be stream-ordered.  tail_split: 0 = the library's cost model, 1 = never
 * split, 2..8 = that split (bounded by one round of pieces and K / 4 K-tiles per piece).
 * The split changes the order of the fp32 sum only.  Partials use whole 256-KiB tiles of ws
 * only (bytes past them are left alone). */
int ospo_gemm_nt_bf16(const void* A, int lda, const void* B, int ldb, int M, int N, int K,
                      const void* A2, int lda2, const void* B2, int ldb2, int K2, float alpha,
                      const void* bias, const void* residual, int ldr, void* C, int ldc,
                      int tail_split, void* ws, size_t ws_bytes, hipStream_t stream);
/* Bytes of split-K workspace a 256x256 GEMM of this shape uses (0: no split); mx = 1 for
 * ospo_gemm_nt_mx8 (K in fp8 elements). */
size_t ospo_gemm_nt_ws_bytes(int M, int N, int K, int K2, int mx, int tail_split);

/* ospo_gemm_nt_bf16 (alpha 1, no bias / residual, N % 256 == 0) with the RoPE
 * forward (ospo_rope_fwd semantics: HF rotate-half, bf16 rounding per op) fused
 * into the epilogue for output columns < rope_cols (a multiple of the 128-wide
 * head; q|k of the fused qkv projection), position = row % T.  rope_cos/sin are
 * the bf16 [T][64] tables.  Replaces q_proj/k_proj + apply_rotary_pos_emb
 * (transformers 4.38 modeling_llama.py, reached from ospo/wrapper/train.py:352). */
int ospo_gemm_nt_rope_bf16(const void* A, int lda, const void* B, int ldb, int M, int N, int K,
                           const void* A2, int lda2, const void* B2, int ldb2, int K2, void* C, int ldc,
                           const void* rope_cos, const void* rope_sin, int T, int rope_cols,
                           int tail_split, void* ws, size_t ws_bytes, hipStream_t stream);

/* LoRA-dropout backward of a frozen Linear with its adapter (peft lora.Linear,
 * dropout before lora_A): C = A.B^T + mask (.) (A2.B2^T) / (1 - drop_p), with
 * the forward's mask over the [M, N] input of the adapter (element idx = m*N + n kept
 * iff the 16-bit half (idx & 1) of drop_hash(idx >> 1, drop_seed) is >= drop_p * 2^16, common.h), i.e.
 * dX = dy.W + dropout'(g . A_cat).  N % 256 == 0, K2 > 0, no bias / residual.
 * keep_bits (optional, 16-B aligned): that mask as the forward's ospo_lora_skinny keep-bit output
 * ([M][N / 8] bytes) -- read instead of re-hashed (same result). */
int ospo_gemm_nt_dropout_bf16(const void* A, int lda, const void* B, int ldb, int M, int N, int K,
                              const void* A2, int lda2, const void* B2, int ldb2, int K2, void* C, int ldc,
                              unsigned drop_seed, float drop_p, const void* keep_bits, int tail_split, void* ws,
                              size_t ws_bytes, hipStream_t stream);

/* down_proj backward fused with the SwiGLU backward (replaces ospo_gemm_nt_dropout_bf16 into dh +
 * ospo_swiglu_bwd; the autograd of `down_proj(act_fn(gate_proj(x)) * up_proj(x))` in HF
 * LlamaMLP.forward, reached from ospo/wrapper/train.py:352-354).  dh = bf16(A.B^T + mask (.) A2.B2^T
 * / (1 - p)) [M, F] is never stored: the epilogue reads gate | up from gu [M, 2F] and writes
 * [dgate | dup] to dgu [M, 2F], bit-identical to the two-launch path.  drop_p = 0: no mask
 * (K2 may be 0).  F % 256 == 0. */
int ospo_gemm_nt_swiglu_bwd_bf16(const void* A, int lda, const void* B, int ldb, int M, int F, int K,
                                 const void* A2, int lda2, const void* B2, int ldb2, int K2,
                                 const void* gu, int ld_gu, void* dgu, int ld_dgu, unsigned drop_seed,
                                 float drop_p, int tail_split, void* ws, size_t ws_bytes, hipStream_t stream);

/* The LoRA dropout mask hash (host copy of the device function): element idx of an
 * adapter input is kept iff the 16-bit half (idx & 1) of ospo_dropout_hash(idx >> 1, seed)
 * is >= p * 2^16 (one hash per two adjacent elements; adapter input widths are even). */
unsigned ospo_dropout_hash(unsigned idx, unsigned seed);

/* Row count of the tile ospo_gemm_nt_bf16 uses for an M x N output (256 or 64). */
int ospo_gemm_nt_tile(int M, int N);

/* C[M,N] (fp32) += alpha * op(A)[M,K] . op(B)[N,K]^T, split over K into
 * `k_splits` workgroup slices summed with fp32 atomics (C must be initialised).
 * a_kmajor = 0: A stored [M][K] (lda >= K); 1: A stored [K][M] (lda >= M).
 * b_kmajor = 0: B stored [N][K];            1: B stored [K][N].
 * Used for the LoRA down-projections u = x.A^T / g = dy.B (skinny N) and the
 * LoRA weight gradients dA = g^T.x, dB = dy^T.u (both operands K-major).
 * diag_nblk > 0 selects the block-diagonal scatter of a packed dB:
 * element (n, j) is kept only when j / diag_r == n / diag_nblk and lands at
 * C + n*diag_r + (j % diag_r)  (ldc ignored) -- peft B_q|B_k|B_v contiguous.
 * Requires K % 64 == 0; N % 64 == 0; M arbitrary (stores predicated on m < M; a
 * K-major A must have lda >= roundup(M, 64) readable columns). */
/* LoRA weight gradients (autograd of peft lora.Linear: dA = g^T . dropout(x), dB = dy^T . u) as one
 * stream over the big operand X [K][N] (row-major, ldx), contracting over its K rows (tokens) against the
 * small S [K][lds] (lds = the padded rank width, 64 or 128), fp32 atomics into C:
 *   mode 0 (dA): C[j * ldc + n] += sum_k S[k][j] X[k][n]           j < s_cols, N % 256 == 0
 *   mode 1 (dB): C[n * r + jr]  += sum_k X[k][n] S[k][(n / nmod) * r + jr]   (block diagonal; r 16 or 32)
 * K % 64 == 0 (rows past the real tokens must hold zeros in S); splits = K-range splits (<= K / 64).
 * drop_p > 0 (mode 0): X is masked as ospo_lora_skinny masked it in the forward (index k * N + n). */
int ospo_lora_wgrad(const void* X, int ldx, int N, const void* S, int lds, int s_cols, int K, int mode, int nmod,
                    int r, float* C, int ldc, int splits, uint32_t drop_seed, float drop_p, hipStream_t stream);
/* dA of one adapter group (peft lora_A.weight.grad of the q|k|v, o, gate|up or down adapters reached from
 * ospo/wrapper/train.py:352; replaces the K-major ospo_gemm_f32acc(_bdrop) product):
 *   C[j * ldc + n] += sum_k S[k][j] . dropout(X)[k][n]      j < s_cols <= 64, n < N
 * X [K][N] bf16 (ldx), S [K][lds] bf16 (lds 64 or 128; rows past the real tokens zero), K % 64 == 0,
 * N % 128 == 0, K * ldx * 2 < 2^31.  One stream over X: a workgroup per 128-column stripe and K range
 * (splits = K ranges per stripe, 1 .. K / 64), fp32 atomics.  drop_p > 0: X masked as ospo_lora_skinny
 * masked it in the forward (element index k * N + n, drop_keep): from keep_bits when non-NULL (the
 * forward's ospo_lora_skinny keep-bit output for this X, K * N / 8 bytes; rows it did not write may hold
 * anything when S is zero there), else by re-hashing. */
int ospo_lora_da(const void* X, int ldx, int N, const void* S, int lds, int s_cols, int K, float* C, int ldc,
                 int splits, uint32_t drop_seed, float drop_p, const void* keep_bits, hipStream_t stream);
int ospo_gemm_f32acc(const void* A, int lda, int a_kmajor, const void* B, int ldb, int b_kmajor,
                     int M, int N, int K, int k_splits, float alpha, float* C, int ldc,
                     int diag_nblk, int diag_r, hipStream_t stream);
/* As ospo_gemm_f32acc with LoRA dropout recomputed on a K-major B [K][N] (the dA product's
 * activations): element (m, n) enters as bf16(B[m][n] / (1 - p)) when drop_keep(m * N + n, seed) (the
 * 16-bit half (idx & 1) of drop_hash(idx >> 1, seed) is >= p * 2^16, common.h), else 0 -- the values ospo_lora_skinny's dropout multiplied in the forward, so the
 * forward need not store the masked copy.  Requires b_kmajor = 1 and 0 < p < 1.  keep_bits (optional):
 * the mask as ospo_lora_skinny's keep-bit output for B ([K][N / 8] bytes, N % 8 == 0), read instead of
 * re-hashed (same result). */
int ospo_gemm_f32acc_bdrop(const void* A, int lda, int a_kmajor, const void* B, int ldb, int b_kmajor,
                           int M, int N, int K, int k_splits, float alpha, float* C, int ldc,
                           int diag_nblk, int diag_r, uint32_t drop_seed, float drop_p, const void* keep_bits,
                           hipStream_t stream);

/* dst[i] (bf16) = round(scale * src[i]) for i < n (fp32 -> bf16 with scale). */
int ospo_f32_to_bf16(const float* src, void* dst, long n, float scale, hipStream_t stream);

/* -------------------------------------------------------------- RMSNorm ---
 * HF LlamaRMSNorm: y = w * bf16(x * rsqrt(mean(x^2) + eps)); rstd saved (fp32).
 * bwd: dx = dres + d/dx  (dres may be NULL); weight frozen (no dw).
 * Requires D % 8 == 0, D <= 16384. */
int ospo_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int M, int D, float eps,
                     hipStream_t stream);
int ospo_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                     const void* dres, void* dx, int M, int D, hipStream_t stream);

/* ----------------------------------------------------------------- RoPE ---
 * HF apply_rotary_pos_emb (rotate-half; position t = row % T) in place on the
 * q and k column blocks of a [rows, ld] buffer: x*cos + rotate_half(x)*sin with
 * each product and the sum rounded to bf16 as eager bf16 PyTorch does.
 * cos_tab/sin_tab: bf16 [T][head_dim/2] (HF LlamaRotaryEmbedding values, the
 * caller computes them once).  bwd applies the transpose rotation to grads. */
int ospo_rope_fwd(void* qkv, int ld, int q_col, int k_col, int S, int T, int n_heads,
                  int head_dim, const void* cos_tab, const void* sin_tab, hipStream_t stream);
int ospo_rope_bwd(void* dqkv, int ld, int q_col, int k_col, int S, int T, int n_heads,
                  int head_dim, const void* cos_tab, const void* sin_tab, hipStream_t stream);

/* --------------------------------------------------------------- SwiGLU ---
 * HF LlamaMLP: h = bf16(bf16(silu(g)) * u) with gu = [g | u] (cols [0,F), [F,2F)). */
int ospo_swiglu_fwd(const void* gu, int ld_gu, void* h, int ld_h, int M, int F, hipStream_t stream);
/* The fp8 variant's producers: as ospo_rmsnorm_fwd / _bwd, ospo_swiglu_fwd / _bwd, plus the MXFP8
 * copy of the bf16 output (q [M, ldq] e4m3, s = scales in ospo_quant_mx8's tile layout; K = D,
 * D, F, 2F; K % 128 == 0) -- byte-identical to ospo_quant_mx8 of the bf16 output, one HBM pass
 * less per GEMM operand. */
int ospo_rmsnorm_fwd_mx8(const void* x, const void* w, void* y, float* rstd, int M, int D, float eps, void* q,
                         int ldq, void* s, hipStream_t stream);
int ospo_rmsnorm_bwd_mx8(const void* dy, const void* x, const void* w, const float* rstd, const void* dres, void* dx,
                         int M, int D, void* q, int ldq, void* s, hipStream_t stream);
int ospo_swiglu_fwd_mx8(const void* gu, int ld_gu, void* h, int ld_h, int M, int F, void* q, int ldq, void* s,
                        hipStream_t stream);
int ospo_swiglu_bwd_mx8(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu, int M, int F,
                        void* q, int ldq, void* s, hipStream_t stream);
int ospo_swiglu_bwd(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu,
                    int M, int F, hipStream_t stream);

/* ------------------------------------------------------------ attention ---
 * Causal softmax attention per (sequence s, head h), HF eager semantics
 * (scores * scale, causal mask, fp32 softmax), flash-style on MFMA.
 * q/k/v/o rows s*T+t, head h at column offset h*head_dim.  lse: fp32
 * [S, H, T] (natural-log sum-exp of the scaled scores).  head_dim == 128.
 * bwd needs the workspace delta fp32 [S*H*T] and, for the 5-product form, ds_ws
 * (ospo_flash_attn_bwd_ws_bytes: bf16 dS^T per (sequence, head), written by the dK/dV
 * kernel and read by dQ = dS.K; NULL = the 7-product form that recomputes S and dP for
 * dQ).  No atomics.  dq/dk/dv are written (bf16) into dqkv.  With rope_cos/rope_sin (bf16 [T][head_dim/2], the
 * ospo_rope_* tables) the RoPE backward is applied to dq and dk before the store
 * (q/k in qkv are then the post-RoPE values); NULL for plain attention. */
int ospo_flash_attn_fwd(const void* qkv, int ld_qkv, int q_col, int k_col, int v_col, void* o,
                        int ld_o, float* lse, int S, int T, int n_heads, int head_dim, float scale,
                        hipStream_t stream);
size_t ospo_flash_attn_bwd_ws_bytes(int S, int T, int n_heads);
int ospo_flash_attn_bwd(const void* qkv, int ld_qkv, int q_col, int k_col, int v_col,
                        const void* o, int ld_o, const void* dout, int ld_do, const float* lse,
                        float* delta_ws, void* ds_ws, void* dqkv, int ld_dqkv, int S, int T,
                        int n_heads, int head_dim, float scale, const void* rope_cos,
                        const void* rope_sin, hipStream_t stream);
/* BASELINE config 5 (MXFP8 decoder Linears): the same kernels also write the MXFP8 copy of what they store,
 * byte-identical to ospo_quant_mx8 of the bf16 output, so the o_proj forward GEMM (operand: the attention
 * output, K8 = n_heads * head_dim) and the q|k|v dX GEMM (operand: dqkv, K8 = its column count) need no
 * quantize pass: q8 e4m3 [S*T, ldq8 bytes], s8 the scales of a [S*T, K8] matrix in ospo_quant_mx8's layout
 * (K8 % 128 == 0; every stored column < K8).  The backward form needs ds_ws (5-product kernels) and
 * q/k/v column offsets that are multiples of 128. */
int ospo_flash_attn_fwd_mx8(const void* qkv, int ld_qkv, int q_col, int k_col, int v_col, void* o, int ld_o,
                            float* lse, int S, int T, int n_heads, int head_dim, float scale, void* q8, int ldq8,
                            void* s8, int K8, hipStream_t stream);
int ospo_flash_attn_bwd_mx8(const void* qkv, int ld_qkv, int q_col, int k_col, int v_col, const void* o,
                            int ld_o, const void* dout, int ld_do, const float* lse, float* delta_ws, void* ds_ws,
                            void* dqkv, int ld_dqkv, int S, int T, int n_heads, int head_dim, float scale,
                            const void* rope_cos, const void* rope_sin, void* q8, int ldq8, void* s8, int K8,
                            hipStream_t stream);

/* ------------------------------------------------------- embed / gather ---
 * preprocess_batch (ospo/wrapper/train.py:224-239, 267-277) + concatenated_inputs
 * (:282-314): x0[s*T+t] = text_emb[text_ids[s % B][t]] for t < Lt (id < 0 -> zero
 * row, the right zero-padding), img_emb[s*N + t - Lt] for t >= Lt; S = 2B.
 * Indices are clamped to the table (vocab / img_vocab rows) so an invalid id
 * cannot fault; the host layer rejects them before launch.
 * gen_aligner_in: out[r] = bf16(gelu(bf16(gen_embed[ids[r]] . w1^T + b1)))
 * (modeling_vlm.py:263-264, first Linear + GELU of projector mlp_gelu). */
int ospo_assemble_inputs(const int* text_ids, int B, int Lt, const void* text_table, int vocab,
                         const void* img_emb, int N, int D, void* x0, hipStream_t stream);
int ospo_gen_aligner_in(const int* ids, int R, const void* gen_embed, int img_vocab, int E, const void* w1,
                        const void* b1, int D, void* out, hipStream_t stream);
/* dst[s*N + i] = src[s*T + t0 + i] (rows of D); scatter: dst rows zero elsewhere. */
int ospo_gather_rows(const void* src, int ld_src, int S, int T, int t0, int N, int D, void* dst,
                     hipStream_t stream);
int ospo_scatter_rows(const void* src, int S, int T, int t0, int N, int D, void* dst, int ld_dst,
                      int total_rows, hipStream_t stream);

/* Grouped row-vector sums (the logits/... metrics of get_batch_loss_metrics, ospo/wrapper/train.py:441-442,
 * without the [S, T, V] logits: sum_v logits = z . colsum(W2) + sum(b2)):
 *   out[g] = (accumulate ? out[g] : 0) + sum_{r < rows_per_group} x[g*rows_per_group + r] . w
 *            [+ add_scale * add[0] when add != NULL]
 * x bf16 rows of D (ldx elements apart), w fp32 [D]; D % 8 == 0.  fp32, deterministic order; ws >=
 * ospo_row_dot_sum_ws_bytes (the per-chunk partials).  Also colsum(W2) = W2^T rows . ones, and sum(b2). */
size_t ospo_row_dot_sum_ws_bytes(int n_groups, int rows_per_group, int D);
int ospo_row_dot_sum(const void* x, long ldx, int n_groups, int rows_per_group, int D, const float* w,
                     const float* add, float add_scale, int accumulate, float* out, void* ws, size_t ws_bytes,
                     hipStream_t stream);

/* y = bf16(gelu(x)); dx = bf16(dy * gelu'(x_pre)) -- gen_head GELU (modeling_vlm.py:49). */
int ospo_gelu_fwd(const void* x, void* y, long n, hipStream_t stream);
int ospo_gelu_bwd(const void* dy, const void* x_pre, void* dx, long n, hipStream_t stream);

/* ---------------------------------------------------------- log-probs ---
 * get_batch_logps (ospo/wrapper/train.py:375-396), average_log_prob=True, on
 * the R = S*N gathered image-token rows: logp[r] = logit[r, lab[r]] - lse[r]
 * (fp32 log-softmax of bf16 logits); seq_logps[s] = mean over its N rows.
 * bwd: dlogits[r, v] = g[r / N] / N * (1[v == lab[r]] - exp(logit - lse)). */
int ospo_logprob_fwd(const void* logits, int V, const int* labels, int R, int N, float* lse,
                     float* token_logp, float* seq_logps, hipStream_t stream);
int ospo_logprob_bwd(const void* logits, int V, const int* labels, const float* lse, int R, int N,
                     const float* g_seq, void* dlogits, hipStream_t stream);

/* ---------------------------------------------------------------- SimPO ---
 * simpo_loss (ospo/wrapper/train.py:317-342) + losses.mean() (:419).
 * logps = [chosen(B) | rejected(B)] fp32.  loss_type 0 = sigmoid, 1 = hinge.
 * fwd writes losses[B], loss_mean[1], rewards[2B] (= beta * logps).
 * bwd: glogps[2B] = d(g_loss * mean(losses)) / d logps. */
int ospo_simpo_fwd(const float* logps, int B, float beta, float gamma_beta_ratio,
                   float label_smoothing, int loss_type, float* losses, float* loss_mean,
                   float* rewards, hipStream_t stream);
int ospo_simpo_bwd(const float* logps, int B, float beta, float gamma_beta_ratio,
                   float label_smoothing, int loss_type, const float* g_loss, float* glogps,
                   hipStream_t stream);

/* ------------------------------------------------------------ LoRA pack ---
 * Build the per-layer fused LoRA operands from the flat bf16 LoRA parameter
 * buffer (layout in ospo_amd/lora.py): for module group g of layer l with
 * nmods modules of rank r, input dim Kin and per-module output Nmod:
 *   Acat [Rp][Kin]   rows j < nmods*r = stacked lora_A, rest zero
 *   AcatT[Kin][Rp]   its transpose
 *   Bcat [nmods*Nmod][Rp] block-diagonal stacked lora_B
 *   BT   [nmods*r][Nmod]  per-module lora_B^T (optional, may be NULL)
 * Rp = roundup(nmods*r, 64).  n_layers layers in one launch: A_flat/B_flat
 * advance by layer_stride elements per layer, the outputs are [n_layers][...]
 * contiguous. */
int ospo_lora_pack(const void* A_flat, const void* B_flat, int nmods, int r, int Kin, int Nmod,
                   int Rp, void* Acat, void* AcatT, void* Bcat, void* BT, int n_layers,
                   long layer_stride, hipStream_t stream);

/* Skinny LoRA products (peft lora.Linear, y += s B(A x)) -- bf16 out, no
 * atomics.  For n-tile j < n_tiles (columns 16j .. 16j+15):
 *   out[m][16j+c] = scale * sum_{k<K} A[m][(j / module_tiles) * a_koff + k] * Bt[16j+c][k]
 * (a_koff = 0: dense, every tile reduces the same K columns of A).  Bt rows
 * >= b_rows read as zero; rows M..M_out-1 and columns 16*n_tiles..out_cols-1
 * of out are written zero.  n_tiles <= 16, K % 32 == 0.
 *   u = s x A_cat^T : A = x [M, K], Bt = A_cat [Rp, K], a_koff = 0
 *   g = s dy B      : A = dy [M, nmods*Nmod], Bt = BT [nmods*r, Nmod],
 *                     K = a_koff = Nmod, module_tiles = r / 16
 * K is split across workgroups; ws (>= ospo_lora_skinny_ws_bytes(M_out, K,
 * n_tiles) bytes, 16-B aligned) holds, after a 4 KiB head of per-row-block
 * arrival counters, the fp32 partials; the last workgroup to arrive at a row
 * block sums them in order (deterministic) and resets its counter.  The first
 * 4 KiB of ws must be ZERO the first time it is used (hipMemset once at
 * allocation); every call leaves them zero again.  Calls sharing a ws must be
 * ordered (same stream).
 * drop_p > 0 (dense mode only): peft lora_dropout on A -- element (m, k) is kept
 * iff drop_keep(m*K + k, drop_seed) (common.h: the 16-bit half (idx & 1) of drop_hash(idx >> 1) is
 * >= drop_p * 2^16; drop_hash is a permutation of the 32-bit pair index for every seed) and becomes
 * bf16(A / (1 - drop_p)); the masked A is also written to xd [M, ld_xd] when xd
 * is non-NULL (the dA = g^T . dropout(x) operand of the backward).  keep_bits (non-NULL only with
 * drop_p > 0, lda % 8 == 0 and K % 64 == 0, xd NULL): the keep decision of every element of rows < M as
 * bits, row-major, 8 per byte -- byte (m*K + k) / 8, bit k % 8 -- which ospo_lora_da reads instead of
 * re-hashing (M*K/8 bytes). */
size_t ospo_lora_skinny_ws_bytes(int M_out, int K, int n_tiles);
int ospo_lora_skinny(const void* A, int lda, const void* Bt, int ldb, int b_rows, int M, int M_out,
                     int K, int n_tiles, int a_koff, int module_tiles, float scale, void* out, int ldo,
                     int out_cols, void* ws, size_t ws_bytes, unsigned drop_seed, float drop_p,
                     void* xd, int ld_xd, void* keep_bits, hipStream_t stream);

/* The MLP's SwiGLU forward fused with the down adapter's u product (HF LlamaMLP.forward's
 * down_proj(act_fn(gate) * up) with peft lora_A on its input; ospo/wrapper/train.py:352):
 *   h[m][k]   = bf16(bf16(silu(gu[m][k])) * gu[m][F + k])      (= ospo_swiglu_fwd, rows < M)
 *   out[m][c] = scale * sum_k dropout(h)[m][k] * Bt[c][k]      (= ospo_lora_skinny on h, dense, n_tiles <= 4)
 * in one stream over gu (h is written, never re-read).  F % 64 == 0; ws, out padding, dropout and keep_bits
 * as ospo_lora_skinny (K = F). */
int ospo_swiglu_fwd_lora_down(const void* gu, int ld_gu, void* h, int ld_h, int M, int M_out, int F,
                              const void* Bt, int ldb, int b_rows, int n_tiles, float scale, void* out, int ldo,
                              int out_cols, void* ws, size_t ws_bytes, unsigned drop_seed, float drop_p,
                              void* keep_bits, hipStream_t stream);

/* Fused LoRA backward over one stream of dy, LoRA rank 16 (replaces ospo_lora_skinny's g plus the
 * dB = dy^T u ospo_gemm_f32acc of the same group; ospo/wrapper/train.py:352 through peft lora.Linear's
 * backward):
 *   out[m][16 j + c] = scale * sum_k dy[m][j*Nmod + k] * Bt[16 j + c][k]   (m < M; rows M..M_out-1 and
 *                      columns 16*nmods..out_cols-1 written zero) -- g, bf16
 *   dB[j*Nmod + k][c] += sum_{m<M} dy[m][j*Nmod + k] * u[m][16 j + c]       -- fp32 atomic adds
 * dy [M, >= nmods*Nmod], Bt [nmods*16, Nmod] (ldb), u [M, >= 16*nmods].  Nmod % 128 == 0, nmods <= 4.
 * ws (>= ospo_lora_gdb_ws_bytes(M, nmods, Nmod) bytes, ZERO at allocation): a head of row-block counters
 * (used only by the ablation library's in-launch sum, left zero), then the fp32 partials of g, summed by a
 * second launch.  Calls sharing a ws must be ordered (same stream). */
size_t ospo_lora_gdb_ws_bytes(int M, int nmods, int Nmod);
int ospo_lora_gdb(const void* dy, int ldy, const void* Bt, int ldb, const void* u, int ldu, int M, int M_out,
                  int nmods, int Nmod, float scale, void* out, int ldo, int out_cols, float* dB, void* ws,
                  size_t ws_bytes, hipStream_t stream);
/* The same for LoRA rank r = 16 or 32 (round 6; configs/peft/lora.yaml ships r = 32): a module's r columns are
 * r / 16 halves of 16 over the same dy columns -- Bt [nmods*r, Nmod], u [M, >= r*nmods], g columns r*j + c,
 * dB [nmods*Nmod, r] -- and the workspace is ospo_lora_gdb_ws_bytes(M, nmods * r / 16, Nmod). */
int ospo_lora_gdb_r(const void* dy, int ldy, const void* Bt, int ldb, const void* u, int ldu, int M, int M_out,
                    int nmods, int Nmod, int r, float scale, void* out, int ldo, int out_cols, float* dB, void* ws,
                    size_t ws_bytes, hipStream_t stream);

/* The SwiGLU backward fused with the gate|up group's g / dB (LoRA rank 16; the backward of
 * down_proj(act_fn(gate) * up) and of gate|up's peft adapters, ospo/wrapper/train.py:352):
 *   dgu = [dgate | dup] = ospo_swiglu_bwd(dh, gu)           (rows < M, bf16, stored)
 *   out, dB             = ospo_lora_gdb(dgu, nmods = 2, Nmod = F, ...)
 * in one stream over (dh, gu): dgu is written once and not read back.  F % 128 == 0; Bt [32, F] (ldb),
 * u [M, >= 32]; out / ws / dB as ospo_lora_gdb with nmods = 2.  Same g bits as the two calls. */
int ospo_swiglu_lora_gdb(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu, const void* Bt,
                         int ldb, const void* u, int ldu, int M, int M_out, int F, float scale, void* out, int ldo,
                         int out_cols, float* dB, void* ws, size_t ws_bytes, hipStream_t stream);
/* rank r = 16 or 32 (round 6): Bt [2r, F], u [M, >= 2r], out / ws / dB as ospo_lora_gdb_r with nmods = 2. */
int ospo_swiglu_lora_gdb_r(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu, const void* Bt,
                           int ldb, const void* u, int ldu, int M, int M_out, int F, int r, float scale, void* out,
                           int ldo, int out_cols, float* dB, void* ws, size_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------------ MXFP8 variant ---
 * BASELINE config 5 / SURVEY §8f rank 1: the frozen Linears of the SimPO step
 * (q|k|v, o, gate|up, down; forward and dX backward -- the products that
 * ospo_gemm_nt_bf16 / _rope_ / _dropout_ run in bf16, reached from
 * ospo/wrapper/train.py:352 and PL's backward) with CDNA4 block-scaled fp8
 * MFMA (OCP MX: e4m3 elements, one E8M0 scale per 32 values along K).
 * ospo_quant_mx8: X bf16 [M, K] -> Q e4m3 [M, ldq bytes] + S (ospo_mx8_scale_bytes(M, K)
 * bytes, the tile layout documented in ospo_amd/csrc/mx8.hip).  K % 128 == 0.
 * ospo_gemm_nt_mx8: C = bf16(alpha * (deq(A8) . deq(B8)^T + A2 . B2^T) + bias) [+ residual],
 * A8/B8 from ospo_quant_mx8 (lda/ldb in bytes), the LoRA K-extension A2/B2 in bf16
 * (as ospo_gemm_nt_bf16).  rope_cols > 0: RoPE epilogue (as ospo_gemm_nt_rope_bf16);
 * drop_p > 0: masked extension (as ospo_gemm_nt_dropout_bf16).  N % 256 == 0. */
size_t ospo_mx8_scale_bytes(int M, int K);
int ospo_quant_mx8(const void* X, int ldx, int M, int K, void* Q, int ldq, void* S, hipStream_t stream);
int ospo_gemm_nt_mx8(const void* A8, int lda, const void* Asc, const void* B8, int ldb, const void* Bsc,
                     int M, int N, int K, const void* A2, int lda2, const void* B2, int ldb2, int K2,
                     float alpha, const void* bias, const void* residual, int ldr, void* C, int ldc,
                     const void* rope_cos, const void* rope_sin, int rope_T, int rope_cols,
                     unsigned drop_seed, float drop_p, int tail_split, void* ws, size_t ws_bytes,
                     hipStream_t stream);

/* ------------------------------------------------------ step-3 T2I decode ---
 * BASELINE config 4 / SURVEY §8f rank 2: the sampling loop of
 * ospo/wrapper/image_generation.py:132-171 (= ospo/inference.py:122-163) over a KV cache,
 * R = 2B rows (row 2b = prompt b, row 2b+1 its unconditional copy), captured once in a
 * hipGraph (ospo_amd/generate.py).  Step-dependent state is read from device counters
 * (pos_dev = position of the current query, step_dev = image-token index).
 * ospo_decode_gemv: out[r][n] = act(x[r] . W[n] + bias[n]) (+ residual[r][n]), R <= 64 rows,
 *   W [N, ldw] (nn.Linear layout), act = GELU(erf) when gelu; ws >= ospo_decode_gemv_ws_bytes.
 *   ldw = 0 (here and in the fused entries below): W is in the MFMA-tiled decode layout, 1-KiB tiles
 *   of 16 rows x 32 k at ((n/16) * (K/32) + k/32) * 512 elements, element 8 * (16 g + l16) + e =
 *   W[16 (n/16) + l16][32 (k/32) + 8 g + e] (ospo_amd.ops.tile_decode_weight); needs R <= 32 and
 *   N % 128 == 0 (OSPO_ERR_UNSUPPORTED otherwise); results bit-identical to the row-major W.
 * ospo_kv_store: q|k|v rows [R][nq] (position pos0 + i, pos0 = *pos_dev or 0): optional
 *   rotate-half RoPE on q and k, k / v into the caches [R][H][Tmax][head_dim], q to q_out.
 * ospo_attn_cache: causal attention of query (r, i) over cached keys [start[r], pos0 + i]
 *   (left padding as the reference's attention mask), HF eager bf16 rounding points.
 * ospo_cfg_sample: logits rows (2b, 2b+1) -> guided bf16 logits, bf16 softmax(l / T), inverse-CDF
 *   token with uniform u[step][b] -> tokens[b][step], next_ids[2b] = next_ids[2b+1].
 * ospo_embed_rows: out[i] = table[ids[i]] (get_input_embeddings for the prompt).
 * ospo_decode_advance: ++*pos_dev, ++*step_dev. */
size_t ospo_decode_gemv_ws_bytes(int R, int N, int K);
int ospo_decode_gemv(const void* W, int ldw, const void* X, int ldx, int R, int N, int K, const void* bias,
                     int gelu, const void* residual, int ldr, void* out, int ldo, void* ws, size_t ws_bytes,
                     hipStream_t stream);
int ospo_kv_store(void* qkv, int ld, int R, int nq, const int* pos_dev, int rope, const void* rope_cos,
                  const void* rope_sin, void* k_cache, void* v_cache, int n_heads, int head_dim, int Tmax,
                  void* q_out, int ld_q, hipStream_t stream);
int ospo_attn_cache(const void* q, int ldq, const void* k_cache, const void* v_cache, int R, int nq, int n_heads,
                    int head_dim, int Tmax, const int* start, const int* pos_dev, float scale, void* out, int ldo,
                    hipStream_t stream);
int ospo_cfg_sample(const void* logits, int ldl, int V, int B, float cfg_weight, float temperature, const float* u,
                    const int* step_dev, int n_steps, int* tokens, int* next_ids, float* probs_out,
                    hipStream_t stream);
int ospo_embed_rows(const int* ids, long n, const void* table, int vocab, int D, void* out, hipStream_t stream);
int ospo_decode_advance(int* pos_dev, int* step_dev, hipStream_t stream);
/* Decode-step fusions of the GEMV split sum with its consumer (bit-identical to the unfused
 * ospo_decode_gemv + consumer; need ospo_decode_gemv_fusable(R, N, K), else OSPO_ERR_UNSUPPORTED):
 * ospo_decode_gemv_kv: q|k|v = X . W^T (W [3 H 128, K]) then RoPE + KV-cache store as ospo_kv_store
 *   (one query per row at *pos_dev; q to q_out);
 * ospo_decode_gemv_swiglu: gate|up = X . W^T (W [2F, K]) then h = SwiGLU as ospo_swiglu_fwd. */
int ospo_decode_gemv_fusable(int R, int N, int K);
int ospo_decode_gemv_kv(const void* W, int ldw, const void* X, int ldx, int R, int n_heads, int head_dim, int K,
                        void* ws, size_t ws_bytes, const int* pos_dev, const void* rope_cos, const void* rope_sin,
                        void* k_cache, void* v_cache, int Tmax, void* q_out, int ldq, hipStream_t stream);
int ospo_decode_gemv_swiglu(const void* W, int ldw, const void* X, int ldx, int R, int F, int K, void* ws,
                            size_t ws_bytes, void* h, int ldh, hipStream_t stream);

/* One Linear of the decode step in ONE launch (round 3; image_generation.py:132-171 through HF
 * LlamaDecoderLayer): W tiled (ospo_decode_gemv with ldw = 0), R <= 32, N % 128 == 0, K % 32 == 0.
 *   input: X, or with ss_in the RMSNorm of X folded in: xn = bf16(ln_w * bf16(X * rsqrt(ss / K + eps)))
 *     as ospo_rmsnorm_fwd, ss[r] = sum over g < ss_groups of ss_in[g * 32 + r] (the row sums of squares
 *     a DL_PLAIN producer wrote, one per 128-column group, ss_groups <= 32; summed in group order);
 *   epi 0 (plain):  out[r][n] = act(X . W^T + bias) (+ residual) as ospo_decode_gemv; with ss_out also
 *     ss_out[n/128 * 32 + r] = sum over the group's 128 columns of out^2 (the next RMSNorm's input);
 *   epi 1 (kv):     N = 3 H 128: q (to out, ldo >= H 128) and the k / v cache rows at *pos_dev, RoPE as
 *     ospo_kv_store (== ospo_decode_gemv_kv);
 *   epi 2 (swiglu): W's 128-row group g = gate rows 64g .. 64g + 63, then up rows F + 64g .. (F = N / 2;
 *     ospo_amd.ops.interleave_gate_up); out[r][64g + c] = bf16(bf16(silu(gate)) * up) (== ospo_swiglu_fwd).
 * The K split is summed inside the launch (the last workgroup per 128-row group, in split order).
 * ws >= ospo_decode_linear_ws_bytes(R, N, K): a 4 KiB head of counters that must be ZERO the first time
 * it is used (every call leaves them zero), then the fp32 partials.  Calls sharing a ws are ordered. */
size_t ospo_decode_linear_ws_bytes(int R, int N, int K);
int ospo_decode_linear(const void* W, const void* X, int ldx, int R, int N, int K, const float* ss_in,
                       int ss_groups, const void* ln_w, float eps, int epi, const void* bias, int gelu,
                       const void* residual, int ldr, void* out, int ldo, float* ss_out, const int* pos_dev,
                       const void* rope_cos, const void* rope_sin, void* k_cache, void* v_cache, int n_heads,
                       int Tmax, void* ws, size_t ws_bytes, hipStream_t stream);
/* Head-range forms (round 5), for a decode step that runs the attention of heads h0 .. h0 + nh - 1 while the
 * projection of the other heads streams (two streams of one hipGraph):
 * ospo_decode_qkv_heads == ospo_decode_linear(epi 1) for heads h0 .. h0 + nh - 1 only, on W_hm = the q|k|v
 *   weight with its rows in head-major 128-row groups (q_h, k_h, v_h for h = 0 .. n_heads - 1; tiled as
 *   ospo_decode_gemv ldw = 0); the same bits per head as the full launch.  D = n_heads * 128.
 * ospo_attn_cache_heads == ospo_attn_cache for heads h0 .. h0 + nh - 1 (16-B aligned rows and caches). */
int ospo_decode_qkv_heads(const void* W_hm, const void* X, int ldx, int R, int D, const float* ss_in, int ss_groups,
                          const void* ln_w, float eps, void* q_out, int ldo, const int* pos_dev, const void* rope_cos,
                          const void* rope_sin, void* k_cache, void* v_cache, int n_heads, int h0, int nh, int Tmax,
                          void* ws, size_t ws_bytes, hipStream_t stream);
int ospo_attn_cache_heads(const void* q, int ldq, const void* k_cache, const void* v_cache, int R, int nq,
                          int n_heads, int h0, int nh, int Tmax, const int* start, const int* pos_dev, float scale,
                          void* out, int ldo, hipStream_t stream);
/* The decode MLP in ONE launch (round 5): ospo_decode_linear(xmid, W_gu, h, epi 2, norm = (ss_in, ln_w,
 * eps)) then ospo_decode_linear(h, W_down, out, epi 0, residual = xmid, ss_out), with the same outputs bit
 * for bit.  The down workgroups issue their first weights while the gate|up workgroups finish, then wait for
 * the h columns they read: flags (>= 2F / 128 words, ZERO the first time they are used with a given
 * (*step_dev, layer) pair -- a value is the epoch step * 64 + layer + 1 of the call that wrote it) and tmo
 * (set to nonzero if a wait gave up: the outputs are then invalid).  ws: ospo_decode_linear's workspace for
 * the down product (>= ospo_decode_linear_ws_bytes(R, D, F)).  OSPO_ERR_UNSUPPORTED when the shapes do not
 * map onto the one-launch form (the caller runs the two launches). */
int ospo_decode_mlp(const void* W_gu, const void* W_down, const void* xmid, int ldx, int R, int D, int F,
                    const float* ss_in, int ss_groups, const void* ln_w, float eps, void* h, int ldh, void* out,
                    int ldo, float* ss_out, const int* step_dev, int layer, unsigned* flags, unsigned* tmo,
                    void* ws, size_t ws_bytes, hipStream_t stream);

/* The decode layer's cached attention and o projection in ONE launch (round 5): ospo_attn_cache(q, ..., nq = 1,
 * attn_out) then ospo_decode_linear(attn_out, W_o, out, epi 0, residual, ss_out), with the same outputs bit for
 * bit.  The attention workgroups take a ticket per head when their rows are stored, the head's last one publishes
 * the head's flag -- flags: >= 2 * n_heads words (flags, then tickets), ZERO before the first call and never
 * touched by the caller between calls with distinct (*step_dev, layer) pairs (a flag's value: epoch step * 64 +
 * layer + 1; the tickets are left zero) -- and the o workgroups, their weights already in flight, wait for the
 * flags of their four heads; tmo is set nonzero if a wait gave up (outputs invalid).  W_o tiled as ospo_decode_gemv ldw = 0; ws: ospo_decode_linear's workspace for
 * (R, D, D).  OSPO_ERR_UNSUPPORTED (nothing launched) unless the o split plan is one 512-k chunk per split. */
int ospo_decode_attn_o(const void* q, int ldq, const void* k_cache, const void* v_cache, int R, int n_heads, int Tmax,
                       const int* start, const int* pos_dev, float scale, void* attn_out, int ld_attn, const void* W_o,
                       const void* residual, int ldr, void* out, int ldo, float* ss_out, const int* step_dev,
                       int layer, unsigned* flags, unsigned* tmo, void* ws, size_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------- VQ image tokenizer ---
 * janus/models/vq_model.py Encoder (:46-124) + quant_conv + VectorQuantizer
 * (:236-282) = gen_vision_model.encode, called per image at ospo/wrapper/train.py:246-264.  fp32
 * (the ids must be exact), NHWC activations, conv weights [Cout][KH][KW][Cin].
 * ospo_vq_conv2d: out = conv(x) + bias (+ residual); zero padding pad_t/pad_l on top/left and
 *   whatever (Ho, Wo, stride) reach past the bottom/right (Downsample's (0,1,0,1) pad).
 * ospo_vq_bmm_nt: out[b] = x[b] . w[b]^T ([n_rows, K] x [n_cols, K]), AttnBlock's q.k^T and p.v^T.
 * ospo_vq_groupnorm: GroupNorm(G, eps) over [B][HW][C] (+ swish), ws >= ospo_vq_groupnorm_ws_bytes.
 * ospo_vq_softmax_rows: in place, rows of softmax(x * scale).
 * ospo_vq_transpose: [B][R][C] -> [B][C][R].
 * ospo_vq_l2norm_rows: F.normalize(x, dim=-1) of [n][d].
 * ospo_vq_quantize: ids[v] = argmin_c |zn_v|^2 + |e_c|^2 - 2 zn_v.e_c (first index on ties),
 *   zn = F.normalize(z), e = the normalised codebook; dmin (optional) = the minimum. */
int ospo_vq_conv2d(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int KH, int KW,
                   int stride, int pad_t, int pad_l, int Ho, int Wo, const float* bias, const float* residual,
                   float* out, hipStream_t stream);
int ospo_vq_bmm_nt(const float* x, const float* w, int B, int n_rows, int n_cols, int K, float* out,
                   hipStream_t stream);
size_t ospo_vq_groupnorm_ws_bytes(int B, int G);
int ospo_vq_groupnorm(const float* x, int B, int HW, int C, int G, const float* gamma, const float* beta,
                      float eps, int swish, float* out, void* ws, size_t ws_bytes, hipStream_t stream);
int ospo_vq_softmax_rows(float* x, int rows, int cols, float scale, hipStream_t stream);
int ospo_vq_transpose(const float* x, int B, int R, int C, float* out, hipStream_t stream);
int ospo_vq_l2norm_rows(const float* x, long n, int d, float* out, hipStream_t stream);
int ospo_vq_quantize(const float* z, long n, int e_dim, const float* codebook_l2, int n_codes, int* ids,
                     float* dmin, hipStream_t stream);
/* Pixel decoder of step-3 sampling (image_generation.py:174-181: decode_code, vq_model.py:505-508):
 * ospo_vq_embed_codes: out[v][0..e) = codebook_l2[ids[v]] (get_codebook_entry :284-298, NHWC);
 * ospo_vq_conv2d_up2: ospo_vq_conv2d (stride 1, symmetric pad) of the nearest-neighbour 2x
 *   upsampling of x (Upsample :411-427), read on the fly: output [B][2H+2pad-KH+1][2W+2pad-KW+1][Cout];
 * ospo_vq_to_uint8: out[i] = (uint8) clip((x[i] + 1) / 2 * 255, 0, 255) (fp32, truncation). */
int ospo_vq_embed_codes(const int* ids, long n, const float* codebook_l2, int n_codes, int e_dim, float* out,
                        hipStream_t stream);
int ospo_vq_conv2d_up2(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int KH, int KW,
                       int pad, const float* bias, const float* residual, float* out, hipStream_t stream);
int ospo_vq_to_uint8(const float* x, long n, unsigned char* out, hipStream_t stream);

/* ------------------------------------------------------------ optimizer ---
 * compute_total_grad_norm (ospo/wrapper/train.py:459-469) + PL clip
 * (ospo/utils/train.py:30, gradient_clip_val) + torch AdamW
 * (train.py:108-115) on bf16 params with bf16 moments, fp32 grads.
 * sumsq_out[0] += sum(g^2), summed in an order that depends on n only (bit-identical
 * on every DP rank holding the same grads; caller zeroes); ws: device scratch of
 * 2048 floats.  adamw reads the device-resident sumsq, so no host sync is needed;
 * step is 1-based. */
int ospo_sumsq(const float* g, long n, float* sumsq_out, float* ws, hipStream_t stream);
int ospo_adamw_clip(void* params, const float* grads, void* exp_avg, void* exp_avg_sq, long n,
                    float lr, float beta1, float beta2, float eps, float weight_decay, int step,
                    const float* sumsq, float max_norm, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* OSPO_HIP_H */
