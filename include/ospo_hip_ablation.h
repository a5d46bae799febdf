/* A/B and ablation knobs of libospo_hip_ablation.so (make -C ospo_amd/csrc ablation), the
 * measurement build used by tools/ only.  The product library (libospo_hip.so) runs the default
 * schedules and exports none of these; some settings below give INVALID results by design
 * (they drop loads or MFMAs to decompose a kernel's time).  Process-global, not thread-safe. */
#ifndef OSPO_HIP_ABLATION_H
#define OSPO_HIP_ABLATION_H
#include "ospo_hip.h"
#ifdef __cplusplus
extern "C" {
#endif

/* NT GEMM schedule for N % 256 == 0: 0 = SP schedule + split-K tail (default); 1 = simple
 * double-buffered 256x256; 2 = simple 160x256; 3 = register-prefetch (v3); 4 = BK=32 LDS ring
 * (v4); 5 = 8-phase without the split tail; 14 = SP + split tail; 17 = 8-phase + split tail;
 * 18 = SP without s_setprio; 19 = SP with refills ahead of the reads; 20-23 = L2 row-group size
 * 2 / 8 / 16 / 4 of the default; 10-13, 15, 16 = decompositions (results INVALID: no loads /
 * no MFMA). */
int ospo_set_gemm_variant(int variant);
/* variant 29 (s_memtime stamps of one steady K-tile): 16 uint32 per wave, [grid][8 waves][16] */
int ospo_gemm_set_debug_buffer(void* buf);
/* LoRA skinny products: 1 = 16-row loop, 2 = 64-row LDS-shared, 3 = 2 with K splits of whole chunks (default). */
int ospo_set_skinny_variant(int v);
/* Decode GEMV schedule: 1 = skinny loop, 2 = LDS-shared activations, 3 = the same with 128 weight
 * rows per workgroup and power-of-two K splits (default). */
int ospo_set_gemv_variant(int v);
/* Force the K-split count of GEMV schedules 2 / 3 (0 = automatic). */
int ospo_set_gemv_splits(int s);
/* Pipelined dK/dV kernel phase stamps (s_memtime sums per wave: first LDS wait, S/dP + softmax
 * sub-phases, dV/dK sub-phases, vmcnt drain, barrier, tile count): 2 banks of 8 uint64 per wave,
 * [kb][S][H][waves][8]; nullptr turns them off. */
int ospo_attn_set_stamps(void* buf);
/* Environment (read once): OSPO_ATTN_WAVES=4 (64-row attention workgroups), OSPO_ATTN_DBG and
 * OSPO_ATTN_DKDV_DBG=1..5 (attention decompositions of the 8-wave round-2 dK/dV kernel, results
 * INVALID; set OSPO_ATTN_DKDV_WAVES=8 with them), OSPO_ATTN_DKDV_R2 (the unpipelined round-2 dK/dV
 * kernel), OSPO_ATTN_DKDV_WAVES=8 (8-wave dK/dV workgroups), OSPO_ATTN_DQ_2SLOT (the 2-slot dQ
 * kernel), OSPO_F32ACC_LEGACY (old tile rule of ospo_gemm_f32acc). */

#ifdef __cplusplus
}
#endif
#endif
