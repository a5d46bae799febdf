# Round 4: counters of the w4 GEMM against the round-3 SP8 kernel (variant 27) and hipBLASLt on one shape:
# L2 hit / miss, fabric bytes, MFMA busy, clock (GRBM), LDS.  One counter group per rocprofv3 pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/w4pmc_${GO_TAG:-sq}
mkdir -p $OUT
export GO_ITERS=${GO_ITERS:-30}
for V in 0 27; do
  i=0
  for SET in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    GO_VARIANT=$V GO_BLAS=$([ $V = 0 ] && echo 1) timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $OUT/v${V}_$i -o p -- python tools/gemm_one.py > $OUT/v${V}_$i.log 2>&1 || { echo "pass v$V $i failed"; tail -3 $OUT/v${V}_$i.log; exit 1; }
  done
done
python tools/w4_pmc_summary.py $OUT
