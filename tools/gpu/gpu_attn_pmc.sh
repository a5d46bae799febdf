# attention kernels on the step shape: DBG decomposition (ablation build) + PMC passes
# (one counter group per rocprofv3 pass; no trace domains with --pmc).
set -o pipefail
mkdir -p gpurun_out/attn_pmc
export TMPDIR=/tmp
for v in 0 4; do
  OSPO_ATTN_DKDV_DBG=$v timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attn_pmc/dbg$v.json 2>/dev/null || { echo "FAILED dbg $v"; exit 1; }
  echo "dbg=$v $(cat gpurun_out/attn_pmc/dbg$v.json)"
done
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/attn_pmc/p$i -o p -- python tools/attn_bench.py > gpurun_out/attn_pmc/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -5 gpurun_out/attn_pmc/p$i.log; exit 1; }
done
echo done
